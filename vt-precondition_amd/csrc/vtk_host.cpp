// vtk_host.cpp — host-side pieces of libvtkrylov.so that need no GPU: operator assembly on
// the host, the splitmix RHS (§8d), the row partition and halo plan of the
// multi-GPU path (§8e), and the CSR-stream tile planner used by the SpMV kernels.
#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "vtk_internal.hpp"
#include "vtk_vlasov.hpp"

namespace vtk {

static std::mutex g_err_mu;
static std::string g_err;

void set_context_free_error(const std::string &msg) {
    std::lock_guard<std::mutex> lk(g_err_mu);
    g_err = msg;
}

std::string context_free_error() {
    std::lock_guard<std::mutex> lk(g_err_mu);
    return g_err;
}

// Greedy CSR-stream row blocks: each tile takes whole align-groups while it stays within
// TILE_ROWS rows and TILE_NNZ nonzeros.  A group that alone exceeds TILE_NNZ is split into
// single-row tiles (rows over TILE_NNZ are then "long": the workgroup-wide reduction path).
void build_tiles(const std::vector<int32_t> &indptr, int align, std::vector<int32_t> &rows,
                 bool &has_long, bool &aligned) {
    const int64_t n = (int64_t)indptr.size() - 1;
    rows.assign(1, 0);
    has_long = false;
    aligned = true;
    int64_t r = 0;
    while (r < n) {
        const int64_t start = r;
        while (r < n) {
            const int64_t g = std::min<int64_t>(r + align, n);
            if (g - start > TILE_ROWS) break;
            if ((int64_t)indptr[g] - indptr[start] > TILE_NNZ) break;
            r = g;
        }
        if (r == start) {
            const int64_t g = std::min<int64_t>(start + align, n);
            if (g - start > 1) aligned = false;
            for (int64_t q = start; q < g; ++q) {
                rows.push_back((int32_t)(q + 1));
                if ((int64_t)indptr[q + 1] - indptr[q] > TILE_NNZ) has_long = true;
            }
            r = g;
        } else {
            rows.push_back((int32_t)r);
        }
    }
}

static bool valid_params(const vtk_vlasov_params *p) {
    if (!p) return false;
    if (p->dim == 1) return p->shape[0] >= 3;
    if (p->dim == 2) return p->shape[0] >= 3 && p->shape[1] >= 2;
    if (p->dim == 4) return p->shape[0] >= 3 && p->shape[1] >= 3 && p->shape[2] >= 2 && p->shape[3] >= 2;
    return false;
}

bool vlasov_params_ok(const vtk_vlasov_params *p) { return valid_params(p); }

}  // namespace vtk

using namespace vtk;

namespace vtk {
// parts of a line of L rows for the band step: the fewest equal parts of <= lp rows, each
// a multiple of 8 rows (whole BJ blocks); 0 when there is none
int band_parts(int64_t L, int lp) {
    for (int h = 1; h <= 32; ++h)
        if (L % h == 0 && (L / h) % 8 == 0 && L / h <= lp) return h;
    return 0;
}

}  // namespace vtk

extern "C" {

int vtk_abi_version(void) { return VTK_ABI_VERSION; }

const char *vtk_status_string(int s) {
    switch (s) {
        case VTK_OK: return "ok";
        case VTK_ERR_ARG: return "invalid argument";
        case VTK_ERR_HIP: return "HIP runtime error";
        case VTK_ERR_RCCL: return "RCCL error";
        case VTK_ERR_SINGULAR: return "singular diagonal block";
        case VTK_ERR_NOMEM: return "out of memory";
        case VTK_ERR_STATE: return "invalid state";
        case VTK_ERR_NODEVICE: return "no HIP device (no CPU fallback)";
        case VTK_ERR_PEER: return "a peer rank failed mid-solve";
        default: return "unknown status";
    }
}

int vtk_vlasov_size(const vtk_vlasov_params *p, int64_t *n, int64_t *nnz) {
    if (!valid_params(p) || !n || !nnz) {
        set_context_free_error("vtk_vlasov_size: invalid parameters");
        return VTK_ERR_ARG;
    }
    *n = vlasov_n(*p);
    *nnz = vlasov_nnz(*p);
    if (*nnz >= (int64_t)1 << 31) {
        set_context_free_error("vtk_vlasov_size: nnz does not fit int32 indices");
        return VTK_ERR_ARG;
    }
    return VTK_OK;
}

int vtk_vlasov_generate(const vtk_vlasov_params *p, int64_t r0, int64_t r1, int32_t *indptr,
                        int32_t *indices, void *data) {
    if (!valid_params(p) || r0 < 0 || r1 < r0 || r1 > vlasov_n(*p) || !indptr || !indices || !data) {
        set_context_free_error("vtk_vlasov_generate: invalid arguments");
        return VTK_ERR_ARG;
    }
    const int64_t nr = r1 - r0;
    indptr[0] = 0;
    for (int64_t i = 0; i < nr; ++i) indptr[i + 1] = indptr[i] + vlasov_row_count(*p, r0 + i);
    const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const int64_t nt = nr < 65536 ? 1 : (int64_t)hw;
    std::vector<std::thread> th;
    for (int64_t t = 0; t < nt; ++t) {
        th.emplace_back([=]() {
            const int64_t a = nr * t / nt, b = nr * (t + 1) / nt;
            VlasovRow row;
            for (int64_t i = a; i < b; ++i) {
                vlasov_row(*p, r0 + i, row);
                const int32_t o = indptr[i];
                for (int k = 0; k < row.count; ++k) {
                    indices[o + k] = (int32_t)row.col[k];
                    if (p->fp32) static_cast<float *>(data)[o + k] = (float)row.val[k];
                    else static_cast<double *>(data)[o + k] = row.val[k];
                }
            }
        });
    }
    for (auto &x : th) x.join();
    return VTK_OK;
}

int vtk_rhs_splitmix(uint64_t seed, int64_t r0, int64_t r1, double *b) {
    if (r1 < r0 || !b) {
        set_context_free_error("vtk_rhs_splitmix: invalid arguments");
        return VTK_ERR_ARG;
    }
    for (int64_t i = r0; i < r1; ++i) b[i - r0] = rhs_value(seed, i);
    return VTK_OK;
}

int vtk_partition_rows(int64_t n, const int32_t *indptr, int world, int align, int64_t *offsets) {
    if (n < 0 || world < 1 || align < 1 || !offsets) {
        set_context_free_error("vtk_partition_rows: invalid arguments");
        return VTK_ERR_ARG;
    }
    offsets[0] = 0;
    offsets[world] = n;
    const int64_t total = indptr ? (int64_t)indptr[n] : n;
    for (int q = 1; q < world; ++q) {
        const int64_t target = total * q / world;
        int64_t r;
        if (indptr) {
            r = std::lower_bound(indptr, indptr + n + 1, (int32_t)target) - indptr;
        } else {
            r = target;
        }
        r = (r + align / 2) / align * align;   // nearest multiple of align
        r = std::max(r, offsets[q - 1]);
        r = std::min(r, n);
        offsets[q] = r;
    }
    return VTK_OK;
}

int vtk_halo_plan(int64_t n_global, const int64_t *offsets, int world, int rank, int64_t nnz,
                  const int32_t *indices, int32_t *local_indices, int64_t *n_halo,
                  int64_t *halo_cols, int64_t *halo_count_per_rank) {
    if (!offsets || world < 1 || rank < 0 || rank >= world || nnz < 0 || (nnz > 0 && !indices) || !n_halo) {
        set_context_free_error("vtk_halo_plan: invalid arguments");
        return VTK_ERR_ARG;
    }
    const int64_t rb = offsets[rank], re = offsets[rank + 1], nl = re - rb;
    std::vector<int64_t> ext;
    for (int64_t k = 0; k < nnz; ++k) {
        const int64_t c = indices[k];
        if (c < 0 || c >= n_global) {
            set_context_free_error("vtk_halo_plan: column index out of range");
            return VTK_ERR_ARG;
        }
        if (c < rb || c >= re) ext.push_back(c);
    }
    std::sort(ext.begin(), ext.end());
    ext.erase(std::unique(ext.begin(), ext.end()), ext.end());
    *n_halo = (int64_t)ext.size();
    if (!halo_cols) return VTK_OK;
    std::memcpy(halo_cols, ext.data(), ext.size() * sizeof(int64_t));
    if (local_indices) {
        for (int64_t k = 0; k < nnz; ++k) {
            const int64_t c = indices[k];
            if (c >= rb && c < re) local_indices[k] = (int32_t)(c - rb);
            else local_indices[k] = (int32_t)(nl + (std::lower_bound(ext.begin(), ext.end(), c) - ext.begin()));
        }
    }
    if (halo_count_per_rank) {
        for (int q = 0; q < world; ++q) {
            halo_count_per_rank[q] = std::lower_bound(ext.begin(), ext.end(), offsets[q + 1]) -
                                     std::lower_bound(ext.begin(), ext.end(), offsets[q]);
        }
    }
    return VTK_OK;
}

int vtk_line_band_plan(int64_t n_local, int64_t line_len, int n_cu, vtk_band_geometry *out) {
    if (!out || line_len <= 0 || n_local <= 0 || n_local % line_len != 0) {
        set_context_free_error("vtk_line_band_plan: the slab must be a positive number of whole lines");
        return VTK_ERR_ARG;
    }
    const int64_t X = n_local / line_len;
    // the band kernels index rows, and columns of the two halo lines, in 32-bit integers
    if (X < 2 || n_local + 2 * line_len >= INT32_MAX / 2) {
        set_context_free_error("vtk_line_band_plan: fewer than 2 lines, or the slab exceeds 32-bit indices");
        return VTK_ERR_ARG;
    }
    const int H = vtk::band_parts(line_len);
    if (H < 1) {
        set_context_free_error("vtk_line_band_plan: no split of the line into equal parts of <= 400 rows, "
                               "each a multiple of 8");
        return VTK_ERR_ARG;
    }
    const int64_t ncu = n_cu > 0 ? n_cu : 256;
    // BAND_WPC workgroups per CU; >= 2 lines per range; the partial slots bound the grid
    const int64_t R = std::min<int64_t>({std::max<int64_t>(1, (int64_t)vtk::BAND_WPC * ncu / H), X / 2,
                                         (int64_t)vtk::GMAX / H});
    out->parts = H;
    out->wg_per_range = H;
    out->waves_per_wg = vtk::BAND_T / 64;
    out->ranges = (int)R;
    out->lines = X;
    return VTK_OK;
}

}  // extern "C"
