// vtk_api.cpp — C-ABI of libvtkrylov.so: contexts, RCCL communicator, CSR operator, block-Jacobi
// preconditioner and the restarted GMRES driver (host orchestration of the gfx950 kernels).
//
// The driver restates scipy.sparse.linalg.gmres (scipy/sparse/linalg/_isolve/iterative.py:
// 692-841) with every vector operation and every reduction on the device; the host only keeps
// SciPy's outer-loop bookkeeping (ptol_max_factor, :816-838) and reads back one 100-byte state
// record per restart cycle.  Inside a cycle the Givens rotations, the inner stop test
// (presid <= ptol, :794) and the breakdown test (:766) run on the device: kernels of columns
// after the stop column return at entry (GmresState::stop_col), so the host enqueues a cycle
// without a per-step round trip and throttles itself with events LOOKAHEAD columns behind.
#include <algorithm>
#include <cctype>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "vtk_internal.hpp"
#include "vtk_vlasov.hpp"

namespace vtk {
std::string context_free_error();
bool vlasov_params_ok(const vtk_vlasov_params *p);
}  // namespace vtk

using namespace vtk;

namespace {

constexpr int LOOKAHEAD = 3;   // columns the host may run ahead of the device

int fail(vtk_ctx *c, int code, const std::string &msg) {
    if (c) c->err = msg;
    else set_context_free_error(msg);
    return code;
}

#define HIPCHK(c, x)                                                                         \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess)                                                                \
            return fail((c), e_ == hipErrorOutOfMemory ? VTK_ERR_NOMEM : VTK_ERR_HIP,        \
                        std::string(#x) + ": " + hipGetErrorString(e_));                     \
    } while (0)

#define NCCLCHK(c, x)                                                                        \
    do {                                                                                     \
        ncclResult_t r_ = (x);                                                               \
        if (r_ != ncclSuccess) {                                                             \
            if (c) (c)->comm_broken = true;                                                  \
            return fail((c), VTK_ERR_RCCL, std::string(#x) + ": " + ncclGetErrorString(r_)); \
        }                                                                                    \
    } while (0)

#define TRY(x)                          \
    do {                                \
        int rc_ = (x);                  \
        if (rc_ != VTK_OK) return rc_;  \
    } while (0)

// device buffer owned by a scope
struct DBuf {
    void *p = nullptr;
    ~DBuf() { if (p) (void)hipFree(p); }
    template <typename T> T *as() const { return static_cast<T *>(p); }
};

int dalloc(vtk_ctx *c, DBuf &b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    HIPCHK(c, hipMalloc(&b.p, bytes));
    return VTK_OK;
}

int64_t round_up(int64_t a, int64_t m) { return (a + m - 1) / m * m; }

// ---- tuning switches (vtk::Tuning): name, member; VTK_<NAME upper> seeds them at creation ----
struct TuneKey { const char *name; int Tuning::*mem; };
constexpr TuneKey TUNE_KEYS[] = {
    {"band", &Tuning::band}, {"band_lsv", &Tuning::band_lsv}, {"sell_canon", &Tuning::sell_canon},
    {"band_canon", &Tuning::band_canon}, {"band_opt", &Tuning::band_opt}, {"band_long_rows", &Tuning::band_long_rows},
    {"lsv_ring", &Tuning::lsv_ring},
    {"prof_perj", &Tuning::prof_perj}, {"comm_solo", &Tuning::comm_solo}, {"auto_band", &Tuning::auto_band},
    {"grid4", &Tuning::grid4}, {"c4_fused", &Tuning::c4_fused}, {"g4_ring", &Tuning::g4_ring},
    {"g4_gr", &Tuning::g4_gr}, {"g4_fast", &Tuning::g4_fast}, {"line_fuse", &Tuning::line_fuse}, {"cyc_ring", &Tuning::cyc_ring},
    {"fail_step", &Tuning::fail_step},
};
// switches of earlier rounds whose alternative lost its A/B: an environment that
// still sets one is told once that it no longer has an effect
constexpr const char *RETIRED_KEYS[] = {"band_canon_sl", "sell_pad", "sell_grid", "plain_grid", "sell_swz", "plain_var",
                                        "band_j3", "lsv_spmv_cap", "line_sweep", "ev_every", "debug_band", "g4_pd",
                                        "g4_xcd", "g4_dc", "g4_dc0", "g4_res", "upd_grid", "upd_xb", "sell_nopad",
                                        "sell_lsv"};

const TuneKey *tune_key(const char *name) {
    if (!name) return nullptr;
    for (const auto &k : TUNE_KEYS)
        if (std::strcmp(k.name, name) == 0) return &k;
    return nullptr;
}

std::string env_name(const char *key) {
    std::string var = "VTK_";
    for (const char *p = key; *p; ++p) var += (char)std::toupper((unsigned char)*p);
    return var;
}

void tune_from_env(Tuning &t) {
    for (const auto &k : TUNE_KEYS)
        if (const char *e = std::getenv(env_name(k.name).c_str()); e && *e) t.*k.mem = std::atoi(e);
    // (a renamed or removed switch must not be silently ignored)
    static bool warned = false;   // once per process, every retired variable that is set
    for (const char *k : RETIRED_KEYS) {
        const std::string var = env_name(k);
        if (!warned && std::getenv(var.c_str()))
            std::fprintf(stderr, "vtkrylov: %s is set but no longer has an effect (retired tuning switch, DESIGN.md §3f)\n",
                         var.c_str());
    }
    warned = true;
}

// ---- kernel profile: HIP events around each launch on the context stream ------------------
hipEvent_t prof_event(vtk_ctx *c) {
    if (!c->prof_pool.empty()) { hipEvent_t e = c->prof_pool.back(); c->prof_pool.pop_back(); return e; }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

int prof_class(vtk_ctx *c, const char *name) {
    for (size_t i = 0; i < c->prof_acc.size(); ++i) if (c->prof_acc[i].name == name) return (int)i;
    c->prof_acc.push_back(vtk_ctx::ProfAcc{name});
    return (int)c->prof_acc.size() - 1;
}

// brackets one launch: start event at construction, stop event at scope exit
struct Prof {
    vtk_ctx *c;
    size_t idx = (size_t)-1;
    Prof(vtk_ctx *c_, const char *name, int col, double bytes) : c(c_) {
        if (!c->prof_on) return;
        vtk_ctx::ProfPending p{prof_class(c, name), col, bytes, prof_event(c), prof_event(c)};
        (void)hipEventRecord(p.e0, c->stream);
        c->prof_pending.push_back(p);
        idx = c->prof_pending.size() - 1;
    }
    ~Prof() { if (idx != (size_t)-1) (void)hipEventRecord(c->prof_pending[idx].e1, c->stream); }
};

// fold pending launches into the per-class counters; launches of columns after the cycle's
// stop column (no-op kernels) are dropped
void prof_flush(vtk_ctx *c, int last_col = 1 << 30) {
    if (c->prof_pending.empty()) return;
    (void)hipStreamSynchronize(c->stream);
    for (auto &p : c->prof_pending) {
        if (p.col <= last_col) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, p.e0, p.e1) == hipSuccess) {
                auto &a = c->prof_acc[p.cls];
                a.launches += 1;
                a.seconds += ms * 1e-3;
                a.bytes += p.bytes;
            }
        }
        c->prof_pool.push_back(p.e0);
        c->prof_pool.push_back(p.e1);
    }
    c->prof_pending.clear();
}

// the BJ operator the kernels apply (vtk_bj_mode): tridiagonal factors when available and not
// switched off, else the inverse rows; null M: identity
BjOp bj_op(const vtk_prec *M) {
    BjOp o;
    if (!M) return o;
    if (M->kind == VTK_PREC_LINE) {
        o.line = &M->line;
        return o;
    }
    o.inv = M->d_inv;
    o.bs = M->bs;
    if (M->tri_ok && M->mode != VTK_BJ_INVERSE) {
        o.tri = M->d_tri;
        o.tri_ld = M->tri_ld;
    }
    return o;
}

// profile class of a standalone preconditioner apply
const char *prec_cls(const vtk_prec *M) { return M && M->kind == VTK_PREC_LINE ? "line_apply" : "bj_apply"; }

// algorithmic bytes per row of one BJ application (tridiagonal: the SELL kernels read only m)
double bj_row_bytes(const vtk_prec *M) {
    if (!M) return 0.0;
    if (M->kind == VTK_PREC_LINE) return M->line.compact ? 8.0 : 24.0;   // m (compact) or l, m, g
    if (bj_op(M).tri) return M->A->use_sell ? 8.0 : 24.0;
    return 8.0 * M->bs;
}

// reducing-kernel grid: a function of the local size on one GPU; GMAX on every rank when
// world > 1 (equal partial-vector lengths for the in-place all-reduce)
int grid_for(vtk_ctx *c, int g) { return c->dist ? GMAX : g; }

int upload_tiles(vtk_ctx *c, const std::vector<int32_t> &indptr, int align, Tiles &t,
                 std::vector<int32_t> *rows_out = nullptr) {
    std::vector<int32_t> rows;
    build_tiles(indptr, align, rows, t.has_long, t.aligned);
    if (rows_out) *rows_out = rows;
    t.ntiles = (int)rows.size() - 1;
    t.align = align;
    t.grid = grid_for(c, std::max(1, std::min(t.ntiles, GMAX)));
    if (t.d_row) (void)hipFree(t.d_row);
    t.d_row = nullptr;
    HIPCHK(c, hipMalloc(&t.d_row, rows.size() * sizeof(int32_t)));
    HIPCHK(c, hipMemcpy(t.d_row, rows.data(), rows.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    return VTK_OK;
}

void free_tiles(Tiles &t) {
    (void)hipFree(t.d_row);
    (void)hipFree(t.d_end);
    t.d_row = t.d_end = nullptr;
}

// Split the tiles of `all` (host row boundaries `rows`) into interior tiles (no row reads a halo
// column) and boundary tiles, as [start, end) lists.  Grids: boundary <= 64 workgroups,
// interior the rest of GMAX, so both launches' partials fit one GMAX-strided slot row.
int upload_split_tiles(vtk_ctx *c, const std::vector<int32_t> &rows, const std::vector<uint8_t> &row_halo,
                       const Tiles &all, Tiles &in, Tiles &bd) {
    std::vector<int32_t> is, ie, bs_, be;
    for (size_t t = 0; t + 1 < rows.size(); ++t) {
        bool h = false;
        for (int32_t r = rows[t]; r < rows[t + 1] && !h; ++r) h = row_halo[(size_t)r] != 0;
        (h ? bs_ : is).push_back(rows[t]);
        (h ? be : ie).push_back(rows[t + 1]);
    }
    auto up = [&](const std::vector<int32_t> &st, const std::vector<int32_t> &en, Tiles &t, int gmax) -> int {
        free_tiles(t);
        t.ntiles = (int)st.size();
        t.align = all.align;
        t.has_long = all.has_long;
        t.aligned = all.aligned;
        t.grid = std::max(1, std::min(t.ntiles, gmax));
        t.nrows = 0;
        for (size_t k = 0; k < st.size(); ++k) t.nrows += en[k] - st[k];
        const size_t nb = std::max<size_t>(st.size(), 1) * sizeof(int32_t);
        HIPCHK(c, hipMalloc(&t.d_row, nb));
        HIPCHK(c, hipMalloc(&t.d_end, nb));
        if (!st.empty()) {
            HIPCHK(c, hipMemcpy(t.d_row, st.data(), st.size() * sizeof(int32_t), hipMemcpyHostToDevice));
            HIPCHK(c, hipMemcpy(t.d_end, en.data(), en.size() * sizeof(int32_t), hipMemcpyHostToDevice));
        }
        return VTK_OK;
    };
    TRY(up(bs_, be, bd, 64));
    TRY(up(is, ie, in, GMAX - bd.grid));
    return VTK_OK;
}

// ---- communicator primitives: RCCL on the context stream, or host-staged hooks ------------

// in-place sum over ranks of `count` doubles in device memory
int comm_allreduce(vtk_ctx *c, double *d, int64_t count) {
    if (c->host_comm) {
        std::vector<double> h((size_t)count);
        HIPCHK(c, hipMemcpyAsync(h.data(), d, count * sizeof(double), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (c->hops.allreduce_sum_f64(c->hops.user, h.data(), count) != 0) return fail(c, VTK_ERR_STATE, "host allreduce hook failed");
        HIPCHK(c, hipMemcpyAsync(d, h.data(), count * sizeof(double), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        return VTK_OK;
    }
    NCCLCHK(c, ncclAllReduce(d, d, (size_t)count, ncclDouble, ncclSum, c->comm, c->stream));
    return VTK_OK;
}

// point-to-point exchange: to rank q scnt[q] elements from send+soff[q], from rank q rcnt[q]
// elements into recv+roff[q] (ncclSend/ncclRecv in one group: xGMI is point-to-point)
int comm_alltoallv(vtk_ctx *c, const void *send, const std::vector<int64_t> &scnt, const std::vector<int64_t> &soff,
                   void *recv, const std::vector<int64_t> &rcnt, const std::vector<int64_t> &roff, ncclDataType_t dt, size_t eb,
                   hipStream_t st = nullptr) {
    const int W = c->world;
    if (!st) st = c->stream;
    if (c->host_comm) {
        const int64_t ns = W ? soff[W - 1] + scnt[W - 1] : 0, nr = W ? roff[W - 1] + rcnt[W - 1] : 0;
        std::vector<char> hs((size_t)std::max<int64_t>(ns, 1) * eb), hr((size_t)std::max<int64_t>(nr, 1) * eb);
        if (ns) HIPCHK(c, hipMemcpyAsync(hs.data(), send, ns * eb, hipMemcpyDeviceToHost, st));
        HIPCHK(c, hipStreamSynchronize(st));
        if (c->hops.alltoallv(c->hops.user, hs.data(), scnt.data(), soff.data(), hr.data(), rcnt.data(), roff.data(), (int64_t)eb) != 0)
            return fail(c, VTK_ERR_STATE, "host alltoallv hook failed");
        if (nr) HIPCHK(c, hipMemcpyAsync(recv, hr.data(), nr * eb, hipMemcpyHostToDevice, st));
        HIPCHK(c, hipStreamSynchronize(st));
        return VTK_OK;
    }
    NCCLCHK(c, ncclGroupStart());
    for (int q = 0; q < W; ++q) {
        if (scnt[q] > 0) NCCLCHK(c, ncclSend((const char *)send + soff[q] * eb, (size_t)scnt[q], dt, q, c->comm, st));
        if (rcnt[q] > 0) NCCLCHK(c, ncclRecv((char *)recv + roff[q] * eb, (size_t)rcnt[q], dt, q, c->comm, st));
    }
    NCCLCHK(c, ncclGroupEnd());
    return VTK_OK;
}

// every rank contributes `count` int64 (device), receives world*count (device)
int comm_allgather_i64(vtk_ctx *c, const int64_t *send, int64_t *recv, int64_t count) {
    if (c->host_comm) {
        std::vector<int64_t> hs((size_t)count), hr((size_t)count * c->world);
        HIPCHK(c, hipMemcpyAsync(hs.data(), send, count * 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (c->hops.allgather(c->hops.user, hs.data(), hr.data(), count * 8) != 0) return fail(c, VTK_ERR_STATE, "host allgather hook failed");
        HIPCHK(c, hipMemcpyAsync(recv, hr.data(), hr.size() * 8, hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        return VTK_OK;
    }
    NCCLCHK(c, ncclAllGather(send, recv, (size_t)count, ncclInt64, c->comm, c->stream));
    return VTK_OK;
}

// partial sums -> consumer view.  Across ranks every reducing kernel runs on exactly GMAX
// workgroups (grid_for), so the partial vectors have the same length on every rank and are
// all-reduced in place: consumers then sum them exactly as on one GPU, with no extra kernel.
Red reduce(vtk_ctx *c, double *part, int cnt, int &rc) {
    rc = VTK_OK;
    if (c->dist) {
        Prof pf(c, "allreduce", -1, 8.0 * cnt);
        rc = comm_allreduce(c, part, cnt);
    }
    return Red{part, cnt};
}

// across ranks the all-reduced partial vectors must have one length on every rank: a reducing
// launch whose grid follows the slab (the 4D and x-line rings) zero-pads its partials to GMAX, as
// every other reducing launch runs GMAX workgroups there (grid_for)
int pad_partials(vtk_ctx *c, double *p0, double *p1, int &g) {
    if (!c->dist || g >= GMAX) return VTK_OK;
    for (double *p : {p0, p1})
        if (p) HIPCHK(c, hipMemsetAsync(p + g, 0, (size_t)(GMAX - g) * sizeof(double), c->stream));
    g = GMAX;
    return VTK_OK;
}

int halo_exchange(vtk_csr *A, const double *x) {
    vtk_ctx *c = A->ctx;
    // no peer of this rank: RCCL point-to-point needs no call; the host-staged alltoallv is a
    // collective every rank joins (with zero counts)
    if (!c->dist || (!c->host_comm && A->n_send == 0 && A->n_halo == 0)) return VTK_OK;
    Prof pf(c, "halo", -1, 16.0 * A->n_send + 8.0 * A->n_halo);
    HIPCHK(c, launch_gather(x, A->d_send_idx, A->n_send, A->d_send_buf, c->stream));
    return comm_alltoallv(c, A->d_send_buf, A->send_cnt, A->send_off, A->d_halo, A->recv_cnt, A->recv_off, ncclDouble, sizeof(double));
}

// the same exchange overlapped: pack and send/recv both on the comm stream once x is final on
// the main stream (ev_pack); the interior tiles start at once, ev_halo marks the halo's arrival
// (the boundary tiles wait on it)
int halo_exchange_async(vtk_csr *A, const double *x) {
    vtk_ctx *c = A->ctx;
    HIPCHK(c, hipEventRecord(c->ev_pack, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->comm_stream, c->ev_pack, 0));
    HIPCHK(c, launch_gather(x, A->d_send_idx, A->n_send, A->d_send_buf, c->comm_stream));
    TRY(comm_alltoallv(c, A->d_send_buf, A->send_cnt, A->send_off, A->d_halo, A->recv_cnt, A->recv_off, ncclDouble,
                       sizeof(double), c->comm_stream));
    HIPCHK(c, hipEventRecord(c->ev_halo, c->comm_stream));
    return VTK_OK;
}

SpmvIn spmv_in(vtk_csr *A, const Tiles *t, const double *x, const Groups *g = nullptr) {
    SpmvIn in{A->d_indptr, A->d_indices, A->d_data, A->fp32, t, (int)A->n_local, x,
              A->ctx->dist ? A->d_halo : nullptr};
    if (A->use_sell) {   // SELL-64 layout: the tiles are not used
        in.sell = &A->sell;
        in.groups = g ? g : &A->g_all;
    }
    in.plain_grid = 2048;   // (grid sweep, C3: 2048 best; 3072: 293 us; 4096-100 000: 256-265)
    // the plain SpMV walks its groups in XCD-contiguous order (C3 PMC fetch 1.40 -> 1.07 GB per
    // launch, time neutral) -- except on the 9-wide 4D rows (648 -> 730 us swizzled: their x +- 1
    // planes are 250 000 rows away, not in the XCD's window); the reducing launches keep
    // blockIdx order, so their partial sums keep their bits
    in.swz = (A->use_sell && A->sell.uniform_w > 8) ? 0 : 1;
    in.plain_var = 1;   // padding gathers branched in the plain SpMV (243.6 -> 221.3 us)
    return in;
}

// the fused SpMV + BJ kernels apply: SELL chunks align with any power-of-two bs <= 32; the
// CSR-stream path needs the BJ tiles aligned and free of long rows
bool bj_fused(const vtk_prec *M) {
    if (!M || M->kind != VTK_PREC_BJACOBI) return false;
    if (M->A->use_sell) return (M->bs & (M->bs - 1)) == 0 && M->bs <= 32;
    return M->fused;
}

// the solver's SELL launches read the line-separable tables when the operator
// has them: the same values, the same sums, 8 B of values per row instead of 40 (tuning band_lsv
// 0: the SELL values).  vtk_spmv keeps the SELL values: it is the measured SpMV
bool lsv_on(const vtk_csr *A) {
    return A->use_sell && A->d_lsv && A->band_L > 0 && !A->fp32 && A->ctx->tune.band_lsv &&
           (!A->ctx->dist || A->band_ghost);
}
SpmvIn lsv_in(SpmvIn in, const vtk_csr *A) {
    if (in.sell && A->d_g4tab && A->ctx->tune.grid4) in.g4 = A->g4;   // 4D grid rows (Grid4)
    if (in.sell && lsv_on(A)) {
        in.lsv = A->d_lsv;
        in.lsv_L = (int)A->band_L;
        in.lsv_lblk = A->band_ghost ? A->band_lblk : -1;
        in.lsv_xord = A->band_ghost ? A->band_xord : 0;
        // tuning sell_canon 0 (A/B): the SELL codes even for canonical rows
        in.lsv_canon = A->lsv_canon && A->ctx->tune.sell_canon ? 1 : 0;
    }
    return in;
}
double matrix_bytes(const vtk_csr *A);
// matrix bytes a solver SELL launch reads (lsv_in)
double solver_matrix_bytes(const vtk_csr *A) {
    const double b = matrix_bytes(A);
    if (A->use_sell && A->d_g4tab && A->ctx->tune.grid4) return (A->fp32 ? 4.0 : 8.0) * (double)A->n_local;   // D only
    if (!lsv_on(A)) return b;
    if (A->lsv_canon && A->ctx->tune.sell_canon) return 8.0 * (double)A->n_local;   // the diagonal only
    return b - 8.0 * (double)A->sell.entries + 8.0 * (double)A->n_local;
}

// interior / boundary pieces of the fused SpMV (world > 1)
bool bj_split(const vtk_prec *M) { return M && (M->A->use_sell ? M->A->g_in.grid > 0 : M->split); }
SpmvIn split_in(vtk_csr *A, vtk_prec *M, const double *x, bool interior) {
    return lsv_in(interior ? spmv_in(A, &M->tiles_in, x, &A->g_in) : spmv_in(A, &M->tiles_bd, x, &A->g_bd), A);
}

// Build the halo plan of a freshly uploaded CSR (indices still GLOBAL on the device), remap
// the device indices to local numbering and exchange the send lists over RCCL.
int setup_halo(vtk_csr *A) {
    vtk_ctx *c = A->ctx;
    const int W = c->world;
    // the indices may still be in flight on the context's (non-blocking) stream (device
    // assembly): hipMemcpy on the null stream does not wait for it
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::vector<int32_t> idx((size_t)A->nnz);
    if (A->nnz) HIPCHK(c, hipMemcpy(idx.data(), A->d_indices, A->nnz * sizeof(int32_t), hipMemcpyDeviceToHost));
    int64_t nh = 0;
    if (vtk_halo_plan(A->n_global, A->offsets.data(), W, c->rank, A->nnz, idx.data(), nullptr, &nh,
                      nullptr, nullptr) != VTK_OK)
        return fail(c, VTK_ERR_ARG, context_free_error());
    A->halo_cols.resize((size_t)nh);
    A->recv_cnt.assign(W, 0);
    if (vtk_halo_plan(A->n_global, A->offsets.data(), W, c->rank, A->nnz, idx.data(), nullptr, &nh,
                      A->halo_cols.data(), A->recv_cnt.data()) != VTK_OK)
        return fail(c, VTK_ERR_ARG, context_free_error());
    A->n_halo = nh;
    A->row_halo.assign((size_t)A->n_local, 0);
    for (int64_t r = 0; r < A->n_local; ++r)
        for (int32_t k = A->h_indptr[r]; k < A->h_indptr[r + 1]; ++k)
            if (idx[k] < A->row_begin || idx[k] >= A->row_end) { A->row_halo[(size_t)r] = 1; break; }
    A->recv_off.assign(W, 0);
    for (int q = 1; q < W; ++q) A->recv_off[q] = A->recv_off[q - 1] + A->recv_cnt[q - 1];
    // remap indices on the device
    DBuf dh;
    TRY(dalloc(c, dh, (size_t)nh * sizeof(int64_t)));
    if (nh) HIPCHK(c, hipMemcpy(dh.p, A->halo_cols.data(), nh * sizeof(int64_t), hipMemcpyHostToDevice));
    HIPCHK(c, launch_remap_cols(A->d_indices, A->nnz, A->row_begin, A->n_local, dh.as<int64_t>(), nh, c->stream));
    // counts matrix: everyone learns what it must send
    DBuf dcnt, dall;
    TRY(dalloc(c, dcnt, W * sizeof(int64_t)));
    TRY(dalloc(c, dall, (size_t)W * W * sizeof(int64_t)));
    HIPCHK(c, hipMemcpyAsync(dcnt.p, A->recv_cnt.data(), W * sizeof(int64_t), hipMemcpyHostToDevice, c->stream));
    TRY(comm_allgather_i64(c, dcnt.as<int64_t>(), dall.as<int64_t>(), W));
    std::vector<int64_t> all((size_t)W * W);
    HIPCHK(c, hipMemcpyAsync(all.data(), dall.p, all.size() * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    A->send_cnt.assign(W, 0);
    A->send_off.assign(W, 0);
    for (int q = 0; q < W; ++q) A->send_cnt[q] = all[(size_t)q * W + c->rank];
    for (int q = 1; q < W; ++q) A->send_off[q] = A->send_off[q - 1] + A->send_cnt[q - 1];
    A->n_send = W ? A->send_off[W - 1] + A->send_cnt[W - 1] : 0;
    // exchange the requested global ids
    DBuf dreq, dsend;
    TRY(dalloc(c, dreq, (size_t)nh * sizeof(int64_t)));
    TRY(dalloc(c, dsend, (size_t)A->n_send * sizeof(int64_t)));
    if (nh) HIPCHK(c, hipMemcpyAsync(dreq.p, A->halo_cols.data(), nh * sizeof(int64_t), hipMemcpyHostToDevice, c->stream));
    // requests travel opposite to the data: send my recv list to each owner
    TRY(comm_alltoallv(c, dreq.p, A->recv_cnt, A->recv_off, dsend.p, A->send_cnt, A->send_off, ncclInt64, sizeof(int64_t)));
    std::vector<int64_t> sg((size_t)A->n_send);
    if (A->n_send) HIPCHK(c, hipMemcpyAsync(sg.data(), dsend.p, A->n_send * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::vector<int32_t> sl((size_t)A->n_send);
    for (int64_t k = 0; k < A->n_send; ++k) {
        const int64_t l = sg[k] - A->row_begin;
        if (l < 0 || l >= A->n_local) return fail(c, VTK_ERR_STATE, "halo request for a row this rank does not own");
        sl[k] = (int32_t)l;
    }
    HIPCHK(c, hipMalloc(&A->d_send_idx, std::max<int64_t>(1, A->n_send) * sizeof(int32_t)));
    HIPCHK(c, hipMalloc(&A->d_send_buf, std::max<int64_t>(1, A->n_send) * sizeof(double)));
    HIPCHK(c, hipMalloc(&A->d_halo, std::max<int64_t>(1, nh) * sizeof(double)));
    if (A->n_send) HIPCHK(c, hipMemcpy(A->d_send_idx, sl.data(), A->n_send * sizeof(int32_t), hipMemcpyHostToDevice));
    return VTK_OK;
}

void free_pack(vtk_csr *A) {
    (void)hipFree(A->sell.d_pk);
    (void)hipFree(A->sell.d_pkoff);
    (void)hipFree(A->sell.d_dict);
    A->sell.d_pk = nullptr;
    A->sell.d_pkoff = nullptr;
    A->sell.d_dict = nullptr;
    A->sell.n_wide = 0;
}

void free_sell(vtk_csr *A) {
    free_pack(A);
    (void)hipFree(A->sell.d_off);
    (void)hipFree(A->sell.d_col);
    (void)hipFree(A->sell.d_val);
    A->sell = Sell{};
    A->use_sell = false;
}

// Bytes of the operator one SpMV reads in the layout in use (the algorithmic figure of the
// profile classes): CSR = values + int32 columns + indptr; SELL = values
// (padding included) + offsets, + int32 columns, or (dictionary-coded) 4-bit codes + 64-B
// dictionaries + the wide chunks' int32 columns.
double matrix_bytes(const vtk_csr *A) {
    const double vb = A->fp32 ? 4.0 : 8.0;
    if (!A->use_sell) return (vb + 4.0) * A->nnz + 4.0 * (A->n_local + 1);
    const Sell &sl = A->sell;
    double b = vb * sl.entries + 8.0 * (sl.nch + 1);
    if (sl.d_pk) b += 4.0 * sl.pk_words + 72.0 * sl.nch + 4.0 * sl.wide_entries;
    else b += 4.0 * sl.entries;
    return b;
}

// SELL-64 copy of the (local-index) CSR on the device.  only_if_compact: stop after the
// widths when the padding would exceed 25 % of nnz (AUTO); *built says whether it exists.
int build_sell(vtk_csr *A, bool only_if_compact, bool *built) {
    vtk_ctx *c = A->ctx;
    *built = A->sell.d_col != nullptr;
    if (*built) return VTK_OK;
    const int64_t n = A->n_local, nch = (n + 63) / 64;
    const size_t scan_bytes = std::max<size_t>(sell_scan_bytes(n), 16);
    DBuf tmp, scan;
    TRY(dalloc(c, tmp, (size_t)(nch + 1) * sizeof(int64_t)));
    TRY(dalloc(c, scan, scan_bytes));
    Sell sl;
    HIPCHK(c, hipMalloc(&sl.d_off, (size_t)(nch + 1) * sizeof(int64_t)));
    auto drop = [&]() { (void)hipFree(sl.d_off); (void)hipFree(sl.d_col); (void)hipFree(sl.d_val); };
    hipError_t e = launch_sell_build(A->d_indptr, A->d_indices, A->d_data, A->fp32, n, sl.d_off, tmp.as<int64_t>(),
                                     scan.p, scan_bytes, nullptr, nullptr, 0, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(&sl.entries, sl.d_off + nch, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) { drop(); return fail(c, VTK_ERR_HIP, std::string("SELL build: ") + hipGetErrorString(e)); }
    // nearly uniform widths (the 4D operator: a few chunks of 64 velocity-boundary rows are one
    // entry narrower) are padded to the widest chunk when that costs <= 2 % more entries: every
    // chunk's offset is then 64 W q and the kernels take the compile-time-width path (no offset
    // loads at the head of each chunk)
    if (nch > 0) {
        std::vector<int64_t> off((size_t)nch + 1);
        e = hipMemcpy(off.data(), sl.d_off, off.size() * sizeof(int64_t), hipMemcpyDeviceToHost);
        if (e != hipSuccess) { drop(); return fail(c, VTK_ERR_HIP, std::string("SELL build: ") + hipGetErrorString(e)); }
        int64_t wmax = 0;
        for (int64_t q = 0; q < nch; ++q) wmax = std::max(wmax, (off[(size_t)q + 1] - off[(size_t)q]) >> 6);
        const int64_t uni = nch * 64 * wmax;
        if (wmax > 0 && uni != sl.entries && (double)uni <= 1.02 * (double)sl.entries) {
            for (int64_t q = 0; q <= nch; ++q) off[(size_t)q] = 64 * wmax * q;
            e = hipMemcpy(sl.d_off, off.data(), off.size() * sizeof(int64_t), hipMemcpyHostToDevice);
            if (e != hipSuccess) { drop(); return fail(c, VTK_ERR_HIP, std::string("SELL build: ") + hipGetErrorString(e)); }
            sl.entries = uni;
        }
    }
    if (only_if_compact && (double)sl.entries > 1.25 * (double)A->nnz + 64.0) { drop(); return VTK_OK; }
    const size_t vb = A->fp32 ? 4 : 8;
    e = hipMalloc(&sl.d_col, (size_t)std::max<int64_t>(sl.entries, 1) * 4);
    if (e == hipSuccess) e = hipMalloc(&sl.d_val, (size_t)std::max<int64_t>(sl.entries, 1) * vb);
    if (e == hipErrorOutOfMemory && only_if_compact) { (void)hipGetLastError(); drop(); return VTK_OK; }
    if (e == hipSuccess) e = launch_sell_build(A->d_indptr, A->d_indices, A->d_data, A->fp32, n, sl.d_off, nullptr,
                                               nullptr, 0, sl.d_col, sl.d_val, 1, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) { drop(); return fail(c, e == hipErrorOutOfMemory ? VTK_ERR_NOMEM : VTK_ERR_HIP,
                                              std::string("SELL build: ") + hipGetErrorString(e)); }
    sl.nch = nch;
    // uniform chunk width (the Vlasov operators: every 64-row chunk holds a full-stencil row)
    {
        std::vector<int64_t> off((size_t)nch + 1);
        if (hipMemcpy(off.data(), sl.d_off, off.size() * sizeof(int64_t), hipMemcpyDeviceToHost) == hipSuccess && nch > 0) {
            const int64_t w0 = (off[1] - off[0]) >> 6;
            bool uni = w0 > 0 && w0 < (1 << 20);
            for (int64_t q = 1; q < nch && uni; ++q) uni = ((off[(size_t)q + 1] - off[(size_t)q]) >> 6) == w0;
            sl.uniform_w = uni ? (int)w0 : 0;
        }
    }
    A->sell = sl;
    *built = true;
    return VTK_OK;
}

// Dictionary-coded columns of the SELL copy (k_sell_pack); the int32 columns stay for the
// chunks with too many distinct offsets.  Best effort: out of memory leaves the copy unpacked.
int build_pack(vtk_csr *A) {
    vtk_ctx *c = A->ctx;
    Sell &sl = A->sell;
    if (sl.d_pk || !sl.d_col) return VTK_OK;
    const int64_t nch = sl.nch;
    const size_t scan_bytes = std::max<size_t>(sell_scan_bytes(A->n_local), 16);
    DBuf tmp, scan, cnt;
    TRY(dalloc(c, tmp, (size_t)(nch + 1) * sizeof(int64_t)));
    TRY(dalloc(c, scan, scan_bytes));
    TRY(dalloc(c, cnt, 2 * sizeof(unsigned long long)));
    int64_t words = 0;
    unsigned long long wide[2] = {0, 0};
    hipError_t e = hipMalloc(&sl.d_pkoff, (size_t)(nch + 1) * sizeof(int64_t));
    if (e == hipSuccess) e = launch_sell_pack(sl.d_off, nch, sl.d_pkoff, tmp.as<int64_t>(), scan.p, scan_bytes, nullptr,
                                              nullptr, nullptr, nullptr, 0, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(&words, sl.d_pkoff + nch, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMalloc(&sl.d_pk, (size_t)std::max<int64_t>(words, 1) * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&sl.d_dict, (size_t)std::max<int64_t>(nch, 1) * 16 * sizeof(int32_t));
    if (e == hipSuccess) e = hipMemsetAsync(cnt.p, 0, 2 * sizeof(unsigned long long), c->stream);
    if (e == hipSuccess) e = launch_sell_pack(sl.d_off, nch, sl.d_pkoff, nullptr, nullptr, 0, sl.d_col, sl.d_pk,
                                              sl.d_dict, cnt.as<unsigned long long>(), 1, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(wide, cnt.p, sizeof(wide), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipErrorOutOfMemory) { (void)hipGetLastError(); free_pack(A); return VTK_OK; }
    if (e != hipSuccess) { free_pack(A); return fail(c, VTK_ERR_HIP, std::string("SELL pack: ") + hipGetErrorString(e)); }
    sl.n_wide = (int64_t)wide[0];
    sl.wide_entries = (int64_t)wide[1];
    sl.pk_words = words;
    return VTK_OK;
}

int upload_groups(vtk_ctx *c, const std::vector<int32_t> &list, int gmax, Groups &g) {
    (void)hipFree(g.d_list);
    g.d_list = nullptr;
    g.count = (int)list.size();
    g.grid = std::max(1, std::min(g.count, gmax));
    HIPCHK(c, hipMalloc(&g.d_list, std::max<size_t>(list.size(), 1) * sizeof(int32_t)));
    if (!list.empty()) HIPCHK(c, hipMemcpy(g.d_list, list.data(), list.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    return VTK_OK;
}

// groups of 4 chunks (256 rows); world > 1: interior groups (no row reads a halo column) and
// boundary groups for the overlapped exchange (grids <= 64 and the rest of GMAX)
int build_groups(vtk_csr *A) {
    vtk_ctx *c = A->ctx;
    const int ng = (int)((A->n_local + 255) / 256);
    A->g_all.count = ng;
    A->g_all.grid = grid_for(c, std::max(1, std::min(ng, GMAX)));
    if (c->dist && A->row_halo.size() == (size_t)A->n_local) {
        std::vector<int32_t> gi, gb;
        for (int g = 0; g < ng; ++g) {
            bool h = false;
            for (int64_t r = 256 * (int64_t)g; r < std::min<int64_t>(A->n_local, 256 * (int64_t)g + 256) && !h; ++r)
                h = A->row_halo[(size_t)r] != 0;
            (h ? gb : gi).push_back(g);
        }
        TRY(upload_groups(c, gb, 64, A->g_bd));
        TRY(upload_groups(c, gi, GMAX - A->g_bd.grid, A->g_in));
    }
    return VTK_OK;
}

int apply_layout(vtk_csr *A, int layout) {
    vtk_ctx *c = A->ctx;
    if (layout == VTK_LAYOUT_CSR) {
        free_sell(A);
    } else {
        bool built = false;
        TRY(build_sell(A, layout == VTK_LAYOUT_AUTO, &built));
        A->use_sell = built;
        if (built && !A->g_all.grid) TRY(build_groups(A));
        if (built && layout == VTK_LAYOUT_SELL32) free_pack(A);
        else if (built) TRY(build_pack(A));
    }
    A->layout = layout;
    (void)c;
    return VTK_OK;
}

int finish_csr(vtk_csr *A) {
    vtk_ctx *c = A->ctx;
    if (c->dist) TRY(setup_halo(A));
    TRY(upload_tiles(c, A->h_indptr, 1, A->tiles));
    TRY(build_groups(A));
    TRY(apply_layout(A, VTK_LAYOUT_AUTO));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VTK_OK;
}

int check_partition(vtk_ctx *c, int64_t n_global, const int64_t *offsets, std::vector<int64_t> &out) {
    out.resize(c->world + 1);
    if (c->world == 1) {
        out[0] = 0;
        out[1] = n_global;
        if (offsets && (offsets[0] != 0 || offsets[1] != n_global)) return fail(c, VTK_ERR_ARG, "offsets must be {0, n}");
        return VTK_OK;
    }
    if (!offsets) return fail(c, VTK_ERR_ARG, "offsets required when world > 1");
    for (int q = 0; q <= c->world; ++q) out[q] = offsets[q];
    if (out[0] != 0 || out[c->world] != n_global) return fail(c, VTK_ERR_ARG, "offsets must span [0, n)");
    for (int q = 0; q < c->world; ++q)
        if (out[q + 1] < out[q]) return fail(c, VTK_ERR_ARG, "offsets must be non-decreasing");
    return VTK_OK;
}

void destroy_csr(vtk_csr *A) {
    if (!A) return;
    (void)hipSetDevice(A->device);
    (void)hipFree(A->d_indptr);
    (void)hipFree(A->d_indices);
    (void)hipFree(A->d_data);
    (void)hipFree(A->tiles.d_row);
    (void)hipFree(A->d_halo);
    (void)hipFree(A->d_send_idx);
    (void)hipFree(A->d_send_buf);
    (void)hipFree(A->d_lsv);
    (void)hipFree(A->d_g4tab);
    (void)hipFree(A->d_g4D);
    free_sell(A);
    (void)hipFree(A->g_in.d_list);
    (void)hipFree(A->g_bd.d_list);
    delete A;
}

// line-band structure check (vtk_csr_set_line_band): VTK_OK when every column of every row lies
// in the lines x-1..x+1 (mod X) of the row's line; VTK_ERR_ARG (no error text) otherwise
// Distributed operators (world > 1, or a one-rank communicator): the slab must hold whole lines
// and its halo must be exactly the two neighbour lines (left: the line before the slab, right: the
// one after it, periodic); the per-step ghost exchange layout is derived here
// into `out`, which the caller commits only once the whole check has passed.
struct BandLayout {
    int lblk = 0;
    int xord = 0;   // bit 0: the slab starts at global line 0, bit 1: it ends at the last line
    int peer[2] = {-1, -1};
    std::vector<int64_t> scnt, soff, rcnt, roff;
    int64_t off_first = -1, off_last = -1, off_left = -1, off_right = -1;
};

int band_check_dist(vtk_csr *A, int64_t L, bool &solo, BandLayout &out) {
    vtk_ctx *c = A->ctx;
    const int64_t n = A->n_local, Xg = A->n_global / L;
    solo = A->n_halo == 0 && A->n_send == 0;
    if (solo) return VTK_OK;   // no neighbour: the one-rank form (periodic wrap inside the slab)
    if (A->n_global % L != 0 || A->row_begin % L != 0 || n < 2 * L || A->n_halo != 2 * L) return VTK_ERR_ARG;
    const int64_t left = (A->row_begin / L - 1 + Xg) % Xg, right = (A->row_end / L) % Xg;
    if (left == right) return VTK_ERR_ARG;
    int64_t gl[2];
    for (int b = 0; b < 2; ++b) {
        gl[b] = A->halo_cols[(size_t)b * L] / L;
        for (int64_t v = 0; v < L; ++v)
            if (A->halo_cols[(size_t)(b * L + v)] != gl[b] * L + v) return VTK_ERR_ARG;
    }
    if (!((gl[0] == left && gl[1] == right) || (gl[0] == right && gl[1] == left))) return VTK_ERR_ARG;
    out.lblk = gl[0] == left ? 0 : 1;
    out.xord = (A->row_begin == 0 ? 1 : 0) | (A->row_end == A->n_global ? 2 : 0);
    auto owner = [&](int64_t line) {
        for (int q = 0; q < c->world; ++q)
            if (A->offsets[q] <= line * L && line * L < A->offsets[q + 1]) return q;
        return -1;
    };
    const int pl = owner(left), pr = owner(right);
    if (pl < 0 || pr < 0 || pl == c->rank || pr == c->rank) return VTK_ERR_ARG;
    out.peer[0] = pl;
    out.peer[1] = pr;
    // per peer: sends [my last line if it is my right neighbour][my first line if it is my left],
    // receives [into the left ghost if it is my left neighbour][into the right ghost if my right]:
    // a pair that is both (two ranks) matches last line -> left ghost, first line -> right ghost
    const int W = c->world;
    out.scnt.assign(W, 0);
    out.soff.assign(W, 0);
    out.rcnt.assign(W, 0);
    out.roff.assign(W, 0);
    int64_t so = 0, ro = 0;
    for (int q = 0; q < W; ++q) {
        out.soff[q] = so;
        out.roff[q] = ro;
        if (q == pr) { out.off_last = so; so += BAND_GHOST_VECS * L; }
        if (q == pl) { out.off_first = so; so += BAND_GHOST_VECS * L; }
        if (q == pl) { out.off_left = ro; ro += BAND_GHOST_VECS * L; }
        if (q == pr) { out.off_right = ro; ro += BAND_GHOST_VECS * L; }
        out.scnt[q] = so - out.soff[q];
        out.rcnt[q] = ro - out.roff[q];
    }
    return VTK_OK;
}

// local check of line length L (no collective): on success `out` holds the layout and the
// v-locality / ghost flags for band_check_all to commit
struct BandCheck {
    BandLayout lay;
    bool vloc = false, ghost = false;
};

int band_check(vtk_csr *A, int64_t L, BandCheck &out) {
    vtk_ctx *c = A->ctx;
    const int64_t n = A->n_local;
    // the structure only: whole lines, >= 2 of them, rows and the two halo lines within the
    // kernels' 32-bit indices.  Whether the band STEP can run on it (line parts of <= 400 rows,
    // multiples of 8: vtk_line_band_plan) is run_gmres's decision; the line path's table SpMV and
    // the SELL launches need the structure alone.
    if (L <= 0 || n <= 0 || n % L != 0 || n / L < 2 || n + 2 * L >= INT32_MAX / 2) return VTK_ERR_ARG;
    bool solo = true;
    if (c->dist && band_check_dist(A, L, solo, out.lay) != VTK_OK) return VTK_ERR_ARG;
    if (solo && n / L < 3) return VTK_ERR_ARG;
    DBuf bad;
    TRY(dalloc(c, bad, sizeof(int)));
    HIPCHK(c, hipMemsetAsync(bad.p, 0, sizeof(int), c->stream));
    if (solo) HIPCHK(c, launch_band_check(A->d_indptr, A->d_indices, n, (int)L, (int)(n / L), bad.as<int>(), c->stream));
    else HIPCHK(c, launch_band_check_dist(A->d_indptr, A->d_indices, n, (int)L, out.lay.lblk, bad.as<int>(), c->stream));
    int hb = 1;
    HIPCHK(c, hipMemcpyAsync(&hb, bad.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (hb & 1) return VTK_ERR_ARG;
    out.vloc = (hb & 2) == 0;
    out.ghost = !solo;
    return VTK_OK;
}

// band_check on every rank, then one agreement: the line band is set on all ranks or on none
// (collective when the context is distributed).  VTK_OK: set; VTK_ERR_ARG: not a line-band
// operator on some rank; other codes: a HIP / communicator failure on this rank.
int band_check_all(vtk_csr *A, int64_t L) {
    vtk_ctx *c = A->ctx;
    BandCheck chk;
    int rc = band_check(A, L, chk);
    // line-separable values (rank-local: the kernels read them or the SELL values, the same bits
    // either way): built into a scope-owned buffer and checked against the CSR bit for bit;
    // committed below together with the layout only once every rank has passed
    DBuf lsv;
    bool lsv_ok = false, canon = false;
    const int64_t n = A->n_local;
    if (rc == VTK_OK && !A->fp32) {
        const size_t nl = (size_t)n + 2 * (size_t)L + 2 * (size_t)(n / L);
        DBuf bad;
        rc = dalloc(c, lsv, nl * sizeof(double));
        if (rc == VTK_OK) rc = dalloc(c, bad, sizeof(int));
        int hb = 1;
        hipError_t e = hipSuccess;
        if (rc == VTK_OK) e = hipMemsetAsync(lsv.p, 0, nl * sizeof(double), c->stream);
        if (rc == VTK_OK && e == hipSuccess) e = hipMemsetAsync(bad.p, 0, sizeof(int), c->stream);
        if (rc == VTK_OK && e == hipSuccess)
            e = launch_lsv_build(A->d_indptr, A->d_indices, static_cast<const double *>(A->d_data), n, (int)L,
                                 chk.ghost ? chk.lay.lblk : -1, chk.ghost ? chk.lay.xord : 0, lsv.as<double>(), bad.as<int>(),
                                 c->stream);
        if (rc == VTK_OK && e == hipSuccess) e = hipMemcpyAsync(&hb, bad.p, sizeof(int), hipMemcpyDeviceToHost, c->stream);
        if (rc == VTK_OK && e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (rc == VTK_OK && e != hipSuccess)
            rc = fail(c, e == hipErrorOutOfMemory ? VTK_ERR_NOMEM : VTK_ERR_HIP, std::string("line values: ") + hipGetErrorString(e));
        lsv_ok = rc == VTK_OK && (hb & 1) == 0;
        canon = lsv_ok && (hb & 2) == 0;
    }
    if (c->dist) {
        // the agreement runs even after a local failure: every rank joins the same collective
        double mine = rc == VTK_OK ? 0.0 : 1.0, bad = 0.0;
        HIPCHK(c, hipMemcpyAsync(&c->d_scal[DC_NQ + 2], &mine, sizeof(double), hipMemcpyHostToDevice, c->stream));
        TRY(comm_allreduce(c, &c->d_scal[DC_NQ + 2], 1));
        HIPCHK(c, hipMemcpyAsync(&bad, &c->d_scal[DC_NQ + 2], sizeof(double), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (rc == VTK_OK && bad != 0.0) rc = VTK_ERR_ARG;
    }
    if (rc != VTK_OK) return rc;
    // every rank passed: commit the layout and the tables (band_L is set by the caller)
    A->band_vloc = chk.vloc;
    A->band_ghost = chk.ghost;
    A->band_lblk = chk.lay.lblk;
    A->band_xord = chk.ghost ? chk.lay.xord : 0;
    A->band_peer[0] = chk.lay.peer[0];
    A->band_peer[1] = chk.lay.peer[1];
    A->band_scnt = chk.lay.scnt;
    A->band_soff = chk.lay.soff;
    A->band_rcnt = chk.lay.rcnt;
    A->band_roff = chk.lay.roff;
    A->band_off_first = chk.lay.off_first;
    A->band_off_last = chk.lay.off_last;
    A->band_off_left = chk.lay.off_left;
    A->band_off_right = chk.lay.off_right;
    (void)hipFree(A->d_lsv);
    A->d_lsv = nullptr;
    A->lsv_canon = false;
    if (lsv_ok) {
        A->d_lsv = lsv.as<double>();
        lsv.p = nullptr;   // owned by the operator now
        A->lsv_canon = canon;
    }
    return VTK_OK;
}

// Line length the drop-in path (vtk_csr_create) tries: the smallest column distance > 1
// (periodic in n) that the first and the last local row both couple to -- for the 2D Vlasov
// operators Nv, their x-neighbour couplings (row = x Nv + v).  0 when there is none.  Collective
// (world > 1): the ranks' candidates must agree, else 0 everywhere.
int line_len_candidate(vtk_csr *A, int64_t &L) {
    vtk_ctx *c = A->ctx;
    const int64_t n = A->n_local, N = A->n_global;
    L = 0;
    // the local candidate; a HIP failure here votes "no candidate" (-1) instead of returning, so
    // that every rank still joins the allgather below
    auto local = [&]() -> int {
        std::vector<int64_t> d[2];
        if (n < 1) return VTK_OK;
        HIPCHK(c, hipStreamSynchronize(c->stream));
        for (int s = 0; s < 2; ++s) {
            const int64_t r = s == 0 ? 0 : n - 1;
            const int32_t k0 = A->h_indptr[(size_t)r], k1 = A->h_indptr[(size_t)r + 1];
            std::vector<int32_t> idx((size_t)std::max(0, k1 - k0));
            if (k1 > k0) HIPCHK(c, hipMemcpy(idx.data(), A->d_indices + k0, (k1 - k0) * sizeof(int32_t), hipMemcpyDeviceToHost));
            for (int32_t l : idx) {
                const int64_t g = l < n ? l + A->row_begin : A->halo_cols[(size_t)(l - n)];
                int64_t dist = std::llabs(g - (A->row_begin + r));
                dist = std::min(dist, N - dist);
                if (dist > 1) d[s].push_back(dist);
            }
            std::sort(d[s].begin(), d[s].end());
        }
        for (int64_t v : d[0])
            if (std::binary_search(d[1].begin(), d[1].end(), v)) { L = v; break; }
        return VTK_OK;
    };
    const int lrc = local();
    if (lrc != VTK_OK) L = -1;
    if (c->dist && c->world > 120) {
        // the agreement below gathers into the context's scalar scratch (room for 120 ranks, no
        // allocation that could fail on one rank only).  Beyond that every rank
        // skips the detection alike -- no collective, the plain path; vtk_csr_set_line_band
        // still sets the band explicitly
        L = 0;
        return lrc;
    }
    if (c->dist) {
        const int W = c->world;
        int64_t *mine = reinterpret_cast<int64_t *>(c->d_scal + 128);
        HIPCHK(c, hipMemcpyAsync(mine, &L, sizeof(int64_t), hipMemcpyHostToDevice, c->stream));
        TRY(comm_allgather_i64(c, mine, mine + 1, 1));
        std::vector<int64_t> h((size_t)W);
        HIPCHK(c, hipMemcpyAsync(h.data(), mine + 1, W * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        for (int64_t v : h)
            if (v != h[0]) { L = 0; break; }
        if (L != 0) L = h[0];
    }
    if (L < 0) L = 0;
    return lrc;
}

// 4D grid structure (vtk::Grid4): tables built and every entry checked on the device; rank-local
// (the kernels read the tables or the SELL copy, the same bits either way: no agreement needed).
// VTK_ERR_ARG when the operator is not such a grid (the state is then unchanged).
int grid4_set(vtk_csr *A, int64_t Ny, int64_t Nvx, int64_t Nvy) {
    vtk_ctx *c = A->ctx;
    const int64_t n = A->n_local, S4 = Ny * Nvx * Nvy;
    if (Ny < 3 || Nvx < 2 || Nvy < 2 || S4 <= 0 || S4 > INT32_MAX || n <= 0 || n % S4 != 0 || A->n_global % S4 != 0 ||
        n + 2 * S4 >= INT32_MAX / 2)
        return VTK_ERR_ARG;
    Grid4 g;
    g.Ny = (int)Ny;
    g.Nvx = (int)Nvx;
    g.Nvy = (int)Nvy;
    g.X = (int)(n / S4);
    if (c->dist) {   // across ranks: whole x planes, the halo = the two neighbour planes
        bool solo = true;
        BandLayout lay;
        if (band_check_dist(A, S4, solo, lay) != VTK_OK) return VTK_ERR_ARG;
        if (!solo) {
            g.lblk = lay.lblk;
            g.xord = (A->row_begin == 0 ? 1 : 0) | (A->row_end == A->n_global ? 2 : 0);
        }
    }
    if (g.lblk < 0 && g.X < 3) return VTK_ERR_ARG;
    DBuf tab, D, bad;
    TRY(dalloc(c, tab, grid4_tab_len(g) * sizeof(double)));
    TRY(dalloc(c, D, (size_t)n * (A->fp32 ? 4 : 8)));
    TRY(dalloc(c, bad, sizeof(int)));
    HIPCHK(c, hipMemsetAsync(tab.p, 0, grid4_tab_len(g) * sizeof(double), c->stream));
    HIPCHK(c, hipMemsetAsync(bad.p, 0, sizeof(int), c->stream));
    HIPCHK(c, launch_grid4_build(A->d_indptr, A->d_indices, A->d_data, A->fp32, n, g, tab.as<double>(), D.p,
                                 bad.as<int>(), c->stream));
    int hb = 1;
    HIPCHK(c, hipMemcpyAsync(&hb, bad.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (hb != 0) return VTK_ERR_ARG;
    (void)hipFree(A->d_g4tab);
    (void)hipFree(A->d_g4D);
    A->d_g4tab = tab.as<double>();
    A->d_g4D = D.p;
    tab.p = D.p = nullptr;
    g.tab = A->d_g4tab;
    g.D = A->d_g4D;
    A->g4 = g;
    return VTK_OK;
}

// the drop-in path's 4D grid detection: the distinct column distances of the first local row
// (periodic in n) are 1, Nvy, Nvx Nvy, Ny Nvx Nvy for the 4D Vlasov operators (0: no candidate)
int grid4_candidate(vtk_csr *A, int64_t &Ny, int64_t &Nvx, int64_t &Nvy) {
    vtk_ctx *c = A->ctx;
    const int64_t n = A->n_local, N = A->n_global;
    Ny = Nvx = Nvy = 0;
    if (n < 1) return VTK_OK;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const int32_t k0 = A->h_indptr[0], k1 = A->h_indptr[1];
    if (k1 - k0 < 5 || k1 - k0 > 64) return VTK_OK;
    std::vector<int32_t> idx((size_t)(k1 - k0));
    HIPCHK(c, hipMemcpy(idx.data(), A->d_indices + k0, (k1 - k0) * sizeof(int32_t), hipMemcpyDeviceToHost));
    std::vector<int64_t> d;
    for (int32_t l : idx) {
        const int64_t g = l < n ? l + A->row_begin : A->halo_cols[(size_t)(l - n)];
        int64_t dist = std::llabs(g - A->row_begin);
        dist = std::min(dist, N - dist);
        if (dist > 0) d.push_back(dist);
    }
    std::sort(d.begin(), d.end());
    d.erase(std::unique(d.begin(), d.end()), d.end());
    // {1, S2, S3, S4}, plus the periodic y wrap S4 - S3 (= (Ny - 1) S3) when Ny > 2
    if (d.size() < 4 || d.size() > 5 || d[0] != 1) return VTK_OK;
    const int64_t S2 = d[1], S3 = d[2], S4 = d.back();
    if (S3 % S2 != 0 || S4 % S3 != 0 || (d.size() == 5 && d[3] != S4 - S3)) return VTK_OK;
    Nvy = S2;
    Nvx = S3 / S2;
    Ny = S4 / S3;
    return VTK_OK;
}

int auto_grid4(vtk_csr *A) {
    if (!A->ctx->tune.auto_band) return VTK_OK;
    int64_t Ny, Nvx, Nvy;
    TRY(grid4_candidate(A, Ny, Nvx, Nvy));
    if (Ny <= 0) return VTK_OK;
    const int rc = grid4_set(A, Ny, Nvx, Nvy);
    // no such grid, or no memory for its tables: the operator keeps the SELL path (the detection is
    // a speed-up the drop-in CSR does not need)
    if (rc == VTK_ERR_NOMEM) A->ctx->err.clear();
    return rc == VTK_ERR_ARG || rc == VTK_ERR_NOMEM ? VTK_OK : rc;
}

// the drop-in path's line-band detection: the same check vtk_csr_set_line_band runs, on the
// candidate line length (tuning auto_band 0: off)
int auto_line_band(vtk_csr *A) {
    if (!A->ctx->tune.auto_band) return VTK_OK;
    int64_t L = 0;
    TRY(line_len_candidate(A, L));
    if (L <= 0) return VTK_OK;   // uniform across ranks: nobody enters the collective below
    const int rc = band_check_all(A, L);   // collective: every rank gets here (L agreed above)
    if (rc == VTK_OK) A->band_L = L;
    else if (rc == VTK_ERR_NOMEM) A->ctx->err.clear();   // no memory for the tables: not detected
    else if (rc != VTK_ERR_ARG) return rc;
    return VTK_OK;
}

// ---- GMRES -----------------------------------------------------------------------------------


struct Solver {
    vtk_csr *A;
    vtk_prec *M;
    vtk_ctx *c;
    int64_t n, ld;
    int m, G;
    double *V, *w, *tmp, *r, *H, *S, *giv;
    double *part[4];
    double *Hraw = nullptr, *dcpart = nullptr;   // DCGS2
    DcCoef *cf = nullptr;
    double *x = nullptr;                         // the solution (the DCGS2 update pass may update it)
    // line-band DCGS2 step (k_band_step): grid, parts per line; w rotates over s.w, s.tmp, w3
    // (step j's w in the buffer j % 3: the band step reads w_{j-1} and w_j, writes w_{j+1})
    bool band = false;
    int band_G = 0, band_H = 1;
    int band_G3 = 0;   // grid of the three-workgroups-per-CU launches (band_opt bit 1, j <= BAND_J3)
    // workgroups (= partials) of the band step launched at step j
    int band_grid(int j, int opt) const { return (opt & 2) && j <= BAND_J3 && band_G3 > 0 ? band_G3 : band_G; }
    double *w3 = nullptr;
    double *ghost = nullptr, *gsend = nullptr, *grecv = nullptr;   // distributed band step
    // across ranks: the first launch of this rank that failed (soft_launch), and the fail_step
    // test hook still to fire in this solve
    int local_rc = VTK_OK;
    bool fail_pending = false;
};

// A launch of the solve that failed.  On one rank: the error returns at once.  Across ranks the
// peers are already inside this step's collectives, so returning would leave them blocked: the
// rank records its error, sets its failure vote (d_scal[DC_VOTE + 1], summed into the step's
// all-reduce by k_dc_finalize) and goes on issuing the same launches and collectives; the vote
// stops every rank's cycle at the same step and vtk_gmres returns the error there (VTK_ERR_PEER
// on the other ranks).  (Pattern: the reference's step runner turns a step's exception into a
// return code, precondition_setup/vtsetup/vt_precondition.py:66-79.)
int soft_launch(Solver &s, hipError_t e, const char *what) {
    vtk_ctx *c = s.c;
    if (e == hipSuccess) return VTK_OK;
    const int code = e == hipErrorOutOfMemory ? VTK_ERR_NOMEM : VTK_ERR_HIP;
    const std::string msg = std::string(what) + ": " + hipGetErrorString(e);
    if (!c->dist) return fail(c, code, msg);
    if (s.local_rc == VTK_OK) {
        s.local_rc = fail(c, code, msg + " (the ranks left the solve together at the next all-reduce)");
        HIPCHK(c, hipMemsetAsync(&c->d_scal[DC_VOTE + 1], 1, sizeof(double), c->stream));
    }
    return VTK_OK;
}
#define SOFT(x) TRY(soft_launch(s, (x), #x))

// w = M^-1 A v (fused when the tiles allow), partials: part[0] = w^2 (h0), part[1] = v0*w
// the x-line ring with the solver's epilogues (k_lsv_ring_epi): one rank, line-separable canonical
// rows, their tables in use (tunings band_lsv, sell_canon), the tridiagonal BJ(8) when bj
// (across ranks: the slab's x-halo lines come from the two neighbour lines of the halo -- band_ghost --
// or, on a rank without neighbours, the one-rank wrap)
bool cyc_ring_ok(vtk_ctx *c, const vtk_csr *A, const vtk_prec *M, bool bj) {
    const bool solo = !c->dist || (A->n_halo == 0 && A->n_send == 0 && !A->band_ghost);
    if (c->tune.cyc_ring <= 0 || (!solo && !A->band_ghost) || !A->d_lsv || !A->lsv_canon || A->band_L <= 0 ||
        A->band_L % 8 != 0 || !c->tune.band_lsv || !c->tune.sell_canon || band_parts(A->band_L) < 1 ||
        A->n_local / A->band_L < (A->band_ghost ? 2 : 3))
        return false;
    if (!bj) return true;
    return M && M->kind == VTK_PREC_BJACOBI && M->bs == 8 && bj_op(M).tri != nullptr;
}

// the 4D grid rows' cycle-start residual through k_g4_ring (tuning g4_ring; BJ(8) tridiag)
// (only for grids whose window and tables fit the kernel's LDS, g4_ring_fits; larger 4D
// grids keep the SELL grid-row kernels)
bool g4_resid_ok(vtk_ctx *c, const vtk_csr *A, const vtk_prec *M) {
    return A->d_g4tab && c->tune.grid4 && c->tune.g4_ring > 0 && A->use_sell &&
           A->sell.uniform_w > 8 && M && M->kind == VTK_PREC_BJACOBI && M->bs == 8 && bj_op(M).tri != nullptr &&
           g4_ring_fits(A->g4, A->n_local, c->tune.g4_gr);
}

// the line path's table SpMV: the line-separable, canonical rows' tables (tunings band_lsv,
// sell_canon) of a uniform width-5 SELL copy; across ranks with the ghost lines
bool line_lsv_ok(vtk_ctx *c, const vtk_csr *A) {
    return A->d_lsv && A->band_L > 0 && c->tune.band_lsv && A->use_sell && A->sell.uniform_w == 5 && A->sell.d_pk &&
           A->sell.n_wide == 0 && (!c->dist || A->band_ghost);
}
// ... and the SpMV inside the sweep kernel (k_line_spmv_dc, tuning line_fuse): one rank, canonical
// rows, compact factors over the whole slab
bool line_fuse_ok(vtk_ctx *c, const vtk_csr *A, const vtk_prec *M) {
    if (!M || M->kind != VTK_PREC_LINE || !line_lsv_ok(c, A) || !A->lsv_canon || !c->tune.sell_canon ||
        !c->tune.line_fuse || c->dist)
        return false;
    const LineOp &lo = M->line;
    const int64_t n = A->n_local;
    return lo.seg >= 1 && lo.seg <= 32 && lo.compact && lo.stride == A->band_L && lo.row0 == 0 && lo.n == n &&
           lo.j0 == 0 && lo.jn == lo.stride && lo.ac && lo.i_lo == 0 && lo.i_hi == n / lo.stride - 1 &&
           n / lo.stride >= 3;
}

int precond_matvec(Solver &s, const double *v, double *w, const int *stop, int col, Red &h0, Red &d0,
                   bool want_dots = true) {
    vtk_ctx *c = s.c;
    vtk_csr *A = s.A;
    TRY(halo_exchange(A, v));
    const double *v0 = want_dots ? s.V : nullptr;
    const double n8 = 8.0 * s.n;
    const double b_csr = solver_matrix_bytes(A);
    const double b_inv = bj_row_bytes(s.M) * s.n;
    int cnt;
    if (!s.M) {
        Prof pf(c, "spmv_w", col, b_csr + 3 * n8);
        const SpmvIn in = lsv_in(spmv_in(A, &A->tiles, v), A);
        HIPCHK(c, launch_spmv(in, EPI_PREC, w, nullptr, BjOp{}, v0, s.part[0], s.part[1], stop, col, c->stream));
        cnt = spmv_grid(in);
    } else if (bj_fused(s.M)) {
        Prof pf(c, "spmv_bj", col, b_csr + b_inv + 3 * n8);   // x, v0, w + CSR + BJ rows
        const SpmvIn in = lsv_in(spmv_in(A, &s.M->tiles, v), A);
        HIPCHK(c, launch_spmv(in, EPI_PREC, w, nullptr, bj_op(s.M), v0, s.part[0], s.part[1], stop, col, c->stream));
        cnt = spmv_grid(in);
    } else {
        {
            Prof pf(c, "spmv", col, b_csr + 2 * n8);
            HIPCHK(c, launch_spmv(lsv_in(spmv_in(A, &A->tiles, v), A), EPI_PLAIN, s.tmp, nullptr, BjOp{}, nullptr, nullptr, nullptr, stop, col, c->stream));
        }
        Prof pf(c, prec_cls(s.M), col, b_inv + 3 * n8);
        HIPCHK(c, launch_bj_apply(bj_op(s.M), s.n, s.tmp, w, v0, s.part[0], s.part[1], s.G, stop, col, c->stream));
        cnt = s.G;
    }
    int rc = VTK_OK;
    if (!want_dots) return rc;
    h0 = reduce(c, s.part[0], cnt, rc);
    TRY(rc);
    d0 = reduce(c, s.part[1], cnt, rc);
    return rc;
}

// One restart cycle with DCGS2 (see vtk_kernels.hip, DCGS2 Arnoldi).  Step j's SpMV, dots,
// finalize and scalar kernels are tagged with column j-1 (the column they finalise), its update
// pass with column j.  After column m-1, a closing reduction finalises it.
int dcgs2_cycle(Solver &s, const int *stop, volatile int *mirror, hipEvent_t *ev) {
    vtk_ctx *c = s.c;
    GmresState *ds = c->d_state;
    const int m = s.m;
    const int64_t n = s.n;
    const double n8 = 8.0 * n;
    // every kernel of step j is tagged j: it returns at entry once stop_col < j
    // SpMV + BJ and the step's dots in one pass for BJ-fused tiles with bs <= 8 (larger blocks
    // would spill the fused kernel's registers)
    // ... except for rows wider than 8 (the 4D operator: 9 entries) without a halo to overlap:
    // there the SpMV + BJ kernel and the streaming dots kernel beat the register-capped fused
    // kernel (C4: 707 + 658 us vs 1473 us per step, 422 vs 405 it/s)
    // (with the 4D grid rows (Grid4) the fused kernel loads no values or codes: tuning c4_fused)
    const bool g4_fits = s.A->d_g4tab && g4_ring_fits(s.A->g4, n, c->tune.g4_gr);
    const bool g4_fused = s.A->d_g4tab && c->tune.grid4 && c->tune.c4_fused && (c->tune.g4_ring <= 0 || !g4_fits);   // C4 A/B: 213.8 -> 210.3 ms
    // grid rows with x staged through LDS (k_g4_ring) for the split step's SpMV + BJ
    const bool g4_ring = s.A->d_g4tab && c->tune.grid4 && c->tune.g4_ring > 0 && s.A->use_sell && s.M &&
                         s.M->kind == VTK_PREC_BJACOBI && s.M->bs == 8 && bj_op(s.M).tri != nullptr && g4_fits;
    const bool wide9 = s.A->use_sell && s.A->sell.uniform_w > 8 && !bj_split(s.M) && !g4_fused;
    // the ring step also across ranks: interior groups while the halo planes
    // are in flight, the boundary planes' groups once they have landed
    const bool ring4 = g4_ring && s.A->use_sell && s.A->sell.uniform_w > 8 && !g4_fused;
    const bool fused = bj_fused(s.M) && s.M->bs <= 8 && !wide9 && !ring4;
    // line Jacobi with segments <= 32 (register sweeps): dots fused into the sweep kernel
    const bool line_dc = s.M && s.M->kind == VTK_PREC_LINE && s.M->line.seg >= 1 &&
                         s.M->line.seg <= 32 && s.G <= GMAX;
    // line path on a line-separable operator: the SpMV from the tables (VTK_BAND_LSV=0: SELL)
    const bool line_lsv = line_dc && line_lsv_ok(c, s.A);
    const Tiles *ft = s.M ? &s.M->tiles : &s.A->tiles;
    const double b_csr = matrix_bytes(s.A);
    const double b_lsv = b_csr - 8.0 * (double)s.A->sell.entries + 8.0 * (double)n;
    // canonical rows: the diagonal only (tuning sell_canon 0: the codes too; A/B)
    const bool line_canon = line_lsv && s.A->lsv_canon && c->tune.sell_canon;
    const double b_inv = bj_row_bytes(s.M) * n;
    // dots (unless the SpMV wrote them: cnt partials), all-reduce across ranks, scalar step
    // (folding the finalize into the boundary launch's last workgroup was measured slower: one
    // workgroup summing 2j+3 x ~1000 partials took as long as the 2j+3-workgroup launch)
    // ev_ar (distributed): recorded on the main stream right after the all-reduce, so a
    // communication the caller then issues on the comm stream starts only once the all-reduce
    // has finished: every RCCL operation of the communicator runs in one order, on every rank
    auto reduce_step = [&](int j, const double *w, int tag, int cnt, hipEvent_t ev_ar = nullptr) -> int {
        if (cnt == 0) {
            Prof pf(c, "dc_dots", tag, n8 * (j + (w ? 2 : 1)));
            SOFT(launch_dc_dots(s.V, s.ld, j, w, n, s.dcpart, s.G, stop, tag, c->stream));
            cnt = s.G;
        }
        const double *part = s.dcpart;
        if (c->dist) {
            { Prof pf(c, "dc_finalize", tag, 0.0);
              HIPCHK(c, launch_dc_finalize(s.dcpart, cnt, j, w != nullptr, c->d_scal, stop, tag, c->stream)); }
            {
                Prof pf(c, "allreduce", tag, 8.0 * DC_NQV);
                TRY(comm_allreduce(c, c->d_scal, DC_NQV));   // the dots + the failure vote
            }
            if (ev_ar) HIPCHK(c, hipEventRecord(ev_ar, c->stream));
            part = nullptr;
        }
        Prof pf(c, "dc_scalar", tag, 0.0);
        HIPCHK(c, launch_dc_scalar(part, cnt, c->d_scal, j, m, w == nullptr, s.Hraw, s.H, s.S, s.giv, s.cf, ds,
                                   c->d_stop, c->stream));
        return VTK_OK;
    };
    const bool band = s.band;
    // line-separable values in the band step (tuning band_lsv 0: the SELL values)
    const bool band_lsv = band && s.A->d_lsv && c->tune.band_lsv;
    const bool band_canon = c->tune.band_canon != 0;       // 0: read the codes anyway (A/B)
    // the band step's variant bits exist for the line-separable, canonical-row instantiations (one
    // rank: launch_band_one_rank; across ranks with ghost lines: launch_band_ghost, round 6): every
    // other launch, and the partial count its successor reads, takes the base grid
    // bits 3 (the LDS-DMA prefetch of J > BAND_PF) and 4 (the alternating walk) pay only on long
    // basis vectors: on smaller ones (C2, the C3 slabs) more of the basis stays in the Infinity
    // Cache between steps, so the DMA's issue and L2 over-fetch cost more than the latency it hides
    // and the halo lines' second read hits anyway (band_long_rows, vtk_internal.hpp)
    const int band_opt = band_lsv && s.A->lsv_canon && band_canon
                             ? (n >= c->tune.band_long_rows ? c->tune.band_opt : c->tune.band_opt & ~(8 | 16))
                             : 0;
    // the band step's matrix bytes: SELL codes + dictionary + (values: 8 B per row from D, or
    // the SELL values)
    const double b_band = band_lsv ? (s.A->lsv_canon && band_canon
                                          ? 8.0 * (double)n   // the diagonal only
                                          : b_csr - 8.0 * (double)s.A->sell.entries + 8.0 * (double)n)
                                   : b_csr;
    bool broke = false;
    // an event every 4 steps: r05 library A/B (profiles/r05_ev_every_ab.json) C3/8 slab +2 %,
    // C3 +0.6 %; a stop is acted on at most 3 steps later (early-exit launches, ~us each)
    constexpr int ev_every = 4;
    int ev_step[LOOKAHEAD + 1];
    int nev = 0, synced = 0;
    for (int j = 0; j < m; ++j) {
        double *pj = s.V + (size_t)j * s.ld;
        int cnt = 0;
        const double b_step = solver_matrix_bytes(s.A) + b_inv + n8 * (j + 2);   // matrix, BJ, p, w, V_j
        // band: step j's w and partials come from the band step j-1 (w in buffer j % 3)
        double *const wb[3] = {s.w, s.tmp, s.w3};
        double *w_cur = band ? wb[j % 3] : s.w;
        if (band && j > 0) {
            cnt = s.band_grid(j - 1, band_opt);
        } else if (fused && band && j == 0 && cyc_ring_ok(c, s.A, s.M, true)) {
            // step 0 of a band cycle through the x-line ring (x = v_0; the j = 0 dots only);
            // across ranks the two halo lines first (12.8 KB at C3)
            TRY(halo_exchange(s.A, pj));
            Prof pf(c, "spmv_bj_dc", j, b_step);
            const bool hl = s.A->band_ghost;
            SOFT(launch_lsv_ring_epi(EPI_PREC_DC, s.A->d_lsv, pj, nullptr, s.M->d_tri + s.M->tri_ld, s.w, nullptr,
                                          nullptr, s.dcpart, n, (int)s.A->band_L, c->tune.cyc_ring, stop, j, &cnt,
                                          c->stream, hl ? s.A->d_halo : nullptr, s.A->band_lblk, s.A->band_xord));
        } else if (fused && bj_split(s.M)) {
            // interior tiles while the halo is in flight, boundary tiles once it has landed;
            // their partials side by side (cnt = both grids)
            SpmvIn in = split_in(s.A, s.M, pj, true), bd = split_in(s.A, s.M, pj, false);
            in.halo = nullptr;   // interior tiles read owned columns only
            const double f_in = (s.A->use_sell ? s.A->g_in.count * 256.0 : (double)s.M->tiles_in.nrows) /
                                std::max<double>(1.0, (double)n);
            // a rank with no x-neighbour data to send or receive (one rank) skips the exchange
            // and its event hand-offs; one without boundary rows skips the boundary launch
            const bool exch = s.A->n_send > 0 || s.A->n_halo > 0 || c->host_comm;
            const bool has_bd = s.A->use_sell ? s.A->g_bd.count > 0 : s.M->tiles_bd.ntiles > 0;
            if (exch) TRY(halo_exchange_async(s.A, pj));
            {
                Prof pf(c, "spmv_bj_dc", j, b_step * std::min(1.0, f_in));
                SOFT(launch_spmv_dc(in, s.w, bj_op(s.M), s.V, s.ld, j, s.dcpart, stop, j, c->stream));
            }
            // the all-reduce below stays behind this rank's exchange on every rank (one order
            // of RCCL operations on the communicator)
            if (exch) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_halo, 0));
            cnt = spmv_grid(in);
            if (has_bd) {
                Prof pf(c, "spmv_bj_dc_bd", j, b_step * std::max(0.0, 1.0 - f_in));
                SOFT(launch_spmv_dc(bd, s.w, bj_op(s.M), s.V, s.ld, j, s.dcpart + spmv_grid(in), stop, j,
                                         c->stream));
                cnt += spmv_grid(bd);
            }
        } else if (fused) {
            TRY(halo_exchange(s.A, pj));
            Prof pf(c, "spmv_bj_dc", j, b_step);
            const SpmvIn in = lsv_in(spmv_in(s.A, ft, pj), s.A);
            SOFT(launch_spmv_dc(in, s.w, bj_op(s.M), s.V, s.ld, j, s.dcpart, stop, j, c->stream));
            cnt = spmv_grid(in);
        } else if (line_dc) {
            // line path: SpMV, then the line sweeps with the step's dots fused behind them
            TRY(halo_exchange(s.A, pj));
            const LineOp &lo = s.M->line;
            if (line_canon && line_fuse_ok(c, s.A, s.M)) {
                // one rank: the SpMV inside the sweep kernel (y never stored)
                Prof pf(c, "line_dc", j, b_inv + 8.0 * (double)n + n8 * (j + 2));   // m, D, p, w, V_j
                SOFT(launch_line_spmv_dc(lo, s.A->d_lsv, pj, s.w, s.V, s.ld, j, s.dcpart, s.G, stop, j, c->stream));
                cnt = s.G;
            } else if (line_lsv) {
                // line-separable values: 12 B of matrix per row (codes + diagonal)
                Prof pf(c, "spmv_lsv", j, (line_canon ? 8.0 * (double)n : b_lsv) + 2 * n8);
                SOFT(launch_lsv_spmv(s.A->sell.d_pk, s.A->sell.d_dict, s.A->d_lsv, pj, c->dist ? s.A->d_halo : nullptr,
                                          s.tmp, n, (int)s.A->band_L, s.A->band_ghost ? s.A->band_lblk : -1, stop, j,
                                          c->stream, line_canon ? 1 : 0, 8192, c->tune.lsv_ring,
                                          s.A->band_ghost ? s.A->band_xord : 0));
            } else {
                Prof pf(c, "spmv", j, b_csr + 2 * n8);
                SOFT(launch_spmv(spmv_in(s.A, &s.A->tiles, pj), EPI_PLAIN, s.tmp, nullptr, BjOp{}, nullptr, nullptr,
                                      nullptr, stop, j, c->stream));
            }
            if (!cnt) {
                Prof pf(c, "line_dc", j, b_inv + n8 * (j + 3));   // r, m, w, p, V_j
                SOFT(launch_line_dc(s.M->line, s.tmp, s.w, s.V, s.ld, j, pj, s.dcpart, s.G, stop, j, c->stream));
                cnt = s.G;
            }
        } else if (ring4) {
            // step 0's dots (|p|^2, p.w, |w|^2) in the same sweep; the later steps' dots in
            // k_dc_dots (fused into the ring they cost 215.6 vs 201.5 ms per C4 solve: the ring
            // then runs at 3 waves/SIMD and its basis reads wait behind the ring's)
            G4Dots dd;
            dd.part = s.dcpart;
            const bool dc = j == 0;
            dd.mode = 2;
            const double b_ring = solver_matrix_bytes(s.A) + b_inv + 2 * n8;   // D, m, x, w
            const double *halo = s.A->g4.lblk >= 0 ? s.A->d_halo : nullptr;
            const double *mt = s.M->d_tri + s.M->tri_ld;
            if (!halo || !bj_split(s.M)) {
                TRY(halo_exchange(s.A, pj));
                Prof pf(c, dc ? "spmv_bj_dc" : "spmv_bj", j, b_ring);
                int grid = 0;
                SOFT(launch_g4_ring(s.A->g4, pj, halo, mt, s.w, n, s.A->fp32, c->tune.g4_ring, c->tune.g4_gr,
                                         dc ? &dd : nullptr, &grid, stop, j, c->stream, 0, -1, 0,
                                         c->tune.g4_fast));
                if (dc) cnt = grid;
            } else {
                // across ranks: the rows [S4, n - S4) read no halo plane -- their groups run while
                // the exchange is in flight (comm stream), the first / last plane's groups after it
                // lands; the partials of the three launches side by side
                const int mode = dc ? dd.mode : 0;
                const int G = g4_ring_group(c->tune.g4_gr);
                const int64_t S4 = (int64_t)s.A->g4.Ny * s.A->g4.Nvx * s.A->g4.Nvy, ng = (n + G - 1) / G;
                int64_t gi_lo = (S4 + G - 1) / G, gi_hi = (n - S4) / G;
                if (gi_hi <= gi_lo) gi_lo = gi_hi = 0;   // no interior group: all after the exchange
                const int64_t wgs = std::max(1, c->tune.g4_ring);
                const int per = (int)std::max<int64_t>({g4_ring_per(ng, S4, G, (int)wgs), mode ? (ng + GMAX - 4) / (GMAX - 3) : 1});
                const bool exch = s.A->n_send > 0 || s.A->n_halo > 0 || c->host_comm;
                if (exch) TRY(halo_exchange_async(s.A, pj));
                int gin = 0, gb0 = 0, gb1 = 0;
                {
                    Prof pf(c, dc ? "spmv_bj_dc" : "spmv_bj", j, b_ring * (double)(gi_hi - gi_lo) * G / std::max<double>(1.0, (double)n));
                    if (gi_hi > gi_lo)
                        SOFT(launch_g4_ring(s.A->g4, pj, halo, mt, s.w, n, s.A->fp32, c->tune.g4_ring,
                                                 c->tune.g4_gr, dc ? &dd : nullptr, &gin, stop, j, c->stream, (int)gi_lo,
                                                 (int)gi_hi, per, c->tune.g4_fast));
                }
                if (exch) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_halo, 0));
                {
                    Prof pf(c, "spmv_bj_bd", j, b_ring * std::max(0.0, 1.0 - (double)(gi_hi - gi_lo) * G / std::max<double>(1.0, (double)n)));
                    dd.part_off = gin;
                    SOFT(launch_g4_ring(s.A->g4, pj, halo, mt, s.w, n, s.A->fp32, c->tune.g4_ring,
                                             c->tune.g4_gr, dc ? &dd : nullptr, &gb0, stop, j, c->stream, 0,
                                             (int)(gi_hi > gi_lo ? gi_lo : ng), per, c->tune.g4_fast));
                    if (gi_hi > gi_lo) {
                        dd.part_off = gin + gb0;
                        SOFT(launch_g4_ring(s.A->g4, pj, halo, mt, s.w, n, s.A->fp32, c->tune.g4_ring,
                                                 c->tune.g4_gr, dc ? &dd : nullptr, &gb1, stop, j, c->stream, (int)gi_hi,
                                                 (int)ng, per, c->tune.g4_fast));
                    }
                }
                if (dc) cnt = gin + gb0 + gb1;
            }
        } else {
            Red h0, d0;
            TRY(precond_matvec(s, pj, s.w, stop, j, h0, d0, false));
        }
        // distributed band step: the x-neighbours' edge lines of v_{j-1} and w_j travel to the
        // ghost buffers on the comm stream once this step's all-reduce has finished (ev_pack:
        // the RCCL operations never overlap; the exchange overlaps the scalar step); the band
        // step waits for them
        const bool ghost_x = band && s.ghost && j <= m - 2;
        if (s.fail_pending && j == c->tune.fail_step) {   // test hook: as if this step's launch failed
            s.fail_pending = false;
            TRY(soft_launch(s, hipErrorLaunchFailure, "injected failure (tuning fail_step)"));
        }
        TRY(reduce_step(j, w_cur, j, cnt, ghost_x && c->dist ? c->ev_pack : nullptr));
        if (ghost_x && !c->dist) HIPCHK(c, hipEventRecord(c->ev_pack, c->stream));
        if (ghost_x) {
            vtk_csr *A = s.A;
            const int L = (int)A->band_L;
            HIPCHK(c, hipStreamWaitEvent(c->comm_stream, c->ev_pack, 0));
            SOFT(launch_ghost_pack(s.V, s.ld, j, w_cur, n, L, s.gsend, A->band_off_first, A->band_off_last,
                                        c->comm_stream));
            TRY(comm_alltoallv(c, s.gsend, A->band_scnt, A->band_soff, s.grecv, A->band_rcnt, A->band_roff, ncclDouble,
                               sizeof(double), c->comm_stream));
            SOFT(launch_ghost_unpack(s.grecv, A->band_off_left, A->band_off_right, j, m, L, s.ghost, c->comm_stream));
            HIPCHK(c, hipEventRecord(c->ev_halo, c->comm_stream));
            HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_halo, 0));
        }
        if (band && j <= m - 2) {
            // update pass of step j + SpMV, BJ and dots of step j+1 in one sweep over the x-lines
            // reads V_k (k < j), w_{j-1} (v_0 at j = 0), w_j; writes v_j (j >= 1), w_{j+1} and, at
            // j = m - 2 only, p_{j+1} (k_dc_update's operand)
            // (VTK_PROF_PERJ=1: one profile class per step index, "band_step_jNN")
            const bool perj = c->tune.prof_perj != 0;
            static const char *const jname[] = {"band_step_j00", "band_step_j01", "band_step_j02", "band_step_j03",
                "band_step_j04", "band_step_j05", "band_step_j06", "band_step_j07", "band_step_j08", "band_step_j09",
                "band_step_j10", "band_step_j11", "band_step_j12", "band_step_j13", "band_step_j14", "band_step_j15",
                "band_step_j16", "band_step_j17", "band_step_j18", "band_step_j19"};
            Prof pf(c, perj && j < 20 ? jname[j] : "band_step", j, b_band + b_inv + n8 * (j + (j >= 1 ? 4 : 3) + (j == m - 2 ? 1 : 0)));
            BandK a;
            a.pk = s.A->sell.d_pk;
            a.dict = s.A->sell.d_dict;
            a.val = static_cast<const double *>(s.A->sell.d_val);
            a.mtri = s.M->d_tri + s.M->tri_ld;
            a.V = s.V;
            a.ld = s.ld;
            a.j = j;
            a.m = m;
            a.w_in = w_cur;
            a.w_prev = wb[(j + 2) % 3];
            a.w_out = wb[(j + 1) % 3];
            a.cf = s.cf;
            a.st = ds;
            a.x = s.x;
            a.H = s.H;
            a.S = s.S;
            a.part = s.dcpart;
            a.n = n;
            a.L = (int)s.A->band_L;
            a.X = (int)(n / s.A->band_L);
            a.H_parts = s.band_H;
            a.ghost = s.ghost;
            a.left_blk = s.A->band_lblk;
            a.xord = s.A->band_xord;
            a.lsv = band_lsv ? s.A->d_lsv : nullptr;
            a.canon = band_lsv && s.A->lsv_canon && band_canon ? 2 : 0;   // 2: the straight-line SpMV per line order
            a.opt = band_opt;
            SOFT(launch_band_step(a, s.band_grid(j, a.opt), s.A->sell.uniform_w, c->stream));
        } else {
            Prof pf(c, "dc_update", j, n8 * (j + 4));
            SOFT(launch_dc_update(s.V, s.ld, j, w_cur, n, s.cf, s.G, ds, s.x, s.H, s.S, m, fused ? 0 : 1, c->stream));
        }
        // throttle: an event every ev_every steps (each record costs the stream a few us); the
        // host waits for the event LOOKAHEAD or more steps back and acts on a stop the device
        // has passed there.  Column cc stops in step cc (early commit) or cc+1: act only once
        // every rank ran it.
        if ((j + 1) % ev_every == 0) {
            HIPCHK(c, hipEventRecord(ev[nev % (LOOKAHEAD + 1)], c->stream));
            ev_step[nev % (LOOKAHEAD + 1)] = j;
            ++nev;
        }
        while (synced < nev && ev_step[synced % (LOOKAHEAD + 1)] <= j - LOOKAHEAD) {
            const int js = ev_step[synced % (LOOKAHEAD + 1)];
            HIPCHK(c, hipEventSynchronize(ev[synced % (LOOKAHEAD + 1)]));
            ++synced;
            if (*mirror <= js - 1) { broke = true; break; }
        }
        if (broke) break;
    }
    if (!broke) TRY(reduce_step(m, nullptr, m, 0));   // closing: only if column m-1 is still open
    return VTK_OK;
}

int run_gmres(vtk_csr *A, vtk_prec *M, const double *b, double *x, double rtol, double atol,
              int restart, int64_t maxiter, int *info, vtk_stats *stout) {
    vtk_ctx *c = A->ctx;
    const auto t0 = std::chrono::steady_clock::now();
    const int64_t n = A->n_local, N = A->n_global;
    if (maxiter <= 0) maxiter = N * 10;                     // iterative.py:726-727
    if (restart <= 0) restart = 20;                         // :729-730
    if (restart > N) restart = (int)N;                      // :731
    if (restart > MAX_RESTART) return fail(c, VTK_ERR_ARG, "restart exceeds MAX_RESTART");
    if (restart < 1) return fail(c, VTK_ERR_ARG, "empty system");
    const int m = restart;
    Solver s{A, M, c, n, round_up(std::max<int64_t>(n, 1), 64), m, grid_for(c, vector_grid(n)), nullptr, nullptr,
             nullptr, nullptr, nullptr, nullptr, nullptr, {c->d_part, c->d_part + GMAX, c->d_part + 2 * GMAX, c->d_part + 3 * GMAX}};
    s.x = x;
    // workspace: V[(m+1) x ld] | w | tmp | r | H[m x (m+1)] | S[m+1] | giv[2m]  (doubles)
    const bool dc = c->orth == VTK_ORTH_DCGS2 || (c->orth == VTK_ORTH_AUTO && m <= DC_MAXJ);
    if (dc && m > DC_MAXJ) return fail(c, VTK_ERR_ARG, "DCGS2 supports restart <= 32 (use VTK_ORTH_MGS)");
    const size_t ndc = dc ? (size_t)(m + 1) * (m + 1) + sizeof(DcCoef) / 8 + 8 + (size_t)DC_NQ * GMAX : 0;
    // line-band DCGS2 step: one rank, SELL of uniform width 5 with coded columns (no wide chunk),
    // f64 values, tridiagonal BJ(8) (the fused step's TRIM apply), restart <= 20
    // tuning band 0 (vtk_gmres_set_band): the band step off (tools/ab_env.py alternates it)
    s.band = dc && c->tune.band && A->band_L > 0 && A->band_L % 8 == 0 &&
             (!c->dist || !A->band_ghost || c->comm || c->host_comm) &&
             A->use_sell && A->sell.uniform_w == 5 && A->sell.d_pk && A->sell.n_wide == 0 && !A->fp32 && M &&
             M->kind == VTK_PREC_BJACOBI && M->bs == 8 && bj_fused(M) && bj_op(M).tri != nullptr && m >= 2 && m <= 20;
    int band_R = 0;
    if (s.band) {
        // parts per line (rows per workgroup <= 400; > 1 needs the v-locality of the couplings),
        // two workgroups per CU, >= 2 lines per range (vtk_line_band_plan)
        vtk_band_geometry g{};
        if (vtk_line_band_plan(n, A->band_L, c->n_cu, &g) != VTK_OK || (g.parts > 1 && !A->band_vloc)) {
            s.band = false;
        } else {
            band_R = g.ranges;
            s.band_H = g.parts;
            s.band_G = band_R * g.parts;
            // three workgroups per CU for the low-j steps: 1.5x the line ranges (>= 2 lines each)
            const int64_t R3 = std::min<int64_t>({std::max<int64_t>(1, 3LL * (c->n_cu > 0 ? c->n_cu : 256) / g.parts),
                                                  g.lines / 2, (int64_t)GMAX / g.parts});
            s.band_G3 = (int)R3 * g.parts;
        }
    }
    // every rank takes the same path: the band step exchanges ghost lines with its neighbours
    // each step, so one rank falling back alone would leave its peers' sends unmatched.  The
    // agreement (an all-reduce and a host sync) is needed only when some rank could take the band:
    // the inputs below are the same on every rank (band_L is set on all ranks or none; the
    // orthogonalisation, the switch, the preconditioner and restart are the callers' uniform
    // arguments), the rest (layout, geometry) is rank-local
    const bool band_possible = dc && c->tune.band && A->band_L > 0 && M && M->kind == VTK_PREC_BJACOBI && M->bs == 8 &&
                               m >= 2 && m <= 20;
    if (c->dist && band_possible) {
        double mine = s.band ? 0.0 : 1.0;
        HIPCHK(c, hipMemcpyAsync(&c->d_scal[DC_NQ + 2], &mine, sizeof(double), hipMemcpyHostToDevice, c->stream));
        TRY(comm_allreduce(c, &c->d_scal[DC_NQ + 2], 1));
        double off = 0.0;
        HIPCHK(c, hipMemcpyAsync(&off, &c->d_scal[DC_NQ + 2], sizeof(double), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (off != 0.0) s.band = false;
    }
    // band: the third w buffer, the ghost lines [2][m+2][L] and the send / receive pieces
    const size_t nghost = (s.band && A->band_ghost)
                              ? (size_t)2 * (m + 2) * A->band_L + 4 * (size_t)BAND_GHOST_VECS * A->band_L : 0;
    const size_t nedge = s.band ? (size_t)s.ld + nghost : 0;
    const size_t nd = (size_t)(m + 1) * s.ld + 3 * (size_t)s.ld + (size_t)m * (m + 1) + (m + 1) + 2 * m + 64 + ndc + nedge + 16;
    if (c->ws_bytes < nd * sizeof(double)) {
        if (c->ws) (void)hipFree(c->ws);
        c->ws = nullptr;
        c->ws_bytes = 0;
        HIPCHK(c, hipMalloc(&c->ws, nd * sizeof(double)));
        c->ws_bytes = nd * sizeof(double);
    }
    double *wp = static_cast<double *>(c->ws);
    s.V = wp; wp += (size_t)(m + 1) * s.ld;
    s.w = wp; wp += s.ld;
    s.tmp = wp; wp += s.ld;
    s.r = wp; wp += s.ld;
    s.H = wp; wp += (size_t)m * (m + 1);
    s.S = wp; wp += m + 1;
    s.giv = wp; wp += 2 * m;
    if (dc) {
        wp = reinterpret_cast<double *>((reinterpret_cast<uintptr_t>(wp) + 63) & ~(uintptr_t)63);
        s.dcpart = wp; wp += (size_t)DC_NQ * GMAX;
        s.Hraw = wp; wp += (size_t)(m + 1) * (m + 1);
        s.cf = reinterpret_cast<DcCoef *>(wp);
        wp += sizeof(DcCoef) / 8 + 8;
        HIPCHK(c, hipMemsetAsync(s.Hraw, 0, (size_t)(m + 1) * (m + 1) * sizeof(double), c->stream));
    }
    if (s.band) {
        wp = reinterpret_cast<double *>((reinterpret_cast<uintptr_t>(wp) + 63) & ~(uintptr_t)63);
        s.w3 = wp;
        if (A->band_ghost) {
            s.ghost = wp + s.ld;
            s.gsend = s.ghost + (size_t)2 * (m + 2) * A->band_L;
            s.grecv = s.gsend + 2 * (size_t)BAND_GHOST_VECS * A->band_L;
        }
        wp += nedge;
    }
    HIPCHK(c, hipMemsetAsync(s.H, 0, (size_t)m * (m + 1) * sizeof(double), c->stream));
    HIPCHK(c, hipMemsetAsync(s.giv, 0, (size_t)2 * m * sizeof(double), c->stream));
    GmresState *ds = c->d_state, *hs = c->h_state;
    std::memset(hs, 0, sizeof(GmresState));
    hs->stop_col = BIG_COL;
    hs->xup_tag = -1;
    HIPCHK(c, hipMemcpyAsync(ds, hs, sizeof(GmresState), hipMemcpyHostToDevice, c->stream));
    if (c->dist) HIPCHK(c, hipMemsetAsync(&c->d_scal[DC_VOTE + 1], 0, sizeof(double), c->stream));   // no failure yet
    s.fail_pending = c->tune.fail_step >= 0;
    int rc;
    const double n8 = 8.0 * n;
    const double b_pc = bj_row_bytes(M) * n + 2 * n8;
    // ||b|| and ||M b|| (iterative.py:708, :714)
    { Prof pf(c, "dot", -1, n8);
      HIPCHK(c, launch_dot(b, nullptr, n, s.part[0], s.G, c->stream)); }
    Red rb = reduce(c, s.part[0], s.G, rc);
    TRY(rc);
    HIPCHK(c, launch_finalize(rb, &ds->scal[0], 1, c->stream));
    // M b goes to V[0]: with x0 = 0 it is the first cycle's psolve(r) (below)
    { Prof pf(c, prec_cls(M), -1, b_pc);
      HIPCHK(c, launch_bj_apply(bj_op(M), n, b, s.V, nullptr, s.part[1], nullptr, s.G, nullptr, 0, c->stream)); }
    Red rmb = reduce(c, s.part[1], s.G, rc);
    TRY(rc);
    HIPCHK(c, launch_finalize(rmb, &ds->scal[1], 1, c->stream));
    // `r = b - matvec(x) if x.any() else b.copy()` (iterative.py:737): any nonzero x0 on any rank
    HIPCHK(c, hipMemsetAsync(&ds->scal[2], 0, sizeof(double), c->stream));
    { Prof pf(c, "any", -1, n8);
      HIPCHK(c, launch_any_nonzero(x, n, &ds->scal[2], c->stream)); }
    if (c->dist) TRY(comm_allreduce(c, &ds->scal[2], 1));
    double x_any = 0.0;
    HIPCHK(c, hipMemcpyAsync(&x_any, &ds->scal[2], sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const bool r_is_b = x_any == 0.0;
    // r = b - A x (iterative.py:737, :816).  When the BJ tiles allow (or M is the identity) the
    // residual kernel also applies M^-1 and writes v0's direction straight into V[0]: the next
    // cycle's psolve(r) (:742) is then already done.
    const bool fres = !M || bj_fused(M);
    const Tiles *rtiles = (M && bj_fused(M)) ? &M->tiles : &A->tiles;
    const SpmvIn rin0 = spmv_in(A, rtiles, x), pin0 = spmv_in(A, &A->tiles, x);
    double *prr = c->d_part + 4 * GMAX, *prz = c->d_part + 5 * GMAX;
    Red rz{prz, spmv_grid(rin0)};
    auto residual = [&]() -> int {
        TRY(halo_exchange(A, x));
        int rc2;
        Red rr;
        if (fres && M && g4_resid_ok(c, A, M)) {   // 4D grid rows: through k_g4_ring
            Prof pf(c, "spmv_resid_bj", -1, solver_matrix_bytes(A) + bj_row_bytes(M) * n + 3 * n8);
            G4Dots dd;
            dd.mode = 3;
            dd.b = b;
            dd.p0 = prr;
            dd.p1 = prz;
            int g = 0;
            SOFT(launch_g4_ring(A->g4, x, A->g4.lblk >= 0 ? A->d_halo : nullptr, M->d_tri + M->tri_ld, s.V, n, A->fp32,
                                     c->tune.g4_ring, c->tune.g4_gr, &dd, &g, nullptr,
                                     0, c->stream, 0, -1, 0, c->tune.g4_fast));
            TRY(pad_partials(c, prr, prz, g));
            rr = reduce(c, prr, g, rc2);
            TRY(rc2);
            rz = reduce(c, prz, g, rc2);
            TRY(rc2);
        } else if (fres && M && cyc_ring_ok(c, A, M, true)) {   // the same through the x-line ring
            Prof pf(c, "spmv_resid_bj", -1, solver_matrix_bytes(A) + bj_row_bytes(M) * n + 3 * n8);
            int g = 0;
            SOFT(launch_lsv_ring_epi(EPI_RESID_PREC, A->d_lsv, x, b, M->d_tri + M->tri_ld, s.V, prr, prz, nullptr,
                                          n, (int)A->band_L, c->tune.cyc_ring, nullptr, 0, &g, c->stream,
                                          A->band_ghost ? A->d_halo : nullptr, A->band_lblk, A->band_xord));
            TRY(pad_partials(c, prr, prz, g));
            rr = reduce(c, prr, g, rc2);
            TRY(rc2);
            rz = reduce(c, prz, g, rc2);
            TRY(rc2);
        } else if (fres) {
            Prof pf(c, "spmv_resid_bj", -1, solver_matrix_bytes(A) + bj_row_bytes(M) * n + 3 * n8);
            SOFT(launch_spmv(lsv_in(spmv_in(A, rtiles, x), A), EPI_RESID_PREC, s.V, b, bj_op(M),
                                  nullptr, prr, prz, nullptr, 0, c->stream));
            rr = reduce(c, prr, spmv_grid(rin0), rc2);
            TRY(rc2);
            rz = reduce(c, prz, spmv_grid(rin0), rc2);
            TRY(rc2);
        } else if (cyc_ring_ok(c, A, M, false)) {
            Prof pf(c, "spmv_resid", -1, solver_matrix_bytes(A) + 3 * n8);
            int g = 0;
            SOFT(launch_lsv_ring_epi(EPI_RESID, A->d_lsv, x, b, nullptr, s.r, prr, nullptr, nullptr, n,
                                          (int)A->band_L, c->tune.cyc_ring, nullptr, 0, &g, c->stream,
                                          A->band_ghost ? A->d_halo : nullptr, A->band_lblk, A->band_xord));
            TRY(pad_partials(c, prr, nullptr, g));
            rr = reduce(c, prr, g, rc2);
            TRY(rc2);
        } else {
            Prof pf(c, "spmv_resid", -1, solver_matrix_bytes(A) + 3 * n8);
            SOFT(launch_spmv(lsv_in(spmv_in(A, &A->tiles, x), A), EPI_RESID, s.r, b, BjOp{}, nullptr, prr, nullptr, nullptr, 0, c->stream));
            rr = reduce(c, prr, spmv_grid(pin0), rc2);
            TRY(rc2);
        }
        HIPCHK(c, launch_finalize(rr, &ds->rnorm, 1, c->stream));
        return VTK_OK;
    };
    if (r_is_b) {
        // r = b: ||r|| = ||b||, and psolve(r) = M b is already in V[0] with its partials
        HIPCHK(c, hipMemcpyAsync(&ds->rnorm, &ds->scal[0], sizeof(double), hipMemcpyDeviceToDevice, c->stream));
        rz = Red{s.part[1], s.G};
    } else {
        TRY(residual());
    }
    HIPCHK(c, hipMemcpyAsync(hs, ds, sizeof(GmresState), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const double bnrm2 = hs->scal[0], Mb_nrm2 = hs->scal[1];
    const double eps = 2.220446049250313e-16;
    atol = std::max(atol, rtol * bnrm2);                    // _get_atol_rtol :19
    vtk_stats st{};
    st.bnorm = bnrm2;
    st.atol_eff = atol;
    st.orth = dc ? VTK_ORTH_DCGS2 : VTK_ORTH_MGS;
    st.band = s.band ? 1 : 0;
    auto done = [&](int inf) {
        *info = inf;
        st.t_solve = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (stout) *stout = st;
        return VTK_OK;
    };
    if (bnrm2 == 0.0) {                                     // :712-713 -> x = b
        HIPCHK(c, hipMemcpyAsync(x, b, n * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        return done(0);
    }
    double rnorm = hs->rnorm;
    if (rnorm < atol) { st.rnorm = rnorm; return done(0); }   // :738-739
    double ptol_max_factor = 1.0;
    double ptol = Mb_nrm2 * std::min(ptol_max_factor, atol / bnrm2);   // :723
    double presid = 0.0;
    const double bytes_spmv = matrix_bytes(A) + 16.0 * n;
    const double bytes_pc = bj_row_bytes(M) * n + 16.0 * n;
    hipEvent_t ev[LOOKAHEAD + 1];
    for (auto &e : ev) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    struct EvGuard { hipEvent_t *e; ~EvGuard() { for (int i = 0; i <= LOOKAHEAD; ++i) (void)hipEventDestroy(e[i]); } } eg{ev};
    volatile int *mirror = c->h_stop;
    int64_t it = 0;
    bool brk = false;
    for (it = 0; it < maxiter; ++it) {
        // cycle start: v0 = M^-1 r / ||M^-1 r||, S = [tmp, 0, ...] (:742-748)
        hs->ptol = ptol;
        HIPCHK(c, hipMemcpyAsync(&ds->ptol, &hs->ptol, sizeof(double), hipMemcpyHostToDevice, c->stream));
        Red rv = rz;
        if (!fres && !(it == 0 && r_is_b)) {
            { Prof pf(c, prec_cls(M), -1, b_pc);
              SOFT(launch_bj_apply(bj_op(M), n, s.r, s.V, nullptr, s.part[0], nullptr, s.G, nullptr, 0, c->stream)); }
            rv = reduce(c, s.part[0], s.G, rc);
            TRY(rc);
        }
        { Prof pf(c, "scale0", -1, 2 * n8);
          SOFT(launch_scale0(rv, s.V, n, s.S, m, ds, s.G, c->stream)); }
        const int *stop = &ds->stop_col;
        *mirror = BIG_COL;
        int enq = 0;
        if (dc) {
            HIPCHK(c, hipMemsetAsync(s.cf->committed, 0, sizeof(s.cf->committed), c->stream));
            TRY(dcgs2_cycle(s, stop, mirror, ev));
        } else
        for (int col = 0; col < m; ++col) {
            double *vcol = s.V + (size_t)col * s.ld;
            Red h0, d0;
            TRY(precond_matvec(s, vcol, s.w, stop, col, h0, d0));
            Red cur = d0;
            for (int k = 0; k <= col; ++k) {
                double *po = s.part[2 + (k & 1)];
                const double *vn = k < col ? s.V + (size_t)(k + 1) * s.ld : nullptr;
                { Prof pf(c, "mgs", col, (vn ? 4 : 3) * n8);
                  SOFT(launch_mgs(cur, s.H + (size_t)col * (m + 1) + k, s.w, s.V + (size_t)k * s.ld, vn, n, po, s.G, stop, col, c->stream)); }
                cur = reduce(c, po, s.G, rc);
                TRY(rc);
            }
            { Prof pf(c, "tail", col, 2 * n8);
              SOFT(launch_tail(h0, cur, s.w, s.V + (size_t)(col + 1) * s.ld, n, col, m, s.H, s.S, s.giv, ds, c->d_stop, s.G, c->stream)); }
            HIPCHK(c, hipEventRecord(ev[col % (LOOKAHEAD + 1)], c->stream));
            enq = col + 1;
            if (col >= LOOKAHEAD) {
                HIPCHK(c, hipEventSynchronize(ev[(col - LOOKAHEAD) % (LOOKAHEAD + 1)]));
                // Act only on a stop at a column whose tail every rank has completed (it is
                // behind the event just synchronised): a later column's flag may already be
                // visible on one rank and not on another, and the ranks must enqueue the same
                // sequence of collectives.
                if (*mirror <= col - LOOKAHEAD) break;
            }
        }
        (void)enq;
        // x += y @ V[:col+1] (:799-814), r = b - A x, rnorm (:816-817)
        const size_t xup_idx = c->prof_pending.size();
        { Prof pf(c, "xupdate", -1, 0.0);   // bytes set once the stop column is known
          SOFT(launch_xupdate(s.H, s.S, s.V, s.ld, x, n, m, ds, s.G, c->stream)); }
        TRY(residual());
        // across ranks: the cycle's failure vote (a launch of some rank failed in this cycle; the
        // per-step vote has already stopped the Arnoldi steps at the same step on every rank)
        double vote = 0.0;
        if (c->dist) {
            TRY(comm_allreduce(c, &c->d_scal[DC_VOTE + 1], 1));
            HIPCHK(c, hipMemcpyAsync(&vote, &c->d_scal[DC_VOTE + 1], sizeof(double), hipMemcpyDeviceToHost, c->stream));
        }
        HIPCHK(c, hipMemcpyAsync(hs, ds, sizeof(GmresState), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (vote != 0.0) {
            prof_flush(c);
            if (s.local_rc != VTK_OK) return s.local_rc;
            return fail(c, VTK_ERR_PEER, "a peer rank failed in restart cycle " + std::to_string(it) +
                                             (hs->breakdown == PEER_FAILED ? " at Arnoldi step " + std::to_string(hs->stop_col + 1) : std::string()) +
                                             "; every rank left the solve there");
        }
        const int last = hs->stop_col < m ? hs->stop_col : m - 1;
        if (c->prof_on) {
            const double xb = n8 * (last + 1) + 2 * n8;   // V[0..last] (or V_last and p_last), x in/out
            if (xup_idx < c->prof_pending.size()) c->prof_pending[xup_idx].bytes = xb;
            if (hs->xup_tag >= 0) {
                // the x update ran in update pass xup_tag: account it as the "xupdate" class and
                // drop the host-enqueued k_xupdate (it returned at entry)
                const int cu = prof_class(c, "dc_update"), cb = prof_class(c, "band_step"), cx = prof_class(c, "xupdate");
                for (size_t i = 0; i < xup_idx && i < c->prof_pending.size(); ++i) {
                    auto &p = c->prof_pending[i];
                    if ((p.cls == cu || p.cls == cb) && p.col == hs->xup_tag) { p.cls = cx; p.col = -1; p.bytes = xb; }
                }
                if (xup_idx < c->prof_pending.size()) c->prof_pending[xup_idx].col = BIG_COL;
            }
            prof_flush(c, last);
        }
        for (int j = 0; j <= last; ++j) st.bytes_moved += bytes_spmv + bytes_pc + 8.0 * n * (2 * j + 8);
        st.bytes_moved += bytes_spmv + 24.0 * n + bytes_pc + 24.0 * n + 8.0 * n * (last + 2);
        rnorm = hs->rnorm;
        presid = hs->presid;
        brk = hs->breakdown != 0;
        st.restarts = it + 1;
        if (rnorm <= atol) break;                                                   // :824
        else if (brk) break;                                                        // :826
        else if (presid <= ptol) ptol_max_factor = std::max(eps, 0.25 * ptol_max_factor);   // :830
        else ptol_max_factor = std::min(1.0, 1.5 * ptol_max_factor);              // :833
        ptol = presid * std::min(ptol_max_factor, atol / rnorm);                    // :835
    }
    prof_flush(c);
    st.inner_iters = hs->inner;
    st.presid = presid;
    st.rnorm = rnorm;
    st.breakdown = brk ? 1 : 0;
    return done(rnorm <= atol ? 0 : (int)std::min<int64_t>(maxiter, INT32_MAX));   // :840
}

}  // namespace

extern "C" {

int vtk_last_error(vtk_ctx *ctx, char *buf, size_t len) {
    if (!buf || len == 0) return VTK_ERR_ARG;
    const std::string e = ctx ? ctx->err : context_free_error();
    std::snprintf(buf, len, "%s", e.c_str());
    return VTK_OK;
}

int vtk_device_count(int *count) {
    if (!count) return VTK_ERR_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return VTK_OK;
}

int vtk_ctx_create(int device, vtk_ctx **out) {
    if (!out) return fail(nullptr, VTK_ERR_ARG, "vtk_ctx_create: out is NULL");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        return fail(nullptr, VTK_ERR_NODEVICE, "vtk_ctx_create: no HIP device visible (the product has no CPU fallback)");
    if (device < 0 || device >= n) return fail(nullptr, VTK_ERR_ARG, "vtk_ctx_create: bad device ordinal");
    auto *c = new vtk_ctx();
    c->device = device;
    tune_from_env(c->tune);   // the only place the library reads its environment
    auto bad = [&](hipError_t e) {
        set_context_free_error(std::string("vtk_ctx_create: ") + hipGetErrorString(e));
        vtk_ctx_destroy(c);
        return e == hipErrorOutOfMemory ? VTK_ERR_NOMEM : VTK_ERR_HIP;
    };
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return bad(e);
    if ((e = hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device)) != hipSuccess) return bad(e);
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) return bad(e);
    if ((e = hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking)) != hipSuccess) return bad(e);
    if ((e = hipEventCreateWithFlags(&c->ev_pack, hipEventDisableTiming)) != hipSuccess) return bad(e);
    if ((e = hipEventCreateWithFlags(&c->ev_halo, hipEventDisableTiming)) != hipSuccess) return bad(e);
    if ((e = hipMalloc(&c->d_part, 8 * GMAX * sizeof(double))) != hipSuccess) return bad(e);
    if ((e = hipMalloc(&c->d_scal, 256 * sizeof(double))) != hipSuccess) return bad(e);
    if ((e = hipMalloc(&c->d_state, sizeof(GmresState))) != hipSuccess) return bad(e);
    if ((e = hipHostMalloc(&c->h_state, sizeof(GmresState), hipHostMallocDefault)) != hipSuccess) return bad(e);
    if ((e = hipHostMalloc(&c->h_stop, 64, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess) return bad(e);
    if ((e = hipHostGetDevicePointer((void **)&c->d_stop, c->h_stop, 0)) != hipSuccess) return bad(e);
    *c->h_stop = BIG_COL;
    *out = c;
    return VTK_OK;
}

void vtk_ctx_destroy(vtk_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    // a communicator whose collective failed may have peers blocked in it: abort, do not destroy
    if (c->comm) (void)(c->comm_broken ? ncclCommAbort(c->comm) : ncclCommDestroy(c->comm));
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    prof_flush(c);
    for (auto e : c->prof_pool) (void)hipEventDestroy(e);
    (void)hipFree(c->d_part);
    (void)hipFree(c->d_scal);
    (void)hipFree(c->d_state);
    if (c->ws) (void)hipFree(c->ws);
    if (c->h_state) (void)hipHostFree(c->h_state);
    if (c->h_stop) (void)hipHostFree(c->h_stop);
    if (c->comm_stream) (void)hipStreamSynchronize(c->comm_stream);
    if (c->ev_pack) (void)hipEventDestroy(c->ev_pack);
    if (c->ev_halo) (void)hipEventDestroy(c->ev_halo);
    if (c->comm_stream) (void)hipStreamDestroy(c->comm_stream);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int vtk_ctx_stream(vtk_ctx *c, void **stream) {
    if (!c || !stream) return VTK_ERR_ARG;
    *stream = (void *)c->stream;
    return VTK_OK;
}

int vtk_ctx_synchronize(vtk_ctx *c) {
    if (!c) return VTK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VTK_OK;
}

int vtk_comm_unique_id(void *out128) {
    if (!out128) return fail(nullptr, VTK_ERR_ARG, "vtk_comm_unique_id: NULL");
    static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id is 128 bytes");
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return fail(nullptr, VTK_ERR_RCCL, ncclGetErrorString(r));
    std::memcpy(out128, &id, sizeof(id));
    return VTK_OK;
}

int vtk_comm_init(vtk_ctx *c, int rank, int world, const void *uid) {
    if (!c || world < 1 || rank < 0 || rank >= world) return fail(c, VTK_ERR_ARG, "vtk_comm_init: bad rank/world");
    HIPCHK(c, hipSetDevice(c->device));
    // world 1: no communicator, unless tuning comm_solo (VTK_COMM_SOLO=1) asks for a one-rank RCCL communicator
    // that runs every distributed code path (halo plan and exchange, all-reduces, split lists)
    const bool force = world == 1 && c->tune.comm_solo;
    if (world == 1 && !force) { c->rank = 0; c->world = 1; c->dist = false; return VTK_OK; }
    if (!uid) return fail(c, VTK_ERR_ARG, "vtk_comm_init: unique id required");
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof(id));
    NCCLCHK(c, ncclCommInitRank(&c->comm, world, id, rank));
    c->rank = rank;
    c->world = world;
    c->dist = true;
    return VTK_OK;
}

int vtk_comm_init_host(vtk_ctx *c, int rank, int world, const vtk_host_comm *ops) {
    if (!c || world < 1 || rank < 0 || rank >= world) return fail(c, VTK_ERR_ARG, "vtk_comm_init_host: bad rank/world");
    if (world > 1 && (!ops || !ops->allreduce_sum_f64 || !ops->alltoallv || !ops->allgather))
        return fail(c, VTK_ERR_ARG, "vtk_comm_init_host: all three hooks are required");
    if (c->comm) return fail(c, VTK_ERR_STATE, "vtk_comm_init_host: RCCL communicator already set");
    c->rank = rank;
    c->world = world;
    c->host_comm = world > 1;
    c->dist = world > 1;
    if (ops) c->hops = *ops;
    return VTK_OK;
}

int vtk_comm_info(vtk_ctx *c, int *rank, int *world) {
    if (!c || !rank || !world) return VTK_ERR_ARG;
    *rank = c->rank;
    *world = c->world;
    return VTK_OK;
}

int vtk_comm_rccl_count(vtk_ctx *c, int *count) {
    if (!c || !count) return VTK_ERR_ARG;
    *count = 0;
    if (c->comm) NCCLCHK(c, ncclCommCount(c->comm, count));
    return VTK_OK;
}

int vtk_csr_create(vtk_ctx *c, int64_t n_global, const int64_t *offsets, int64_t nnz,
                   const int32_t *indptr, const int32_t *indices, const void *data, int fp32,
                   int kind, vtk_csr **out) {
    if (!c || !out || n_global < 0 || nnz < 0 || !indptr || (nnz > 0 && (!indices || !data)))
        return fail(c, VTK_ERR_ARG, "vtk_csr_create: invalid arguments");
    if (nnz >= ((int64_t)1 << 31)) return fail(c, VTK_ERR_ARG, "vtk_csr_create: nnz must fit int32");
    *out = nullptr;
    HIPCHK(c, hipSetDevice(c->device));
    std::vector<int64_t> offs;
    TRY(check_partition(c, n_global, offsets, offs));
    auto *A = new vtk_csr();
    struct Guard { vtk_csr *&a; ~Guard() { if (a) destroy_csr(a); } } g{A};
    A->ctx = c;
    A->device = c->device;
    A->n_global = n_global;
    A->offsets = offs;
    A->row_begin = offs[c->rank];
    A->row_end = offs[c->rank + 1];
    A->n_local = A->row_end - A->row_begin;
    A->nnz = nnz;
    A->fp32 = fp32 ? 1 : 0;
    const int64_t nl = A->n_local;
    A->h_indptr.resize(nl + 1);
    const hipMemcpyKind k = kind == VTK_PTR_DEVICE ? hipMemcpyDeviceToHost : hipMemcpyHostToHost;
    HIPCHK(c, hipMemcpy(A->h_indptr.data(), indptr, (nl + 1) * sizeof(int32_t), k));
    if (A->h_indptr[0] != 0 || A->h_indptr[nl] != nnz) return fail(c, VTK_ERR_ARG, "vtk_csr_create: indptr must start at 0 and end at nnz");
    for (int64_t i = 0; i < nl; ++i)
        if (A->h_indptr[i + 1] < A->h_indptr[i]) return fail(c, VTK_ERR_ARG, "vtk_csr_create: indptr not monotone");
    if (kind == VTK_PTR_HOST) {
        for (int64_t kk = 0; kk < nnz; ++kk)
            if (indices[kk] < 0 || indices[kk] >= n_global) return fail(c, VTK_ERR_ARG, "vtk_csr_create: column index out of range");
    }
    const size_t vb = fp32 ? sizeof(float) : sizeof(double);
    HIPCHK(c, hipMalloc(&A->d_indptr, (nl + 1) * sizeof(int32_t)));
    HIPCHK(c, hipMalloc(&A->d_indices, std::max<int64_t>(nnz, 1) * sizeof(int32_t)));
    HIPCHK(c, hipMalloc(&A->d_data, std::max<int64_t>(nnz, 1) * vb));
    const hipMemcpyKind kd = kind == VTK_PTR_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    HIPCHK(c, hipMemcpy(A->d_indptr, A->h_indptr.data(), (nl + 1) * sizeof(int32_t), hipMemcpyHostToDevice));
    if (nnz) {
        HIPCHK(c, hipMemcpy(A->d_indices, indices, nnz * sizeof(int32_t), kd));
        HIPCHK(c, hipMemcpy(A->d_data, data, nnz * vb, kd));
        // device-to-device copies on the null stream: complete before the context's
        // (non-blocking) stream reads the arrays
        if (kind == VTK_PTR_DEVICE) HIPCHK(c, hipStreamSynchronize(nullptr));
    }
    if (kind == VTK_PTR_DEVICE && nnz) {   // device input: the same range check on the device
        DBuf mmb;
        TRY(dalloc(c, mmb, 2 * sizeof(int)));
        int mm[2] = {INT_MAX, INT_MIN};
        HIPCHK(c, hipMemcpy(mmb.p, mm, sizeof(mm), hipMemcpyHostToDevice));
        HIPCHK(c, launch_index_range(A->d_indices, nnz, mmb.as<int>(), c->stream));
        HIPCHK(c, hipMemcpyAsync(mm, mmb.p, sizeof(mm), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (mm[0] < 0 || (int64_t)mm[1] >= n_global)
            return fail(c, VTK_ERR_ARG, "vtk_csr_create: column index out of range");
    }
    TRY(finish_csr(A));
    // the drop-in path gets the fast solver too: the 2D / 4D Vlasov structure is found in the CSR
    TRY(auto_line_band(A));
    if (A->band_L == 0) TRY(auto_grid4(A));
    *out = A;
    A = nullptr;
    return VTK_OK;
}

int vtk_csr_create_vlasov(vtk_ctx *c, const vtk_vlasov_params *p, const int64_t *offsets, vtk_csr **out) {
    if (!c || !out || !vlasov_params_ok(p)) return fail(c, VTK_ERR_ARG, "vtk_csr_create_vlasov: invalid arguments");
    *out = nullptr;
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t N = vlasov_n(*p);
    if (vlasov_nnz(*p) >= ((int64_t)1 << 31)) return fail(c, VTK_ERR_ARG, "vtk_csr_create_vlasov: nnz must fit int32");
    std::vector<int64_t> offs;
    TRY(check_partition(c, N, offsets, offs));
    auto *A = new vtk_csr();
    struct Guard { vtk_csr *&a; ~Guard() { if (a) destroy_csr(a); } } g{A};
    A->ctx = c;
    A->device = c->device;
    A->n_global = N;
    A->offsets = offs;
    A->row_begin = offs[c->rank];
    A->row_end = offs[c->rank + 1];
    A->n_local = A->row_end - A->row_begin;
    A->fp32 = p->fp32 ? 1 : 0;
    const int64_t nl = A->n_local;
    HIPCHK(c, hipMalloc(&A->d_indptr, (nl + 1) * sizeof(int32_t)));
    HIPCHK(c, launch_vlasov_counts(*p, A->row_begin, nl, A->d_indptr, c->stream));
    size_t tb = 0;
    HIPCHK(c, launch_exclusive_scan(nullptr, nullptr, nl + 1, nullptr, &tb, c->stream));
    DBuf tmp, cnt;
    TRY(dalloc(c, tmp, tb));
    TRY(dalloc(c, cnt, (nl + 1) * sizeof(int32_t)));
    HIPCHK(c, hipMemcpyAsync(cnt.p, A->d_indptr, (nl + 1) * sizeof(int32_t), hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, launch_exclusive_scan(cnt.as<int32_t>(), A->d_indptr, nl + 1, tmp.p, &tb, c->stream));
    A->h_indptr.resize(nl + 1);
    HIPCHK(c, hipMemcpyAsync(A->h_indptr.data(), A->d_indptr, (nl + 1) * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    A->nnz = A->h_indptr[nl];
    const size_t vb = A->fp32 ? sizeof(float) : sizeof(double);
    HIPCHK(c, hipMalloc(&A->d_indices, std::max<int64_t>(A->nnz, 1) * sizeof(int32_t)));
    HIPCHK(c, hipMalloc(&A->d_data, std::max<int64_t>(A->nnz, 1) * vb));
    HIPCHK(c, launch_vlasov_fill(*p, A->row_begin, nl, A->d_indptr, A->d_indices, A->d_data, c->stream));
    TRY(finish_csr(A));
    // the 2D operator's rows form x-lines of Nv rows coupled to the neighbouring lines only
    if (p->dim == 2) {
        const int brc = band_check_all(A, p->shape[1]);
        if (brc == VTK_OK) A->band_L = p->shape[1];
        else if (brc != VTK_ERR_ARG) return brc;
    }
    // the 4D operator's rows are grid rows (couplings by one coordinate each)
    if (p->dim == 4) {
        const int grc = grid4_set(A, p->shape[1], p->shape[2], p->shape[3]);
        if (grc != VTK_OK && grc != VTK_ERR_ARG) return grc;
    }
    *out = A;
    A = nullptr;
    return VTK_OK;
}

int vtk_csr_info(vtk_csr *A, int64_t *n_global, int64_t *row_begin, int64_t *row_end, int64_t *nnz, int64_t *n_halo) {
    if (!A) return VTK_ERR_ARG;
    if (n_global) *n_global = A->n_global;
    if (row_begin) *row_begin = A->row_begin;
    if (row_end) *row_end = A->row_end;
    if (nnz) *nnz = A->nnz;
    if (n_halo) *n_halo = A->n_halo;
    return VTK_OK;
}

int vtk_csr_download(vtk_csr *A, int32_t *indptr, int32_t *indices, void *data) {
    if (!A || !indptr || (A->nnz && (!indices || !data))) return VTK_ERR_ARG;
    vtk_ctx *c = A->ctx;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::memcpy(indptr, A->h_indptr.data(), A->h_indptr.size() * sizeof(int32_t));
    if (!A->nnz) return VTK_OK;
    HIPCHK(c, hipMemcpy(indices, A->d_indices, A->nnz * sizeof(int32_t), hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(data, A->d_data, A->nnz * (A->fp32 ? sizeof(float) : sizeof(double)), hipMemcpyDeviceToHost));
    for (int64_t k = 0; k < A->nnz; ++k) {
        const int64_t l = indices[k];
        indices[k] = (int32_t)(l < A->n_local ? l + A->row_begin : A->halo_cols[l - A->n_local]);
    }
    return VTK_OK;
}

void vtk_csr_destroy(vtk_csr *A) { destroy_csr(A); }

// host <-> device staging for the *_HOST forms
struct Staged {
    vtk_ctx *c;
    DBuf buf;
    double *d = nullptr;
};

static int stage_in(vtk_ctx *c, const double *src, int64_t n, int kind, Staged &s) {
    s.c = c;
    if (kind == VTK_PTR_DEVICE) { s.d = const_cast<double *>(src); return VTK_OK; }
    TRY(dalloc(c, s.buf, std::max<int64_t>(n, 1) * sizeof(double)));
    s.d = s.buf.as<double>();
    if (n && src) HIPCHK(c, hipMemcpyAsync(s.d, src, n * sizeof(double), hipMemcpyHostToDevice, c->stream));
    return VTK_OK;
}

int vtk_spmv(vtk_csr *A, const double *x, double *y, int kind) {
    if (!A || !x || !y) return VTK_ERR_ARG;
    vtk_ctx *c = A->ctx;
    HIPCHK(c, hipSetDevice(c->device));
    Staged sx, sy;
    TRY(stage_in(c, x, A->n_local, kind, sx));
    TRY(stage_in(c, kind == VTK_PTR_DEVICE ? y : nullptr, A->n_local, kind, sy));
    TRY(halo_exchange(A, sx.d));
    {
        Prof pf(c, "spmv", -1, matrix_bytes(A) + 16.0 * A->n_local);
        HIPCHK(c, launch_spmv(spmv_in(A, &A->tiles, sx.d), EPI_PLAIN, sy.d, nullptr, BjOp{}, nullptr, nullptr, nullptr, nullptr, 0, c->stream));
    }
    if (c->prof_on) prof_flush(c);
    if (kind == VTK_PTR_HOST) {
        HIPCHK(c, hipMemcpyAsync(y, sy.d, A->n_local * sizeof(double), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return VTK_OK;
}

int vtk_bjacobi_create(vtk_csr *A, int bs, vtk_prec **out) { return vtk_bjacobi_create_ex(A, bs, VTK_BJ_SETUP_EXACT, out); }

int vtk_bjacobi_create_ex(vtk_csr *A, int bs, int setup, vtk_prec **out) {
    if (!A || !out || bs < 1 || bs > 64) return fail(A ? A->ctx : nullptr, VTK_ERR_ARG, "vtk_bjacobi_create: block size must be in [1, 64]");
    if (setup != VTK_BJ_SETUP_EXACT && setup != VTK_BJ_SETUP_MFMA && setup != VTK_BJ_SETUP_AUTO)
        return fail(A->ctx, VTK_ERR_ARG, "vtk_bjacobi_create_ex: unknown setup");
    if (setup == VTK_BJ_SETUP_AUTO) setup = (bs == 16 || bs == 32) ? VTK_BJ_SETUP_MFMA : VTK_BJ_SETUP_EXACT;
    if (setup == VTK_BJ_SETUP_MFMA && bs != 16 && bs != 32)
        return fail(A->ctx, VTK_ERR_ARG, "vtk_bjacobi_create_ex: the MFMA setup takes bs 16 or 32");
    vtk_ctx *c = A->ctx;
    *out = nullptr;
    HIPCHK(c, hipSetDevice(c->device));
    if (A->row_begin % bs != 0) return fail(c, VTK_ERR_ARG, "vtk_bjacobi_create: rank row block must start at a multiple of the block size");
    auto *M = new vtk_prec();
    struct Guard { vtk_prec *&m; ~Guard() { if (m) vtk_prec_destroy(m); } } g{M};
    M->A = A;
    M->device = c->device;
    M->bs = bs;
    M->nb = (A->n_local + bs - 1) / bs;
    HIPCHK(c, hipMalloc(&M->d_inv, std::max<int64_t>(M->nb, 1) * bs * bs * sizeof(double)));
    DBuf sing, work;
    TRY(dalloc(c, sing, sizeof(int)));
    const bool pow2 = (bs & (bs - 1)) == 0 && bs <= 32;
    if (!pow2) TRY(dalloc(c, work, std::max<int64_t>(M->nb, 1) * bs * bs * sizeof(double)));
    const int init = INT32_MAX;
    HIPCHK(c, hipMemcpyAsync(sing.p, &init, sizeof(int), hipMemcpyHostToDevice, c->stream));
    {
        Prof pf(c, setup == VTK_BJ_SETUP_MFMA ? "bj_setup_mfma" : "bj_setup", -1,
                (double)M->nb * bs * bs * 8.0 + matrix_bytes(A));
        if (setup == VTK_BJ_SETUP_MFMA)
            HIPCHK(c, launch_bj_setup_mfma(A->d_indptr, A->d_indices, A->d_data, A->fp32, A->n_local, bs, M->d_inv,
                                           sing.as<int>(), c->stream));
        else
            HIPCHK(c, launch_bj_setup(A->d_indptr, A->d_indices, A->d_data, A->fp32, A->n_local, bs, M->d_inv,
                                      sing.as<int>(), work.as<double>(), c->stream));
    }
    prof_flush(c);
    int sb = 0;
    HIPCHK(c, hipMemcpyAsync(&sb, sing.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (sb != INT32_MAX) return fail(c, VTK_ERR_SINGULAR, "vtk_bjacobi_create: singular diagonal block " + std::to_string(sb + A->row_begin / bs));
    if (bs == 2 || bs == 4 || bs == 8) {
        // tridiagonal blocks (the v-direction coupling of the Vlasov operators): LU factors
        M->tri_ld = std::max<int64_t>(M->nb, 1) * bs;
        HIPCHK(c, hipMalloc(&M->d_tri, 3 * M->tri_ld * sizeof(double)));
        DBuf flags;
        TRY(dalloc(c, flags, sizeof(int)));
        HIPCHK(c, hipMemsetAsync(flags.p, 0, sizeof(int), c->stream));
        HIPCHK(c, launch_bj_tri_setup(A->d_indptr, A->d_indices, A->d_data, A->fp32, A->n_local, bs, M->d_inv,
                                      M->d_tri, M->tri_ld, flags.as<int>(), c->stream));
        int fl = 0;
        HIPCHK(c, hipMemcpyAsync(&fl, flags.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        M->tri_ok = fl == 0;
        if (!M->tri_ok) {
            (void)hipFree(M->d_tri);
            M->d_tri = nullptr;
        }
    }
    if (pow2) {
        std::vector<int32_t> rows;
        TRY(upload_tiles(c, A->h_indptr, bs, M->tiles, &rows));
        M->fused = M->tiles.aligned && !M->tiles.has_long;
        if (M->fused && c->dist && A->row_halo.size() == (size_t)A->n_local) {
            TRY(upload_split_tiles(c, rows, A->row_halo, M->tiles, M->tiles_in, M->tiles_bd));
            M->split = true;
        }
    }
    *out = M;
    M = nullptr;
    return VTK_OK;
}

int vtk_linejacobi_create(vtk_csr *A, int64_t stride, int64_t seg, vtk_prec **out) {
    if (!A || !out) return VTK_ERR_ARG;
    vtk_ctx *c = A->ctx;
    *out = nullptr;
    if (stride < 1 || seg < 1) return fail(c, VTK_ERR_ARG, "vtk_linejacobi_create: stride and seg must be >= 1");
    if (A->n_global > 0 && stride >= A->n_global && A->n_global > 1)
        return fail(c, VTK_ERR_ARG, "vtk_linejacobi_create: stride must be below n (no line has two rows)");
    HIPCHK(c, hipSetDevice(c->device));
    auto *M = new vtk_prec();
    struct Guard { vtk_prec *&m; ~Guard() { if (m) vtk_prec_destroy(m); } } g{M};
    M->A = A;
    M->device = c->device;
    M->kind = VTK_PREC_LINE;
    M->bs = 0;
    M->line = line_plan(A->n_local, A->row_begin, stride, seg);
    HIPCHK(c, hipMalloc(&M->line.f, 3 * std::max<int64_t>(A->n_local, 1) * sizeof(double)));
    DBuf bad, ext;
    const int64_t jn = M->line.jn;
    TRY(dalloc(c, bad, sizeof(unsigned long long)));
    TRY(dalloc(c, ext, 4 * std::max<int64_t>(jn, 1) * sizeof(unsigned long long)));
    const unsigned long long none = ~0ull;
    std::vector<unsigned long long> hx(4 * (size_t)jn);
    for (int64_t j = 0; j < jn; ++j) {   // min | max | min | max
        hx[j] = none; hx[jn + j] = 0; hx[2 * jn + j] = none; hx[3 * jn + j] = 0;
    }
    HIPCHK(c, hipMemcpyAsync(bad.p, &none, sizeof(none), hipMemcpyHostToDevice, c->stream));
    if (jn) HIPCHK(c, hipMemcpyAsync(ext.p, hx.data(), hx.size() * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, launch_line_setup(A->d_indptr, A->d_indices, A->d_data, A->fp32, M->line,
                                bad.as<unsigned long long>(), ext.as<unsigned long long>(), c->stream));
    unsigned long long br = none;
    HIPCHK(c, hipMemcpyAsync(&br, bad.p, sizeof(br), hipMemcpyDeviceToHost, c->stream));
    if (jn) HIPCHK(c, hipMemcpyAsync(hx.data(), ext.p, hx.size() * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (br != none) return fail(c, VTK_ERR_SINGULAR, "vtk_linejacobi_create: zero or non-finite line pivot at row " + std::to_string(br));
    // x-invariant couplings (every line's a's bit-equal, likewise its c's): the apply forms l and
    // g from a_j, c_j and m (16 B/row read instead of 32); lines without any a (c) take 0
    bool inv = jn > 0;
    std::vector<double> ac(2 * (size_t)std::max<int64_t>(jn, 1), 0.0);
    for (int64_t j = 0; j < jn && inv; ++j) {
        for (int w = 0; w < 2; ++w) {
            const unsigned long long lo = hx[2 * w * jn + j], hi = hx[(2 * w + 1) * jn + j];
            if (lo > hi) continue;   // no row of this line has the coupling
            if (lo != hi) { inv = false; break; }
            std::memcpy(&ac[w * jn + j], &lo, 8);
        }
    }
    if (inv) {
        HIPCHK(c, hipMalloc(&M->line.ac, ac.size() * sizeof(double)));
        HIPCHK(c, hipMemcpy(M->line.ac, ac.data(), ac.size() * sizeof(double), hipMemcpyHostToDevice));
        M->line.compact = 1;
    }
    M->line_compact_ok = inv;
    *out = M;
    M = nullptr;
    return VTK_OK;
}

int vtk_linejacobi_factors(vtk_prec *M, double *f, int kind) {
    if (!M || !f) return VTK_ERR_ARG;
    vtk_ctx *c = M->A->ctx;
    if (M->kind != VTK_PREC_LINE) return fail(c, VTK_ERR_STATE, "vtk_linejacobi_factors: not a line-Jacobi preconditioner");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (M->line.n > 0)
        HIPCHK(c, hipMemcpy(f, M->line.f, 3 * M->line.n * sizeof(double), kind == VTK_PTR_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost));
    return VTK_OK;
}

int vtk_linejacobi_set_compact(vtk_prec *M, int on) {
    if (!M) return VTK_ERR_ARG;
    vtk_ctx *c = M->A->ctx;
    if (M->kind != VTK_PREC_LINE) return fail(c, VTK_ERR_STATE, "vtk_linejacobi_set_compact: not a line-Jacobi preconditioner");
    if (on && !M->line_compact_ok) return fail(c, VTK_ERR_ARG, "vtk_linejacobi_set_compact: the x-couplings are not constant along the lines");
    M->line.compact = on ? 1 : 0;
    return VTK_OK;
}

int vtk_linejacobi_get_compact(vtk_prec *M, int *in_use, int *available) {
    if (!M) return VTK_ERR_ARG;
    if (M->kind != VTK_PREC_LINE) return fail(M->A->ctx, VTK_ERR_STATE, "vtk_linejacobi_get_compact: not a line-Jacobi preconditioner");
    if (in_use) *in_use = M->line.compact;
    if (available) *available = M->line_compact_ok ? 1 : 0;
    return VTK_OK;
}

int vtk_prec_apply(vtk_prec *M, const double *r, double *z, int kind) { return vtk_bjacobi_apply(M, r, z, kind); }

// w = M^-1 A x through the launch the solver's split DCGS2 step uses for this operator (ADVICE r5:
// the kernel-level pin of k_g4_ring against k_sell<EPI_PREC>): the 4D ring kernel when it applies
// -- across ranks in the solver's form, interior groups while the halo planes travel, then the
// first / last planes' groups --, else the SELL / CSR SpMV with the BJ epilogue, else SpMV + apply
int vtk_precond_matvec(vtk_csr *A, vtk_prec *M, const double *x, double *w, int kind) {
    if (!A || !x || !w || (M && M->A != A)) return fail(A ? A->ctx : nullptr, VTK_ERR_ARG, "vtk_precond_matvec: bad arguments");
    vtk_ctx *c = A->ctx;
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t n = A->n_local;
    Staged sx, sw;
    TRY(stage_in(c, x, n, kind, sx));
    TRY(stage_in(c, kind == VTK_PTR_DEVICE ? w : nullptr, n, kind, sw));
    const bool ring = A->d_g4tab && c->tune.grid4 && c->tune.g4_ring > 0 && A->use_sell && M &&
                      M->kind == VTK_PREC_BJACOBI && M->bs == 8 && bj_op(M).tri != nullptr &&
                      g4_ring_fits(A->g4, n, c->tune.g4_gr);
    double *p0 = c->d_part, *p1 = c->d_part + GMAX;
    if (ring) {
        const double *halo = A->g4.lblk >= 0 ? A->d_halo : nullptr;
        const double *mt = M->d_tri + M->tri_ld;
        Prof pf(c, "spmv_bj", -1, solver_matrix_bytes(A) + bj_row_bytes(M) * n + 16.0 * n);
        if (!halo) {
            TRY(halo_exchange(A, sx.d));
            HIPCHK(c, launch_g4_ring(A->g4, sx.d, nullptr, mt, sw.d, n, A->fp32, c->tune.g4_ring, c->tune.g4_gr, nullptr,
                                     nullptr, nullptr, 0, c->stream, 0, -1, 0, c->tune.g4_fast));
        } else {   // dcgs2_cycle's split form (mode 0)
            const int G = g4_ring_group(c->tune.g4_gr);
            const int64_t S4 = (int64_t)A->g4.Ny * A->g4.Nvx * A->g4.Nvy, ng = (n + G - 1) / G;
            int64_t gi_lo = (S4 + G - 1) / G, gi_hi = (n - S4) / G;
            if (gi_hi <= gi_lo) gi_lo = gi_hi = 0;
            const int per = (int)g4_ring_per(ng, S4, G, std::max(1, c->tune.g4_ring));
            TRY(halo_exchange_async(A, sx.d));
            if (gi_hi > gi_lo)
                HIPCHK(c, launch_g4_ring(A->g4, sx.d, halo, mt, sw.d, n, A->fp32, c->tune.g4_ring, c->tune.g4_gr, nullptr,
                                         nullptr, nullptr, 0, c->stream, (int)gi_lo, (int)gi_hi, per, c->tune.g4_fast));
            HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_halo, 0));
            HIPCHK(c, launch_g4_ring(A->g4, sx.d, halo, mt, sw.d, n, A->fp32, c->tune.g4_ring, c->tune.g4_gr, nullptr,
                                     nullptr, nullptr, 0, c->stream, 0, (int)(gi_hi > gi_lo ? gi_lo : ng), per,
                                     c->tune.g4_fast));
            if (gi_hi > gi_lo)
                HIPCHK(c, launch_g4_ring(A->g4, sx.d, halo, mt, sw.d, n, A->fp32, c->tune.g4_ring, c->tune.g4_gr, nullptr,
                                         nullptr, nullptr, 0, c->stream, (int)gi_hi, (int)ng, per, c->tune.g4_fast));
        }
    } else if (line_fuse_ok(c, A, M)) {
        // the line step's form: y = A x formed inside the sweep kernel (k_line_spmv_dc; its step-0
        // dots go to a scratch), the ADVICE r5 pin of the fused kernel against SpMV + sweeps below
        DBuf part;
        TRY(dalloc(c, part, (size_t)DC_NQ * GMAX * sizeof(double)));
        Prof pf(c, "line_dc", -1, bj_row_bytes(M) * n + 24.0 * n);
        HIPCHK(c, launch_line_spmv_dc(M->line, A->d_lsv, sx.d, sw.d, sx.d, n, 0, part.as<double>(), vector_grid(n),
                                      nullptr, 0, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));   // part is freed on return
    } else if (!M || bj_fused(M)) {
        TRY(halo_exchange(A, sx.d));
        Prof pf(c, M ? "spmv_bj" : "spmv_w", -1, solver_matrix_bytes(A) + bj_row_bytes(M) * n + 16.0 * n);
        HIPCHK(c, launch_spmv(lsv_in(spmv_in(A, M ? &M->tiles : &A->tiles, sx.d), A), EPI_PREC, sw.d, nullptr,
                              M ? bj_op(M) : BjOp{}, nullptr, p0, p1, nullptr, 0, c->stream));
    } else {
        TRY(halo_exchange(A, sx.d));
        DBuf t;
        TRY(dalloc(c, t, std::max<int64_t>(n, 1) * sizeof(double)));
        HIPCHK(c, launch_spmv(lsv_in(spmv_in(A, &A->tiles, sx.d), A), EPI_PLAIN, t.as<double>(), nullptr, BjOp{}, nullptr,
                              nullptr, nullptr, nullptr, 0, c->stream));
        HIPCHK(c, launch_bj_apply(bj_op(M), n, t.as<double>(), sw.d, nullptr, nullptr, nullptr, vector_grid(n), nullptr, 0,
                                  c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));   // t is freed on return
    }
    if (c->prof_on) prof_flush(c);
    if (kind == VTK_PTR_HOST) {
        HIPCHK(c, hipMemcpyAsync(w, sw.d, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return VTK_OK;
}

int vtk_prec_kind_of(vtk_prec *M, int *kind) {
    if (!M || !kind) return VTK_ERR_ARG;
    *kind = M->kind;
    return VTK_OK;
}

int vtk_bjacobi_inverse(vtk_prec *M, double *inv, int kind) {
    if (!M || !inv) return VTK_ERR_ARG;
    vtk_ctx *c = M->A->ctx;
    if (M->kind != VTK_PREC_BJACOBI) return fail(c, VTK_ERR_STATE, "vtk_bjacobi_inverse: not a block-Jacobi preconditioner");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(inv, M->d_inv, M->nb * M->bs * M->bs * sizeof(double), kind == VTK_PTR_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost));
    return VTK_OK;
}

int vtk_bjacobi_apply(vtk_prec *M, const double *r, double *z, int kind) {
    if (!M || !r || !z) return VTK_ERR_ARG;
    vtk_ctx *c = M->A->ctx;
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t n = M->A->n_local;
    Staged sr, sz;
    TRY(stage_in(c, r, n, kind, sr));
    TRY(stage_in(c, kind == VTK_PTR_DEVICE ? z : nullptr, n, kind, sz));
    {
        Prof pf(c, M->kind == VTK_PREC_LINE ? "line_apply" : "bj_apply", -1, bj_row_bytes(M) * n + 16.0 * n);
        HIPCHK(c, launch_bj_apply(bj_op(M), n, sr.d, sz.d, nullptr, nullptr, nullptr, vector_grid(n), nullptr, 0, c->stream));
    }
    if (c->prof_on) prof_flush(c);
    if (kind == VTK_PTR_HOST) {
        HIPCHK(c, hipMemcpyAsync(z, sz.d, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return VTK_OK;
}

int vtk_csr_set_layout(vtk_csr *A, int layout) {
    if (!A) return VTK_ERR_ARG;
    vtk_ctx *c = A->ctx;
    if (layout != VTK_LAYOUT_AUTO && layout != VTK_LAYOUT_CSR && layout != VTK_LAYOUT_SELL &&
        layout != VTK_LAYOUT_SELL32)
        return fail(c, VTK_ERR_ARG, "vtk_csr_set_layout: unknown layout");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return apply_layout(A, layout);
}

int vtk_csr_get_layout(vtk_csr *A, int *layout_in_use) {
    if (!A || !layout_in_use) return VTK_ERR_ARG;
    *layout_in_use = A->use_sell ? (A->sell.d_pk ? VTK_LAYOUT_SELL : VTK_LAYOUT_SELL32) : VTK_LAYOUT_CSR;
    return VTK_OK;
}

int vtk_csr_layout_info(vtk_csr *A, vtk_layout_info *out) {
    if (!A || !out) return VTK_ERR_ARG;
    vtk_layout_info li{};
    int lay = VTK_LAYOUT_CSR;
    (void)vtk_csr_get_layout(A, &lay);
    li.layout = lay;
    li.matrix_bytes = matrix_bytes(A);
    li.sell_chunks = A->use_sell ? A->sell.nch : 0;
    li.sell_entries = A->use_sell ? A->sell.entries : 0;
    li.wide_chunks = A->use_sell && A->sell.d_pk ? A->sell.n_wide : 0;
    *out = li;
    return VTK_OK;
}

int vtk_bjacobi_set_mode(vtk_prec *M, int mode) {
    if (!M) return VTK_ERR_ARG;
    vtk_ctx *c = M->A->ctx;
    if (M->kind != VTK_PREC_BJACOBI) return fail(c, VTK_ERR_STATE, "vtk_bjacobi_set_mode: not a block-Jacobi preconditioner");
    if (mode != VTK_BJ_AUTO && mode != VTK_BJ_INVERSE && mode != VTK_BJ_TRIDIAG)
        return fail(c, VTK_ERR_ARG, "vtk_bjacobi_set_mode: unknown mode");
    if (mode == VTK_BJ_TRIDIAG && !M->tri_ok)
        return fail(c, VTK_ERR_ARG, "vtk_bjacobi_set_mode: blocks are not tridiagonal (bs 2/4/8) or their factors failed the check");
    M->mode = mode;
    return VTK_OK;
}

int vtk_bjacobi_get_mode(vtk_prec *M, int *mode_in_use, int *tridiag_available) {
    if (!M) return VTK_ERR_ARG;
    if (M->kind != VTK_PREC_BJACOBI) return fail(M->A->ctx, VTK_ERR_STATE, "vtk_bjacobi_get_mode: not a block-Jacobi preconditioner");
    if (mode_in_use) *mode_in_use = bj_op(M).tri ? VTK_BJ_TRIDIAG : VTK_BJ_INVERSE;
    if (tridiag_available) *tridiag_available = M->tri_ok ? 1 : 0;
    return VTK_OK;
}

void vtk_prec_destroy(vtk_prec *M) {
    if (!M) return;
    (void)hipSetDevice(M->device);
    (void)hipFree(M->d_inv);
    (void)hipFree(M->d_tri);
    (void)hipFree(M->line.f);
    (void)hipFree(M->line.ac);
    free_tiles(M->tiles);
    free_tiles(M->tiles_in);
    free_tiles(M->tiles_bd);
    delete M;
}

int vtk_csr_set_line_band(vtk_csr *A, int64_t line_len) {
    if (!A) return fail(nullptr, VTK_ERR_ARG, "vtk_csr_set_line_band: A is NULL");
    vtk_ctx *c = A->ctx;
    HIPCHK(c, hipSetDevice(c->device));
    if (line_len == 0) {
        A->band_L = 0;
        return VTK_OK;
    }
    const int rc = band_check_all(A, line_len);
    if (rc == VTK_ERR_ARG)
        return fail(c, VTK_ERR_ARG, "vtk_csr_set_line_band: not a line-band operator for this line length "
                                    "(line_len | n, >= 3 lines, every column in lines x-1..x+1, n + 2 line_len "
                                    "< 2^30; across ranks: slabs of whole lines whose halo is the two neighbour lines)");
    TRY(rc);
    A->band_L = line_len;
    return VTK_OK;
}

int vtk_csr_get_line_band(vtk_csr *A, int64_t *line_len) {
    if (!A || !line_len) return fail(A ? A->ctx : nullptr, VTK_ERR_ARG, "vtk_csr_get_line_band: NULL argument");
    *line_len = A->band_L;
    return VTK_OK;
}

int vtk_csr_set_grid4(vtk_csr *A, int64_t Ny, int64_t Nvx, int64_t Nvy) {
    if (!A) return fail(nullptr, VTK_ERR_ARG, "vtk_csr_set_grid4: A is NULL");
    vtk_ctx *c = A->ctx;
    HIPCHK(c, hipSetDevice(c->device));
    if (Ny == 0) {   // clear
        (void)hipFree(A->d_g4tab);
        (void)hipFree(A->d_g4D);
        A->d_g4tab = nullptr;
        A->d_g4D = nullptr;
        A->g4 = Grid4{};
        return VTK_OK;
    }
    const int rc = grid4_set(A, Ny, Nvx, Nvy);
    if (rc == VTK_ERR_ARG)
        return fail(c, VTK_ERR_ARG, "vtk_csr_set_grid4: not a 4D grid operator of these extents (rows = whole x planes "
                                    "of Ny*Nvx*Nvy rows, Ny >= 3, Nvx, Nvy >= 2, each row coupled to x+-1, y+-1, "
                                    "vx+-1, vy+-1 in ascending column order with values by one coordinate each)");
    return rc;
}

int vtk_csr_get_grid4(vtk_csr *A, int64_t *dims) {
    if (!A || !dims) return fail(A ? A->ctx : nullptr, VTK_ERR_ARG, "vtk_csr_get_grid4: NULL argument");
    dims[0] = A->d_g4tab ? A->g4.Ny : 0;
    dims[1] = A->d_g4tab ? A->g4.Nvx : 0;
    dims[2] = A->d_g4tab ? A->g4.Nvy : 0;
    return VTK_OK;
}

int vtk_csr_get_line_values(vtk_csr *A, int *separable) {
    if (!A || !separable) return fail(A ? A->ctx : nullptr, VTK_ERR_ARG, "vtk_csr_get_line_values: NULL argument");
    *separable = A->band_L > 0 && A->d_lsv != nullptr ? (A->lsv_canon ? 2 : 1) : 0;
    return VTK_OK;
}

int vtk_gmres_set_band(vtk_ctx *c, int on) {
    if (!c) return fail(nullptr, VTK_ERR_ARG, "vtk_gmres_set_band: ctx is NULL");
    c->tune.band = on != 0;
    return VTK_OK;
}

int vtk_ctx_set_tuning(vtk_ctx *c, const char *key, int value) {
    if (!c) return fail(nullptr, VTK_ERR_ARG, "vtk_ctx_set_tuning: ctx is NULL");
    const TuneKey *k = tune_key(key);
    if (!k) return fail(c, VTK_ERR_ARG, std::string("vtk_ctx_set_tuning: unknown key ") + (key ? key : "(null)"));
    c->tune.*k->mem = value;
    return VTK_OK;
}

int vtk_ctx_get_tuning(vtk_ctx *c, const char *key, int *value) {
    if (!c || !value) return fail(c, VTK_ERR_ARG, "vtk_ctx_get_tuning: NULL argument");
    const TuneKey *k = tune_key(key);
    if (!k) return fail(c, VTK_ERR_ARG, std::string("vtk_ctx_get_tuning: unknown key ") + (key ? key : "(null)"));
    *value = c->tune.*k->mem;
    return VTK_OK;
}

int vtk_gmres_set_orth(vtk_ctx *c, int orth) {
    if (!c || (orth != VTK_ORTH_MGS && orth != VTK_ORTH_DCGS2 && orth != VTK_ORTH_AUTO))
        return fail(c, VTK_ERR_ARG, "vtk_gmres_set_orth: unknown scheme");
    c->orth = orth;
    return VTK_OK;
}

int vtk_profile_enable(vtk_ctx *c, int on) {
    if (!c) return VTK_ERR_ARG;
    prof_flush(c);
    c->prof_on = on != 0;
    if (c->prof_on) c->prof_acc.clear();
    return VTK_OK;
}

int vtk_profile_read(vtk_ctx *c, vtk_kernel_profile *out, int max_entries, int *n_entries) {
    if (!c || !n_entries || (max_entries > 0 && !out)) return VTK_ERR_ARG;
    prof_flush(c);
    *n_entries = (int)c->prof_acc.size();
    for (int i = 0; i < max_entries && i < (int)c->prof_acc.size(); ++i) {
        const auto &a = c->prof_acc[i];
        std::snprintf(out[i].name, sizeof(out[i].name), "%s", a.name.c_str());
        out[i].launches = a.launches;
        out[i].seconds = a.seconds;
        out[i].bytes = a.bytes;
    }
    return VTK_OK;
}

int vtk_gmres(vtk_csr *A, vtk_prec *M, const double *b, double *x, double rtol, double atol,
              int restart, int64_t maxiter, int kind, int *info, vtk_stats *st) {
    if (!A || !b || !x || !info) return VTK_ERR_ARG;
    vtk_ctx *c = A->ctx;
    if (M && M->A != A) return fail(c, VTK_ERR_ARG, "vtk_gmres: preconditioner built for another operator");
    if (!(rtol >= 0.0) || !(atol >= 0.0)) return fail(c, VTK_ERR_ARG, "vtk_gmres: tolerances must be non-negative");
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t n = A->n_local;
    Staged sb, sx;
    TRY(stage_in(c, b, n, kind, sb));
    TRY(stage_in(c, x, n, kind, sx));
    TRY(run_gmres(A, M, sb.d, sx.d, rtol, atol, restart, maxiter, info, st));
    if (kind == VTK_PTR_HOST) {
        HIPCHK(c, hipMemcpyAsync(x, sx.d, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VTK_OK;
}

}  // extern "C"
