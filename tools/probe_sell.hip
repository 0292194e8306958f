// probe_sell.hip — SELL-64 (sliced ELL, one wavefront per 64-row chunk) vs the CSR-stream tiles
// on the C3 operator (2D Vlasov 25000 x 800, 20M rows, 100M nnz).  Each row's products are
// summed serially in stored order in both layouts, so y must be bit-identical.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/probe_sell.hip -o tools/bin/probe_sell
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../vt-precondition_amd/csrc/vtk_vlasov.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int NT = 256;
constexpr int TILE_ROWS = 512, TILE_NNZ = 4096;

__device__ __forceinline__ int xcd_swizzle(int b, int g) {
    constexpr int NX = 8;
    const int q = g / NX, r = g % NX, x = b % NX;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / NX;
}

// production CSR-stream (plain epilogue)
template <typename VT>
__global__ __launch_bounds__(NT) void k_stream(const int *__restrict__ indptr, const int *__restrict__ indices,
                                               const VT *__restrict__ data, const int *__restrict__ tile_row,
                                               int ntiles, const double *__restrict__ x, double *__restrict__ y) {
    __shared__ double prod[TILE_NNZ];
    __shared__ int rp[TILE_ROWS + 1];
    const int tid = threadIdx.x;
    for (int t = xcd_swizzle(blockIdx.x, gridDim.x); t < ntiles; t += gridDim.x) {
        const int r0 = tile_row[t], r1 = tile_row[t + 1], nr = r1 - r0;
        const int nz0 = indptr[r0], nnz = indptr[r1] - nz0;
        for (int i = tid; i <= nr; i += NT) rp[i] = indptr[r0 + i] - nz0;
        const int *ci = indices + nz0;
        const VT *cv = data + nz0;
        int e = tid;
        constexpr int U = 4;
        for (; e + (U - 1) * NT < nnz; e += U * NT) {
            int c[U];
            double d[U];
#pragma unroll
            for (int u = 0; u < U; ++u) { c[u] = ci[e + u * NT]; d[u] = (double)cv[e + u * NT]; }
#pragma unroll
            for (int u = 0; u < U; ++u) prod[e + u * NT] = d[u] * x[c[u]];
        }
        for (; e < nnz; e += NT) prod[e] = (double)cv[e] * x[ci[e]];
        __syncthreads();
        for (int base = 0; base < nr; base += NT) {
            const int i = base + tid;
            if (i < nr) {
                double s = 0.0;
                for (int k = rp[i]; k < rp[i + 1]; ++k) s += prod[k];
                y[r0 + i] = s;
            }
        }
        __syncthreads();
    }
}

// SELL-64: chunk q holds rows 64q..64q+63; entry k of row lane at off[q] + k*64 + lane; col -1 pads.
// W: entries loaded per batch (all loads of a batch issued before the gathers).
template <typename VT, int W, bool SWZ, bool NTL>
__global__ __launch_bounds__(NT) void k_sell(const long *__restrict__ off, const int *__restrict__ col,
                                             const VT *__restrict__ val, int nchunks, int n,
                                             const double *__restrict__ x, double *__restrict__ y) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int ngr = (nchunks + 3) / 4;
    const int b = SWZ ? xcd_swizzle(blockIdx.x, gridDim.x) : blockIdx.x;
    for (int g = b; g < ngr; g += gridDim.x) {
        const int q = 4 * g + wv;
        if (q >= nchunks) continue;
        const long o0 = off[q], o1 = off[q + 1];
        const int w = (int)((o1 - o0) >> 6);
        const int *cc = col + o0 + lane;
        const VT *vv = val + o0 + lane;
        double s = 0.0;
        for (int k0 = 0; k0 < w; k0 += W) {
            int c[W];
            double d[W];
#pragma unroll
            for (int u = 0; u < W; ++u) {
                const bool ok = k0 + u < w;
                if (NTL) {
                    c[u] = ok ? __builtin_nontemporal_load(cc + (k0 + u) * 64) : -1;
                    d[u] = ok ? (double)__builtin_nontemporal_load(vv + (k0 + u) * 64) : 0.0;
                } else {
                    c[u] = ok ? cc[(k0 + u) * 64] : -1;
                    d[u] = ok ? (double)vv[(k0 + u) * 64] : 0.0;
                }
            }
            double xv[W];
#pragma unroll
            for (int u = 0; u < W; ++u) xv[u] = c[u] >= 0 ? x[c[u]] : 0.0;
#pragma unroll
            for (int u = 0; u < W; ++u)
                if (c[u] >= 0) s += d[u] * xv[u];
        }
        const int r = q * 64 + lane;
        if (r < n) y[r] = s;
    }
}

__global__ void k_gen_counts(vtk_vlasov_params p, int n, int *cnt) {
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) cnt[r] = vtk::vlasov_row_count(p, r);
}
template <typename VT>
__global__ void k_gen_fill(vtk_vlasov_params p, int n, const int *indptr, int *ix, VT *d) {
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
        vtk::VlasovRow row;
        vtk::vlasov_row(p, r, row);
        for (int k = 0; k < row.count; ++k) { ix[indptr[r] + k] = (int)row.col[k]; d[indptr[r] + k] = (VT)row.val[k]; }
    }
}

template <typename VT>
int run(vtk_vlasov_params p) {
    const int n = (int)(p.shape[0] * p.shape[1] * (p.dim == 4 ? p.shape[2] * p.shape[3] : 1));
    std::vector<int> cnt(n), ip(n + 1);
    int *dcnt; CK(hipMalloc(&dcnt, n * 4));
    hipLaunchKernelGGL(k_gen_counts, dim3(2048), dim3(256), 0, 0, p, n, dcnt);
    CK(hipMemcpy(cnt.data(), dcnt, n * 4, hipMemcpyDeviceToHost));
    ip[0] = 0;
    for (int i = 0; i < n; ++i) ip[i + 1] = ip[i] + cnt[i];
    const int nnz = ip[n];
    int *dip, *dix; VT *dd; double *x, *y; char *junk;
    CK(hipMalloc(&dip, (n + 1) * 4)); CK(hipMalloc(&dix, (nnz + 16) * 4)); CK(hipMalloc(&dd, (size_t)(nnz + 16) * sizeof(VT)));
    CK(hipMalloc(&x, n * 8)); CK(hipMalloc(&y, n * 8)); CK(hipMalloc(&junk, 1L << 30));
    CK(hipMemcpy(dip, ip.data(), (n + 1) * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_gen_fill<VT>, dim3(2048), dim3(256), 0, 0, p, n, dip, dix, dd);
    std::vector<double> hx(n);
    for (int i = 0; i < n; ++i) hx[i] = vtk::rhs_value(0xC0FFEE, i);
    CK(hipMemcpy(x, hx.data(), n * 8, hipMemcpyHostToDevice));
    // host copies for the SELL build
    std::vector<int> hix(nnz);
    std::vector<VT> hd(nnz);
    CK(hipMemcpy(hix.data(), dix, (size_t)nnz * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hd.data(), dd, (size_t)nnz * sizeof(VT), hipMemcpyDeviceToHost));
    const int nch = (n + 63) / 64;
    std::vector<long> off(nch + 1, 0);
    for (int q = 0; q < nch; ++q) {
        int w = 0;
        for (int r = q * 64; r < std::min(n, q * 64 + 64); ++r) w = std::max(w, ip[r + 1] - ip[r]);
        off[q + 1] = off[q] + 64L * w;
    }
    std::vector<int> scol(off[nch], -1);
    std::vector<VT> sval(off[nch], (VT)0);
    for (int q = 0; q < nch; ++q)
        for (int r = q * 64; r < std::min(n, q * 64 + 64); ++r)
            for (int k = ip[r]; k < ip[r + 1]; ++k) {
                const long e = off[q] + (long)(k - ip[r]) * 64 + (r - q * 64);
                scol[e] = hix[k];
                sval[e] = hd[k];
            }
    long *doff; int *dscol; VT *dsval;
    CK(hipMalloc(&doff, (nch + 1) * 8)); CK(hipMalloc(&dscol, off[nch] * 4)); CK(hipMalloc(&dsval, off[nch] * sizeof(VT)));
    CK(hipMemcpy(doff, off.data(), (nch + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dscol, scol.data(), off[nch] * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dsval, sval.data(), off[nch] * sizeof(VT), hipMemcpyHostToDevice));
    std::vector<int> tr(1, 0);
    for (int r = 0; r < n;) {
        int s = r;
        while (r < n && r + 1 - s <= TILE_ROWS && ip[r + 1] - ip[s] <= TILE_NNZ) ++r;
        tr.push_back(r);
    }
    const int ntiles = (int)tr.size() - 1;
    int *dtr; CK(hipMalloc(&dtr, tr.size() * 4));
    CK(hipMemcpy(dtr, tr.data(), tr.size() * 4, hipMemcpyHostToDevice));
    const double B = (4.0 + sizeof(VT)) * nnz + 4.0 * (n + 1) + 16.0 * n;
    printf("n=%d nnz=%d tiles=%d chunks=%d sell_entries=%ld (pad %.2f%%) B=%.3f GB\n", n, nnz, ntiles, nch, off[nch],
           100.0 * (off[nch] - nnz) / nnz, B / 1e9);
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<double> yref(n), hy(n);
    bool have_ref = false;
    auto timeit = [&](const char *name, auto launch) {
        CK(hipMemset(y, 0, n * 8));
        launch(); CK(hipDeviceSynchronize());
        CK(hipMemcpy(hy.data(), y, (size_t)n * 8, hipMemcpyDeviceToHost));
        bool same = true;
        if (!have_ref) { yref = hy; have_ref = true; }
        else same = std::memcmp(hy.data(), yref.data(), (size_t)n * 8) == 0;
        std::vector<float> hot, cold;
        for (int rep = 0; rep < 10; ++rep) {
            CK(hipEventRecord(e0, 0)); launch(); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); hot.push_back(ms);
        }
        for (int rep = 0; rep < 10; ++rep) {
            CK(hipMemsetAsync(junk, rep, 1L << 30, 0));
            CK(hipEventRecord(e0, 0)); launch(); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); cold.push_back(ms);
        }
        std::sort(hot.begin(), hot.end());
        std::sort(cold.begin(), cold.end());
        const double th = hot[5] * 1e-3, tc = cold[5] * 1e-3;
        printf("%-30s hot %7.1f us %5.2f TB/s   cold %7.1f us %5.2f TB/s   %s\n", name, th * 1e6, B / th / 1e12,
               tc * 1e6, B / tc / 1e12, same ? "bit-identical" : "MISMATCH");
    };
    timeit("csr-stream G=1024", [&] { hipLaunchKernelGGL(k_stream<VT>, dim3(std::min(1024, ntiles)), dim3(NT), 0, 0, dip, dix, dd, dtr, ntiles, x, y); });
    for (int G : {1024, 2048}) {
        char nm[64];
        snprintf(nm, 64, "sell nt W=8 G=%d", G);
        timeit(nm, [&] { hipLaunchKernelGGL((k_sell<VT, 8, false, true>), dim3(G), dim3(NT), 0, 0, doff, dscol, dsval, nch, n, x, y); });
        snprintf(nm, 64, "sell nt W=12 G=%d", G);
        timeit(nm, [&] { hipLaunchKernelGGL((k_sell<VT, 12, false, true>), dim3(G), dim3(NT), 0, 0, doff, dscol, dsval, nch, n, x, y); });
        snprintf(nm, 64, "sell nt W=16 G=%d", G);
        timeit(nm, [&] { hipLaunchKernelGGL((k_sell<VT, 16, false, true>), dim3(G), dim3(NT), 0, 0, doff, dscol, dsval, nch, n, x, y); });
        snprintf(nm, 64, "sell nt W=5 G=%d", G);
        timeit(nm, [&] { hipLaunchKernelGGL((k_sell<VT, 5, false, true>), dim3(G), dim3(NT), 0, 0, doff, dscol, dsval, nch, n, x, y); });
    }
    return 0;
}

int main(int argc, char **argv) {
    vtk_vlasov_params p{};
    p.vmax = 6; p.E0 = 0.5; p.nu = 0.05; p.alpha = 0.25; p.cfl = 4;
    const bool c4 = argc > 1 && std::strcmp(argv[1], "c4") == 0;
    if (c4) {
        p.dim = 4; p.shape[0] = 200; p.shape[1] = 125; p.shape[2] = 50; p.shape[3] = 40; p.fp32 = 1;
        printf("C4 (4D 200x125x50x40, f32 values)\n");
        return run<float>(p);
    }
    p.dim = 2; p.shape[0] = 25000; p.shape[1] = 800;
    printf("C3 (2D 25000x800, f64)\n");
    return run<double>(p);
}
