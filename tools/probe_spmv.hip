// probe_spmv.hip — SpMV variants on the C3 operator (2D Vlasov 25000 x 800, 20M rows, 100M nnz).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I. tools/probe_spmv.hip -o tools/bin/probe_spmv
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../vt-precondition_amd/csrc/vtk_vlasov.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int NT = 256;
typedef int i4v __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));
constexpr int TILE_ROWS = 512, TILE_NNZ = 4096;

template <typename T> __device__ __forceinline__ T ldg(const T *p, bool nt) {
    return nt ? __builtin_nontemporal_load(p) : *p;
}

// CSR-stream (as in vtk_kernels.hip), NT_LOADS: streamed arrays non-temporal
template <bool NTL, int UNR>
__global__ __launch_bounds__(NT) void k_stream(const int *__restrict__ indptr, const int *__restrict__ indices,
                                               const double *__restrict__ data, const int *__restrict__ tile_row, int ntiles,
                                               const double *__restrict__ x, double *__restrict__ y) {
    __shared__ double prod[TILE_NNZ];
    __shared__ int rp[TILE_ROWS + 1];
    const int tid = threadIdx.x;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int r0 = tile_row[t], r1 = tile_row[t + 1], nr = r1 - r0;
        const int nz0 = indptr[r0], nnz = indptr[r1] - nz0;
        for (int i = tid; i <= nr; i += NT) rp[i] = ldg(indptr + r0 + i, NTL) - nz0;
        const int *ci = indices + nz0;
        const double *cv = data + nz0;
        int e = tid;
        for (; e + (UNR - 1) * NT < nnz; e += UNR * NT) {
            int c[UNR];
            double d[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u) { c[u] = ldg(ci + e + u * NT, NTL); d[u] = ldg(cv + e + u * NT, NTL); }
#pragma unroll
            for (int u = 0; u < UNR; ++u) prod[e + u * NT] = d[u] * x[c[u]];
        }
        for (; e < nnz; e += NT) prod[e] = ldg(cv + e, NTL) * x[ldg(ci + e, NTL)];
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


// vectorised CSR-stream: each lane loads 4 consecutive nnz (int4 indices, 2x double2 values)
// from a 4-aligned base; arrays are padded so the last quad stays in bounds.
template <int TR, int TN, int UNR>
__global__ __launch_bounds__(NT) void k_stream4(const int *__restrict__ indptr, const int *__restrict__ indices,
                                                const double *__restrict__ data, const int *__restrict__ tile_row, int ntiles,
                                                const double *__restrict__ x, double *__restrict__ y) {
    __shared__ double prod[TN + 8];
    __shared__ int rp[TR + 1];
    const int tid = threadIdx.x;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int r0 = tile_row[t], r1 = tile_row[t + 1], nr = r1 - r0;
        const int nz0 = indptr[r0], nz1 = indptr[r1];
        for (int i = tid; i <= nr; i += NT) rp[i] = indptr[r0 + i] - nz0;
        const int base = nz0 & ~3;
        for (int q = base + 4 * tid; q < nz1; q += 4 * NT * UNR) {
            i4v c[UNR];
            d2v d0[UNR], d1[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                const int qq = q + 4 * NT * u;
                if (qq < nz1) {
                    c[u] = __builtin_nontemporal_load((const i4v *)(indices + qq));
                    d0[u] = __builtin_nontemporal_load((const d2v *)(data + qq));
                    d1[u] = __builtin_nontemporal_load((const d2v *)(data + qq + 2));
                }
            }
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                const int qq = q + 4 * NT * u;
                if (qq < nz1) {
                    const int e = qq - nz0;
                    if (e >= 0 && e < nz1 - nz0) prod[e] = d0[u].x * x[c[u].x];
                    if (e + 1 >= 0 && e + 1 < nz1 - nz0) prod[e + 1] = d0[u].y * x[c[u].y];
                    if (e + 2 >= 0 && e + 2 < nz1 - nz0) prod[e + 2] = d1[u].x * x[c[u].z];
                    if (e + 3 >= 0 && e + 3 < nz1 - nz0) prod[e + 3] = d1[u].y * x[c[u].w];
                }
            }
        }
        __syncthreads();
        for (int base2 = 0; base2 < nr; base2 += NT) {
            const int i = base2 + tid;
            if (i < nr) {
                double s = 0.0;
                for (int k = rp[i]; k < rp[i + 1]; ++k) s += prod[k];
                y[r0 + i] = s;
            }
        }
        __syncthreads();
    }
}


// CSR-stream, unroll 8, nt streamed loads, XCD-aware tile order: workgroup b runs on XCD b % 8
// (round-robin dispatch); give each XCD a contiguous range of tiles so neighbouring tiles (which
// share x-window lines) hit the same L2.
template <int UNR, int XCD>
__global__ __launch_bounds__(NT) void k_stream_x(const int *__restrict__ indptr, const int *__restrict__ indices,
                                                 const double *__restrict__ data, const int *__restrict__ tile_row, int ntiles,
                                                 const double *__restrict__ x, double *__restrict__ y) {
    __shared__ double prod[TILE_NNZ];
    __shared__ int rp[TILE_ROWS + 1];
    const int tid = threadIdx.x;
    const int G = gridDim.x, b = blockIdx.x;
    const int per_x = (ntiles + 7) / 8;          // tiles per XCD chunk
    const int xcd = b % 8, j = b / 8, gx = (G + 7 - xcd) / 8;   // blocks on this XCD
    for (int tt = j; ; tt += gx) {
        int t;
        if (XCD) { if (tt >= per_x) break; t = xcd * per_x + tt; if (t >= ntiles) break; }
        else { t = b + (tt - j) * G; if (tt != j && false) break; if (t >= ntiles) break; }
        const int r0 = tile_row[t], r1 = tile_row[t + 1], nr = r1 - r0;
        const int nz0 = indptr[r0], nnz = indptr[r1] - nz0;
        for (int i = tid; i <= nr; i += NT) rp[i] = __builtin_nontemporal_load(indptr + r0 + i) - nz0;
        const int *ci = indices + nz0;
        const double *cv = data + nz0;
        int e = tid;
        for (; e + (UNR - 1) * NT < nnz; e += UNR * NT) {
            int c[UNR];
            double d[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u) { c[u] = __builtin_nontemporal_load(ci + e + u * NT); d[u] = __builtin_nontemporal_load(cv + e + u * NT); }
#pragma unroll
            for (int u = 0; u < UNR; ++u) prod[e + u * NT] = d[u] * x[c[u]];
        }
        for (; e < nnz; e += NT) prod[e] = __builtin_nontemporal_load(cv + e) * x[__builtin_nontemporal_load(ci + e)];
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

// one lane per row, direct loads
template <bool NTL>
__global__ __launch_bounds__(NT) void k_row(const int *__restrict__ indptr, const int *__restrict__ indices,
                                            const double *__restrict__ data, int n, const double *__restrict__ x,
                                            double *__restrict__ y) {
    for (int r = blockIdx.x * NT + threadIdx.x; r < n; r += gridDim.x * NT) {
        const int k0 = ldg(indptr + r, NTL), k1 = ldg(indptr + r + 1, NTL);
        double s = 0.0;
        for (int k = k0; k < k1; ++k) s += ldg(data + k, NTL) * x[ldg(indices + k, NTL)];
        y[r] = s;
    }
}

// one wavefront per 64 rows, LDS-free: lanes cooperatively load the wave's nnz window
// coalesced (like stream), products to registers -> LDS per wave (no block barrier)
template <bool NTL>
__global__ __launch_bounds__(NT) void k_wave(const int *__restrict__ indptr, const int *__restrict__ indices,
                                             const double *__restrict__ data, int n, const double *__restrict__ x,
                                             double *__restrict__ y) {
    __shared__ double prod[4][64 * 10];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    double *pp = prod[wv];
    const int nwaves = gridDim.x * 4;
    for (int r0 = (blockIdx.x * 4 + wv) * 64; r0 < n; r0 += nwaves * 64) {
        const int r1 = min(r0 + 64, n);
        const int nz0 = indptr[r0], nz1 = indptr[r1];
        const int nnz = nz1 - nz0;   // <= 640 for <= 10 nnz/row
        for (int e = lane; e < nnz; e += 64) pp[e] = ldg(data + nz0 + e, NTL) * x[ldg(indices + nz0 + e, NTL)];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        const int r = r0 + lane;
        if (r < r1) {
            const int k0 = indptr[r] - nz0, k1 = indptr[r + 1] - nz0;
            double s = 0.0;
            for (int k = k0; k < k1; ++k) s += pp[k];
            y[r] = s;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

__global__ void k_gen_counts(vtk_vlasov_params p, int n, int *cnt) {
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) cnt[r] = vtk::vlasov_row_count(p, r);
}
__global__ void k_gen_fill(vtk_vlasov_params p, int n, const int *indptr, int *ix, double *d) {
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
        vtk::VlasovRow row;
        vtk::vlasov_row(p, r, row);
        for (int k = 0; k < row.count; ++k) { ix[indptr[r] + k] = (int)row.col[k]; d[indptr[r] + k] = row.val[k]; }
    }
}

int main(int argc, char **argv) {
    vtk_vlasov_params p{};
    p.dim = 2; p.shape[0] = argc > 1 ? atol(argv[1]) : 25000; p.shape[1] = 800;
    p.vmax = 6; p.E0 = 0.5; p.nu = 0.05; p.alpha = 0.25; p.cfl = 4;
    const int n = (int)(p.shape[0] * p.shape[1]);
    std::vector<int> cnt(n), ip(n + 1);
    int *dcnt; CK(hipMalloc(&dcnt, n * 4));
    hipLaunchKernelGGL(k_gen_counts, dim3(2048), dim3(256), 0, 0, p, n, dcnt);
    CK(hipMemcpy(cnt.data(), dcnt, n * 4, hipMemcpyDeviceToHost));
    ip[0] = 0;
    for (int i = 0; i < n; ++i) ip[i + 1] = ip[i] + cnt[i];
    const int nnz = ip[n];
    int *dip, *dix; double *dd, *x, *y, *y2; char *junk;
    CK(hipMalloc(&dip, (n + 1) * 4)); CK(hipMalloc(&dix, (nnz + 16) * 4)); CK(hipMalloc(&dd, (nnz + 16) * 8)); CK(hipMemset(dix, 0, (nnz + 16) * 4)); CK(hipMemset(dd, 0, (nnz + 16) * 8));
    CK(hipMalloc(&x, n * 8)); CK(hipMalloc(&y, n * 8)); CK(hipMalloc(&y2, n * 8)); CK(hipMalloc(&junk, 1L << 30));
    CK(hipMemcpy(dip, ip.data(), (n + 1) * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_gen_fill, dim3(2048), dim3(256), 0, 0, p, n, dip, dix, dd);
    std::vector<double> hx(n);
    for (int i = 0; i < n; ++i) hx[i] = vtk::rhs_value(0xC0FFEE, i);
    CK(hipMemcpy(x, hx.data(), n * 8, hipMemcpyHostToDevice));
    auto mk_tiles = [&](int TRr, int TNn, int &nt_out) {
        std::vector<int> tr(1, 0);
        for (int r = 0; r < n;) {
            int s = r;
            while (r < n && r + 1 - s <= TRr && ip[r + 1] - ip[s] <= TNn) ++r;
            tr.push_back(r);
        }
        nt_out = (int)tr.size() - 1;
        int *d; CK(hipMalloc(&d, tr.size() * 4));
        CK(hipMemcpy(d, tr.data(), tr.size() * 4, hipMemcpyHostToDevice));
        return d;
    };
    int ntiles, nt2, nt3;
    int *dtr = mk_tiles(TILE_ROWS, TILE_NNZ, ntiles);
    int *dtr2 = mk_tiles(256, 2048, nt2);
    int *dtr3 = mk_tiles(1024, 8192, nt3);
    const double B = 12.0 * nnz + 4.0 * (n + 1) + 16.0 * n;
    printf("n=%d nnz=%d tiles=%d B=%.3f GB\n", n, nnz, ntiles, B / 1e9);
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, auto launch) {
        launch(); CK(hipDeviceSynchronize());
        std::vector<float> ts;
        for (int rep = 0; rep < 20; ++rep) {
            if (rep % 2 == 0) CK(hipMemsetAsync(junk, rep, 1L << 30, 0));
            CK(hipEventRecord(e0, 0)); launch(); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        CK(hipMemcpy(y2, y, 8, hipMemcpyDeviceToDevice));
        std::vector<double> hy(n);
        CK(hipMemcpy(hy.data(), y, n * 8, hipMemcpyDeviceToHost));
        double cs = 0; for (int i = 0; i < n; ++i) cs += hy[i] * (1 + (i % 7));
        printf("%-28s min %7.1f us  med %7.1f us  -> %.2f TB/s (med)  checksum %.15e\n", name, ts[0] * 1e3, ts[ts.size() / 2] * 1e3,
               B / (ts[ts.size() / 2] * 1e-3) / 1e12, cs);
        CK(hipMemset(y, 0, n * 8));
    };
    for (int G : {1024, 2048, 100000}) {
        const int g = std::min(G, ntiles);
        char nm[64];
        snprintf(nm, 64, "stream nt unr8 G=%d", g);
        timeit(nm, [&] { hipLaunchKernelGGL((k_stream<true, 8>), dim3(g), dim3(NT), 0, 0, dip, dix, dd, dtr, ntiles, x, y); });
        snprintf(nm, 64, "stream_x xcd unr8 G=%d", g);
        timeit(nm, [&] { hipLaunchKernelGGL((k_stream_x<8, 1>), dim3(g), dim3(NT), 0, 0, dip, dix, dd, dtr, ntiles, x, y); });
        snprintf(nm, 64, "stream_x xcd unr4 G=%d", g);
        timeit(nm, [&] { hipLaunchKernelGGL((k_stream_x<4, 1>), dim3(g), dim3(NT), 0, 0, dip, dix, dd, dtr, ntiles, x, y); });
    }
    for (int G : {2048}) {
        char nm[64];
        snprintf(nm, 64, "wave G=%d", G);
        timeit(nm, [&] { hipLaunchKernelGGL((k_wave<false>), dim3(G), dim3(NT), 0, 0, dip, dix, dd, n, x, y); });
    }
    // pure streaming read roof for reference: sum of data array
    return 0;
}
