// probe_fused.hip — A/B of the fused SpMV + block-Jacobi(8) kernel on C3 (20M rows), every knob
// a template parameter, variants interleaved in one process (cdna_hip_programming.md §5.4 r24).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/probe_fused.hip -o tools/bin/probe_fused
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <functional>
#include <string>
#include <vector>

#include "../vt-precondition_amd/csrc/vtk_vlasov.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int NT = 256;
constexpr int BS = 8;
typedef double d2v __attribute__((ext_vector_type(2)));

template <bool NTL, typename T> __device__ __forceinline__ T ld(const T *p) {
    if constexpr (NTL) return __builtin_nontemporal_load(p); else return *p;
}
template <bool NTL> __device__ __forceinline__ d2v ld2(const double *p) {
    if constexpr (NTL) return __builtin_nontemporal_load((const d2v *)p); else return *(const d2v *)p;
}

// TR rows / TN nnz per tile; U: unroll of the CSR stream loop; PREF: BJ rows + v0 loaded at tile
// start; NTL: nt loads on CSR / inv / v0; XNT: x gathers nt too
template <int TR, int TN, int U, bool PREF, bool NTL>
__global__ __launch_bounds__(NT) void k_fused(const int *__restrict__ indptr, const int *__restrict__ indices,
                                              const double *__restrict__ data, const int *__restrict__ tile_row, int ntiles,
                                              const double *__restrict__ x, const double *__restrict__ inv,
                                              const double *__restrict__ v0, double *__restrict__ w, double *part0, double *part1) {
    __shared__ double prod[TN];
    __shared__ int rp[TR + 1];
    __shared__ double red[8];
    const int tid = threadIdx.x, lane = tid & 63;
    constexpr int RPT = (TR + NT - 1) / NT;
    double acc0 = 0.0, acc1 = 0.0;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int r0 = tile_row[t], r1 = tile_row[t + 1], nr = r1 - r0;
        const int nz0 = indptr[r0], nnz = indptr[r1] - nz0;
        double m[RPT][BS], pv[RPT];
        if constexpr (PREF) {
#pragma unroll
            for (int q = 0; q < RPT; ++q) {
                const int i = q * NT + tid;
                if (i < nr) {
#pragma unroll
                    for (int j = 0; j < BS; j += 2) { d2v tt = ld2<NTL>(inv + (size_t)(r0 + i) * BS + j); m[q][j] = tt.x; m[q][j + 1] = tt.y; }
                    pv[q] = ld<NTL>(v0 + r0 + i);
                }
            }
        }
        for (int i = tid; i <= nr; i += NT) rp[i] = ld<NTL>(indptr + r0 + i) - nz0;
        const int *ci = indices + nz0;
        const double *cv = data + nz0;
        int e = tid;
        for (; e + (U - 1) * NT < nnz; e += U * NT) {
            int c[U];
            double d[U];
#pragma unroll
            for (int u = 0; u < U; ++u) { c[u] = ld<NTL>(ci + e + u * NT); d[u] = ld<NTL>(cv + e + u * NT); }
#pragma unroll
            for (int u = 0; u < U; ++u) prod[e + u * NT] = d[u] * x[c[u]];
        }
        for (; e < nnz; e += NT) prod[e] = ld<NTL>(cv + e) * x[ld<NTL>(ci + e)];
        __syncthreads();
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int i = q * NT + tid;
            const bool act = i < nr;
            double s = 0.0;
            if (act) for (int k = rp[i]; k < rp[i + 1]; ++k) s += prod[k];
            if constexpr (!PREF) {
                if (act) {
#pragma unroll
                    for (int j = 0; j < BS; j += 2) { d2v tt = ld2<NTL>(inv + (size_t)(r0 + i) * BS + j); m[q][j] = tt.x; m[q][j + 1] = tt.y; }
                    pv[q] = ld<NTL>(v0 + r0 + i);
                }
            }
            const int gb = lane & ~(BS - 1);
            double z = 0.0;
#pragma unroll
            for (int j = 0; j < BS; ++j) {
                const double yj = __shfl(s, gb + j, 64);
                if (act) z += m[q][j] * yj;
            }
            if (act) { w[r0 + i] = z; acc0 += z * z; acc1 += pv[q] * z; }
        }
        __syncthreads();
    }
    for (int off = 32; off > 0; off >>= 1) { acc0 += __shfl_down(acc0, off, 64); acc1 += __shfl_down(acc1, off, 64); }
    if (lane == 0) { red[tid >> 6] = acc0; red[4 + (tid >> 6)] = acc1; }
    __syncthreads();
    if (tid == 0) { part0[blockIdx.x] = red[0] + red[1] + red[2] + red[3]; part1[blockIdx.x] = red[4] + red[5] + red[6] + red[7]; }
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
__global__ void k_fill(double *p, long n, double s) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) p[i] = s * (double)(i % 1000) * 1e-3;
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
    int *dip, *dix; double *dd, *x, *w, *inv, *v0, *part, *V; char *junk;
    const long ld = (n + 63) / 64 * 64;
    CK(hipMalloc(&dip, (n + 1) * 4)); CK(hipMalloc(&dix, nnz * 4)); CK(hipMalloc(&dd, nnz * 8));
    CK(hipMalloc(&V, 3 * ld * 8)); CK(hipMalloc(&w, ld * 8)); CK(hipMalloc(&inv, (size_t)n * BS * 8));
    CK(hipMalloc(&part, 2L * 131072 * 8)); CK(hipMalloc(&junk, 1L << 30));
    x = V; v0 = V + ld;
    CK(hipMemcpy(dip, ip.data(), (n + 1) * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_gen_fill, dim3(2048), dim3(256), 0, 0, p, n, dip, dix, dd);
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, V, 3 * ld, 1.0);
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, inv, (long)n * BS, 0.1);
    CK(hipDeviceSynchronize());
    auto mk_tiles = [&](int TRr, int TNn, int &nt_out) {
        std::vector<int> tr(1, 0);
        for (int r = 0; r < n;) {
            int s = r;
            while (r < n) { int g = std::min(r + BS, n); if (g - s > TRr || ip[g] - ip[s] > TNn) break; r = g; }
            tr.push_back(r);
        }
        nt_out = (int)tr.size() - 1;
        int *d; CK(hipMalloc(&d, tr.size() * 4));
        CK(hipMemcpy(d, tr.data(), tr.size() * 4, hipMemcpyHostToDevice));
        return d;
    };
    int nt512, nt256, nt1024;
    int *t512 = mk_tiles(512, 4096, nt512), *t256 = mk_tiles(256, 2048, nt256), *t1024 = mk_tiles(1024, 8192, nt1024);
    const double B = 12.0 * nnz + 4.0 * (n + 1) + 8.0 * n + 8.0 * n + 64.0 * n + 8.0 * n;   // CSR+x+w+inv+v0
    printf("n=%d nnz=%d B=%.3f GB\n", n, nnz, B / 1e9);
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::map<std::string, std::vector<float>> res;
    std::vector<std::pair<std::string, std::function<void()>>> vars;
#define V(NAME, TR, TN, U, PREF, NTL, TL, NTILES, G) \
    vars.push_back({NAME, [&] { hipLaunchKernelGGL((k_fused<TR, TN, U, PREF, NTL>), dim3(std::min(G, NTILES)), dim3(NT), 0, 0, dip, dix, dd, TL, NTILES, x, inv, v0, w, part, part + 131072); }});
    V("512 u4 plain G1024", 512, 4096, 4, false, false, t512, nt512, 1024)
    V("512 u4 nt G1024", 512, 4096, 4, false, true, t512, nt512, 1024)
    V("512 u4 pref G1024", 512, 4096, 4, true, false, t512, nt512, 1024)
    V("512 u4 pref nt G1024", 512, 4096, 4, true, true, t512, nt512, 1024)
    V("512 u8 plain G1024", 512, 4096, 8, false, false, t512, nt512, 1024)
    V("512 u8 pref G1024", 512, 4096, 8, true, false, t512, nt512, 1024)
    V("512 u2 plain G1024", 512, 4096, 2, false, false, t512, nt512, 1024)
    V("512 u4 plain Gall", 512, 4096, 4, false, false, t512, nt512, 1 << 30)
    V("512 u4 pref Gall", 512, 4096, 4, true, false, t512, nt512, 1 << 30)
    V("256 u4 plain G2048", 256, 2048, 4, false, false, t256, nt256, 2048)
    V("256 u4 pref G2048", 256, 2048, 4, true, false, t256, nt256, 2048)
    V("256 u4 plain Gall", 256, 2048, 4, false, false, t256, nt256, 1 << 30)
    V("256 u8 pref Gall", 256, 2048, 8, true, false, t256, nt256, 1 << 30)
    V("1024 u4 plain G1024", 1024, 8192, 4, false, false, t1024, nt1024, 1024)
    V("1024 u4 pref G1024", 1024, 8192, 4, true, false, t1024, nt1024, 1024)
    for (auto &v : vars) v.second();
    CK(hipDeviceSynchronize());
    for (int rep = 0; rep < 8; ++rep) {
        for (auto &v : vars) {
            CK(hipMemsetAsync(junk, rep, 1L << 29, 0));
            CK(hipEventRecord(e0, 0)); v.second(); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); res[v.first].push_back(ms);
        }
    }
    for (auto &v : vars) {
        auto ts = res[v.first];
        std::sort(ts.begin(), ts.end());
        printf("%-24s min %7.1f us  med %7.1f us  -> %.2f TB/s (med)\n", v.first.c_str(), ts[0] * 1e3, ts[ts.size() / 2] * 1e3, B / (ts[ts.size() / 2] * 1e-3) / 1e12);
    }
    return 0;
}
