// probe_mgs.hip — micro-benchmark of MGS-step variants on the C3 vector size (n = 20M fp64),
// run as a chain j = 0..J like the real Arnoldi step, to see whether keeping w resident in the
// 256 MB Infinity Cache (non-temporal loads of the streamed basis vectors) lowers HBM traffic.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/probe_mgs.hip -o build/probe_mgs
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));
constexpr int NT = 256;

// MODE: 0 plain, 1 nt on v loads, 2 nt on everything, 3 nt on w only, 4 nt on vk only
template <int MODE>
__global__ __launch_bounds__(NT) void k_mgs(const double *hp, int G, double *__restrict__ w,
                                            const double *__restrict__ vk, const double *__restrict__ vn,
                                            long n, double *part, int rev) {
    __shared__ double red[4];
    double h = 0.0;
    for (int i = threadIdx.x; i < G; i += NT) h += hp[i];
    for (int off = 32; off > 0; off >>= 1) h += __shfl_down(h, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = h;
    __syncthreads();
    h = red[0] + red[1] + red[2] + red[3];
    h = h * 1e-30;
    double acc = 0.0;
    const long stride = 2L * gridDim.x * NT;
    for (long i0 = 2L * (blockIdx.x * NT + threadIdx.x); i0 < n; i0 += stride) {
        const long i = rev ? (n - 2 - i0) : i0;
        d2 wv, kv, nv;
        if (MODE == 2 || MODE == 3) wv = __builtin_nontemporal_load((const d2 *)(w + i));
        else wv = *(const d2 *)(w + i);
        if (MODE == 1 || MODE == 2) { kv = __builtin_nontemporal_load((const d2 *)(vk + i)); nv = __builtin_nontemporal_load((const d2 *)(vn + i)); }
        else if (MODE >= 4) { kv = __builtin_nontemporal_load((const d2 *)(vk + i)); nv = *(const d2 *)(vn + i); }
        else { kv = *(const d2 *)(vk + i); nv = *(const d2 *)(vn + i); }
        wv.x = wv.x - h * kv.x;
        wv.y = wv.y - h * kv.y;
        if (MODE == 2 || MODE == 6) __builtin_nontemporal_store(wv, (d2 *)(w + i));
        else if (MODE == 5) { /* read-only: no store */ }
        else *(d2 *)(w + i) = wv;
        acc += nv.x * wv.x;
        acc += nv.y * wv.y;
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void k_fill(double *p, long n, double s) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) p[i] = s * (double)(i % 1000) * 1e-3;
}

template <int MODE>
float run_chain(double *w, double *V, long ld, long n, int J, int G, double *part, hipStream_t s, std::vector<float> &per, int alt) {
    hipEvent_t e[64];
    for (int i = 0; i <= J + 1; ++i) CK(hipEventCreate(&e[i]));
    CK(hipEventRecord(e[0], s));
    for (int k = 0; k <= J; ++k) {
        hipLaunchKernelGGL(k_mgs<MODE>, dim3(G), dim3(NT), 0, s, part + (k & 1) * 2048, G, w, V + k * ld, V + (k + 1) * ld, n, part + ((k + 1) & 1) * 2048, alt ? (k & 1) : 0);
        CK(hipEventRecord(e[k + 1], s));
    }
    CK(hipEventSynchronize(e[J + 1]));
    float tot;
    CK(hipEventElapsedTime(&tot, e[0], e[J + 1]));
    per.resize(J + 1);
    for (int k = 0; k <= J; ++k) CK(hipEventElapsedTime(&per[k], e[k], e[k + 1]));
    for (int i = 0; i <= J + 1; ++i) CK(hipEventDestroy(e[i]));
    return tot;
}

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 20000000L;
    const int J = 10;
    const long ld = (n + 63) / 64 * 64;
    double *w, *V, *part, *junk;
    CK(hipMalloc(&w, ld * 8));
    CK(hipMalloc(&V, (J + 2) * ld * 8));
    CK(hipMalloc(&part, 4096 * 8));
    CK(hipMalloc(&junk, 1L << 30));
    CK(hipMemset(part, 0, 4096 * 8));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, s, w, n, 1.0);
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, s, V, (J + 2) * ld, 0.5);
    CK(hipStreamSynchronize(s));
    const double bytes_mid = 32.0 * n;
    for (int G : {1024}) {
        for (int rep = 0; rep < 2; ++rep) {
            for (int alt = 0; alt < 1; ++alt) {
            for (int mode : {4, 5, 6}) {
                CK(hipMemsetAsync(junk, rep, 1L << 30, s));   // flush caches
                std::vector<float> per;
                float t = 0;
                switch (mode) {
                    case 0: t = run_chain<0>(w, V, ld, n, J, G, part, s, per, alt); break;
                    case 1: t = run_chain<1>(w, V, ld, n, J, G, part, s, per, alt); break;
                    case 4: t = run_chain<4>(w, V, ld, n, J, G, part, s, per, alt); break;
                    case 5: t = run_chain<5>(w, V, ld, n, J, G, part, s, per, alt); break;
                    case 6: t = run_chain<6>(w, V, ld, n, J, G, part, s, per, alt); break;
                }
                std::vector<float> q(per.begin() + 1, per.end());
                std::sort(q.begin(), q.end());
                const double med = q[q.size() / 2];
                printf("G=%d rep=%d alt=%d mode=%d chain(J=%d) %.3f ms  per-step median %.1f us  first %.1f us  -> %.2f TB/s algorithmic(32n)\n",
                       G, rep, alt, mode, J, t, med * 1e3, per[0] * 1e3, bytes_mid / (med * 1e-3) / 1e12);
            }
            }
        }
    }
    // smaller vectors (C2: 5M, C1: 1M) for the cache-resident regime
    return 0;
}
