// probe_stream.hip — ceilings for the SpMV's memory pattern on C3 (100M nnz, 20M rows):
//   A: indices(4 B) + values(8 B) per lane per nnz, coalesced, summed in registers
//   B: same data, 16 B per lane (int4 + 2 x double2)
//   C: A + x gather (no LDS)       D: B + x gather (no LDS)
//   E: pure 16-B copy-read of the same 1.2 GB (reference roof)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe_stream.hip -o tools/bin/probe_stream
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
constexpr int NT = 256;
typedef int i4v __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));

template <bool GATHER>
__global__ __launch_bounds__(NT) void kA(const int *__restrict__ ix, const double *__restrict__ d, long nnz,
                                         const double *__restrict__ x, double *out) {
    double acc = 0;
    for (long e = (long)blockIdx.x * NT + threadIdx.x; e < nnz; e += (long)gridDim.x * NT) {
        const int c = ix[e];
        acc += d[e] * (GATHER ? x[c] : (double)c);
    }
    if (acc == 12345.678) out[0] = acc;
}
template <bool GATHER>
__global__ __launch_bounds__(NT) void kB(const int *__restrict__ ix, const double *__restrict__ d, long nnz,
                                         const double *__restrict__ x, double *out) {
    double acc = 0;
    for (long q = 4 * ((long)blockIdx.x * NT + threadIdx.x); q < nnz; q += 4L * gridDim.x * NT) {
        const i4v c = *(const i4v *)(ix + q);
        const d2v a = *(const d2v *)(d + q), b = *(const d2v *)(d + q + 2);
        if (GATHER) acc += a.x * x[c.x] + a.y * x[c.y] + b.x * x[c.z] + b.y * x[c.w];
        else acc += a.x * c.x + a.y * c.y + b.x * c.z + b.y * c.w;
    }
    if (acc == 12345.678) out[0] = acc;
}
__global__ __launch_bounds__(NT) void kE(const d2v *__restrict__ p, long n2, double *out) {
    d2v acc = {0, 0};
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n2; i += (long)gridDim.x * NT) acc += p[i];
    if (acc.x == 12345.678) out[0] = acc.y;
}
template <int U>
__global__ __launch_bounds__(NT) void kAU(const int *__restrict__ ix, const double *__restrict__ d, long nnz,
                                          const double *__restrict__ x, double *out) {
    double acc = 0;
    const long S = (long)gridDim.x * NT;
    long e = (long)blockIdx.x * NT + threadIdx.x;
    for (; e + (U - 1) * S < nnz; e += U * S) {
        int c[U]; double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) { c[u] = ix[e + u * S]; v[u] = d[e + u * S]; }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u] * x[c[u]];
    }
    for (; e < nnz; e += S) acc += d[e] * x[ix[e]];
    if (acc == 12345.678) out[0] = acc;
}
template <int U>
__global__ __launch_bounds__(NT) void kEU(const d2v *__restrict__ p, long n2, double *out) {
    d2v acc = {0, 0};
    const long S = (long)gridDim.x * NT;
    long i = (long)blockIdx.x * NT + threadIdx.x;
    for (; i + (U - 1) * S < n2; i += U * S) {
        d2v t[U];
#pragma unroll
        for (int u = 0; u < U; ++u) t[u] = p[i + u * S];
#pragma unroll
        for (int u = 0; u < U; ++u) acc += t[u];
    }
    for (; i < n2; i += S) acc += p[i];
    if (acc.x == 12345.678) out[0] = acc.y;
}
__global__ void k_fill_ix(int *ix, long nnz, int n) {
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < nnz; e += (long)gridDim.x * blockDim.x) {
        const long r = e / 5, k = e % 5;
        const long off[5] = {-800, -1, 0, 1, 800};
        long c = r + off[k];
        c = (c % n + n) % n;
        ix[e] = (int)c;
    }
}

int main() {
    const int n = 20000000;
    const long nnz = 5L * n;
    int *ix; double *d, *x, *out; char *junk;
    CK(hipMalloc(&ix, nnz * 4 + 64)); CK(hipMalloc(&d, nnz * 8 + 64)); CK(hipMalloc(&x, (long)n * 8));
    CK(hipMalloc(&out, 64)); CK(hipMalloc(&junk, 1L << 30));
    hipLaunchKernelGGL(k_fill_ix, dim3(4096), dim3(256), 0, 0, ix, nnz, n);
    CK(hipMemset(d, 0, nnz * 8)); CK(hipMemset(x, 0, (long)n * 8));
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, double bytes, auto f) {
        f(); CK(hipDeviceSynchronize());
        std::vector<float> ts;
        for (int r = 0; r < 10; ++r) {
            CK(hipMemsetAsync(junk, r, 1L << 29, 0));
            CK(hipEventRecord(e0, 0)); f(); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("%-34s med %7.1f us -> %.2f TB/s\n", name, ts[5] * 1e3, bytes / (ts[5] * 1e-3) / 1e12);
    };
    const double B = 12.0 * nnz, Bx = B + 8.0 * n;
    for (int G : {1024, 2048, 4096}) {
        char nm[64];
        snprintf(nm, 64, "A 4B+8B G=%d", G); timeit(nm, B, [&] { hipLaunchKernelGGL(kA<false>, dim3(G), dim3(NT), 0, 0, ix, d, nnz, x, out); });
        snprintf(nm, 64, "AU2 +gather G=%d", G); timeit(nm, Bx, [&] { hipLaunchKernelGGL(kAU<2>, dim3(G), dim3(NT), 0, 0, ix, d, nnz, x, out); });
        snprintf(nm, 64, "AU4 +gather G=%d", G); timeit(nm, Bx, [&] { hipLaunchKernelGGL(kAU<4>, dim3(G), dim3(NT), 0, 0, ix, d, nnz, x, out); });
        snprintf(nm, 64, "AU8 +gather G=%d", G); timeit(nm, Bx, [&] { hipLaunchKernelGGL(kAU<8>, dim3(G), dim3(NT), 0, 0, ix, d, nnz, x, out); });
        snprintf(nm, 64, "E 16B G=%d", G); timeit(nm, 8.0 * nnz, [&] { hipLaunchKernelGGL(kE, dim3(G), dim3(NT), 0, 0, (const d2v *)d, nnz / 2, out); });
        snprintf(nm, 64, "EU2 16B G=%d", G); timeit(nm, 8.0 * nnz, [&] { hipLaunchKernelGGL(kEU<2>, dim3(G), dim3(NT), 0, 0, (const d2v *)d, nnz / 2, out); });
        snprintf(nm, 64, "EU4 16B G=%d", G); timeit(nm, 8.0 * nnz, [&] { hipLaunchKernelGGL(kEU<4>, dim3(G), dim3(NT), 0, 0, (const d2v *)d, nnz / 2, out); });
        snprintf(nm, 64, "EU8 16B G=%d", G); timeit(nm, 8.0 * nnz, [&] { hipLaunchKernelGGL(kEU<8>, dim3(G), dim3(NT), 0, 0, (const d2v *)d, nnz / 2, out); });
    }
    return 0;
}
