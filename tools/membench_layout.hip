// tools/membench_layout.hip -- does the basis layout set the band step's streaming ceiling?
// (DESIGN.md §3g).  The band step at j reads j basis rows + 2 w rows of every line (plus D, m) and
// writes 2; today the basis is vector-major (V_k at k * ld), so a workgroup's line reads j + 2
// separate 3.2 KB pieces 160 MB apart.  This bench reads NV "vectors" and writes 2 in the band
// step's walk (workgroup = half line of 400 rows, contiguous line ranges, 7 waves, 2 per CU) for
//   LAY 0  vector-major   V[k][x][v]     (today)
//   LAY 1  line-major     V[x][k][v]     (a line's NV rows contiguous: 20 x 6.4 KB)
//   LAY 2  part-major     V[x][h][k][v'] (a workgroup's NV pieces contiguous: 20 x 3.2 KB)
//   LAY 3  vector-major, lines stored interleaved: line t of range r at slot t R + r (every
//          workgroup's t-th line side by side in memory: the walks move through one window)
//   LAY 4  line-major with the interleaved line slots
// each with the loads of line x + 1 issued before line x is consumed (PF, as the band step's
// register prefetch) or at the line head.  Also a float4 copy (the guide's 6.29 TB/s reference)
// and a grid-stride read of NV vectors.  Build: hipcc --offload-arch=gfx950 -O3 -o ... this file
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                               \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
            std::exit(2);                                                                    \
        }                                                                                    \
    } while (0)

__device__ __forceinline__ double ldn(const double *p) { return __builtin_nontemporal_load(p); }

template <int NV, int LAY>
__device__ __forceinline__ int64_t vaddr(int k, int x, int h, int t, int L, int LP, int64_t ld) {
    if constexpr (LAY == 0 || LAY == 3) return (int64_t)k * ld + (int64_t)x * L + h * LP + t;
    else if constexpr (LAY == 1 || LAY == 4) return ((int64_t)x * NV + k) * L + h * LP + t;
    else return (((int64_t)x * (L / LP) + h) * NV + k) * LP + t;
}

template <int NV, int LAY, bool PF>
__global__ __launch_bounds__(448) void k_walk(const double *__restrict__ V, int64_t n, int L, int H, int64_t ld,
                                              double *__restrict__ o0, double *__restrict__ o1) {
    const int LP = L / H, X = (int)(n / L);
    const int b = blockIdx.x, R = (int)gridDim.x / H, rb = b / H, h = b % H;
    const int xa = (int)((int64_t)rb * X / R), xb = (int)((int64_t)(rb + 1) * X / R);
    const int t = threadIdx.x;
    if (t >= LP) return;
    double nx[NV];
    // LAY 3 / 4: the storage slot of line x (range rb, t = x - xa): t R + rb (ranges of nl or
    // nl + 1 lines; slots past X wrap into the short ranges' gaps -- a bench, not a bijection)
    auto slot = [&](int x) { return (LAY >= 3) ? ((x - xa) * R + rb) % X : x; };
    auto load = [&](int x, double *o) {
#pragma unroll
        for (int k = 0; k < NV; ++k) o[k] = ldn(V + vaddr<NV, LAY>(k, slot(x), h, t, L, LP, ld));
    };
    if constexpr (PF) load(xa, nx);
    for (int x = xa; x < xb; ++x) {
        double cu[NV];
        if constexpr (PF) {
#pragma unroll
            for (int k = 0; k < NV; ++k) cu[k] = nx[k];
            if (x + 1 < xb) load(x + 1, nx);
        } else {
            load(x, cu);
        }
        double a = 0.0, c = 0.0;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            a += cu[k];
            c -= cu[k];
        }
        const int64_t i = (int64_t)slot(x) * L + h * LP + t;
        __builtin_nontemporal_store(a, o0 + i);
        __builtin_nontemporal_store(c, o1 + i);
    }
}

template <int NV>
__global__ __launch_bounds__(256) void k_rows(const double *__restrict__ V, int64_t n, int64_t ld,
                                              double *__restrict__ o0, double *__restrict__ o1) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        double a = 0.0, b = 0.0;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const double v = ldn(V + (size_t)k * ld + i);
            a += v;
            b -= v;
        }
        __builtin_nontemporal_store(a, o0 + i);
        __builtin_nontemporal_store(b, o1 + i);
    }
}

__global__ __launch_bounds__(256) void k_copy4(const float4 *__restrict__ a, float4 *__restrict__ b, int64_t n4) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) b[i] = a[i];
}

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? std::atoll(argv[1]) : 20000000;
    constexpr int NV = 20;
    const int L = 800, H = 2;
    int dev = 0, ncu = 0;
    CHK(hipGetDevice(&dev));
    CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    const int64_t ld = (n + 63) / 64 * 64;
    double *V, *o0, *o1;
    CHK(hipMalloc(&V, sizeof(double) * NV * ld));
    CHK(hipMalloc(&o0, sizeof(double) * n));
    CHK(hipMalloc(&o1, sizeof(double) * n));
    CHK(hipMemset(V, 0, sizeof(double) * NV * ld));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const int X = (int)(n / L);
    auto run = [&](const char *name, double bytes, auto launch) {
        launch();
        CHK(hipDeviceSynchronize());
        std::vector<float> ts;
        for (int r = 0; r < 9; ++r) {
            CHK(hipEventRecord(e0));
            launch();
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        std::printf("%-34s %8.1f us  %7.1f GB/s\n", name, 1e3 * ts[4], bytes / (1e-3 * ts[4]) / 1e9);
        std::fflush(stdout);
    };
    const double bw = 8.0 * n * (NV + 2);
    const int64_t n4 = (int64_t)NV * ld * 8 / 16 / 2;
    run("copy float4 (read+write)", 32.0 * n4, [&] {
        hipLaunchKernelGGL(k_copy4, dim3(ncu * 8), dim3(256), 0, 0, (const float4 *)V, (float4 *)V + n4, n4);
    });
    run("gridstride NV=20", bw, [&] { hipLaunchKernelGGL(k_rows<NV>, dim3(ncu * 8), dim3(256), 0, 0, V, n, ld, o0, o1); });
    for (int rep = 0; rep < 2; ++rep) {
        const int R = std::min(2 * ncu / H, X / 2);
#define W(LAY_, PF_, NAME_) \
        run(NAME_, bw, [&] { hipLaunchKernelGGL((k_walk<NV, LAY_, PF_>), dim3(R * H), dim3(448), 0, 0, V, n, L, H, ld, o0, o1); })
        W(0, false, "walk vector-major head");
        W(0, true, "walk vector-major prefetch");
        W(1, false, "walk line-major head");
        W(1, true, "walk line-major prefetch");
        W(2, false, "walk part-major head");
        W(2, true, "walk part-major prefetch");
        W(3, false, "walk interleaved head");
        W(3, true, "walk interleaved prefetch");
        W(4, false, "walk interleaved line-major head");
        W(4, true, "walk interleaved line-major prefetch");
#undef W
    }
    CHK(hipFree(V));
    CHK(hipFree(o0));
    CHK(hipFree(o1));
    return 0;
}
