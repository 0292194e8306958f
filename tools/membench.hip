// tools/membench.hip -- HBM read-rate ceiling of the band step's access shape.
// Reads NV vectors of n doubles and writes 2 (the band step at j = NV - 2), one row per lane
// (8 B per load, as k_band_step) or two rows per lane (16 B), nontemporal or plain, grid-stride
// or the band step's line-part walk (workgroup = 400 rows of one line part, lines of 800 rows
// in ranges).  Prints GB/s per variant.  Build: hipcc --offload-arch=gfx950 -O3 -o membench membench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                      \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(2);                                                           \
        }                                                                           \
    } while (0)

constexpr int NV = 20;
__constant__ int64_t LDV;   // vector stride in doubles (n + pad)

template <bool NT>
__device__ __forceinline__ double ld(const double *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ double2 ld2(const double2 *p) {
    if constexpr (NT) {
        double2 r;
        r.x = __builtin_nontemporal_load(&p->x);
        r.y = __builtin_nontemporal_load(&p->y);
        return r;
    } else {
        return *p;
    }
}

// grid-stride, one row per lane
template <bool NT>
__global__ __launch_bounds__(256) void k_rows8(const double *__restrict__ V, int64_t n, double *__restrict__ o0,
                                               double *__restrict__ o1) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        double a = 0.0, b = 0.0;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const double v = ld<NT>(V + (size_t)k * LDV + i);
            a += v;
            b -= v;
        }
        __builtin_nontemporal_store(a, o0 + i);
        __builtin_nontemporal_store(b, o1 + i);
    }
}

// grid-stride, two rows per lane
template <bool NT>
__global__ __launch_bounds__(256) void k_rows16(const double *__restrict__ V, int64_t n, double *__restrict__ o0,
                                                double *__restrict__ o1) {
    const int64_t n2 = n / 2;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256) {
        double ax = 0.0, ay = 0.0, bx = 0.0, by = 0.0;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const double2 v = ld2<NT>(reinterpret_cast<const double2 *>(V + (size_t)k * LDV) + i);
            ax += v.x;
            ay += v.y;
            bx -= v.x;
            by -= v.y;
        }
        double2 *p0 = reinterpret_cast<double2 *>(o0) + i, *p1 = reinterpret_cast<double2 *>(o1) + i;
        __builtin_nontemporal_store(ax, &p0->x);
        __builtin_nontemporal_store(ay, &p0->y);
        __builtin_nontemporal_store(bx, &p1->x);
        __builtin_nontemporal_store(by, &p1->y);
    }
}

// the band step's walk: workgroup (range r, part h) reads rows [x L + h LP, + LP) of its lines
// x in order, one row per lane (T threads, LP rows: lanes >= LP idle) or two (RPL = 2)
template <bool NT, int RPL, int T, int MODE = 0, int NBAR = 0>
__global__ __launch_bounds__(T) void k_walk(const double *__restrict__ V, int64_t n, int L, int H,
                                            double *__restrict__ o0, double *__restrict__ o1) {
    const int LP = L / H, X = (int)(n / L);
    const int b = blockIdx.x, R = (int)gridDim.x / H, rb = b / H, h = b % H;
    const int xa = (int)((int64_t)rb * X / R), xb = (int)((int64_t)(rb + 1) * X / R);
    const int t = threadIdx.x;
    const int nl = xb - xa;
    const int rot = MODE == 1 ? (int)(((int64_t)rb * 7919) % (nl > 0 ? nl : 1)) : 0;
    const int nit = MODE == 2 ? (X - rb + R - 1) / R : (MODE >= 8 ? X / R : nl);
    for (int it = 0; it < nit; ++it) {
        // MODE 0: lines xa.. in order; 1: the same range from a per-range rotated start (wraps);
        // 2: lines rb, rb + R, ... (interleaved over ranges); K = MODE >= 8: chunks of K lines,
        // chunk c of range rb = lines (c R + rb) K ..
        int x = MODE == 2 ? rb + it * R : xa + (it + rot) % nl;
        if (MODE >= 8) x = ((it / MODE) * R + rb) * MODE + it % MODE;
        if (x >= X) break;
        const int64_t row0 = (int64_t)x * L + h * LP;
        if constexpr (RPL == 1) {
            if (t < LP) {
                const int64_t i = row0 + t;
                double a = 0.0, c = 0.0;
#pragma unroll
                for (int k = 0; k < NV; ++k) {
                    const double v = ld<NT>(V + (size_t)k * LDV + i);
                    a += v;
                    c -= v;
                }
                __builtin_nontemporal_store(a, o0 + i);
                __builtin_nontemporal_store(c, o1 + i);
            }
#pragma unroll
            for (int q = 0; q < NBAR; ++q) __syncthreads();   // the band step's barriers per line
        } else {
            if (2 * t < LP) {
                const int64_t i = (row0 >> 1) + t;
                double ax = 0.0, ay = 0.0, bx = 0.0, by = 0.0;
#pragma unroll
                for (int k = 0; k < NV; ++k) {
                    const double2 v = ld2<NT>(reinterpret_cast<const double2 *>(V + (size_t)k * LDV) + i);
                    ax += v.x;
                    ay += v.y;
                    bx -= v.x;
                    by -= v.y;
                }
                double2 *p0 = reinterpret_cast<double2 *>(o0) + i, *p1 = reinterpret_cast<double2 *>(o1) + i;
                __builtin_nontemporal_store(ax, &p0->x);
                __builtin_nontemporal_store(ay, &p0->y);
                __builtin_nontemporal_store(bx, &p1->x);
                __builtin_nontemporal_store(by, &p1->y);
            }
        }
    }
}

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? std::atoll(argv[1]) : 20000000;
    const int L = 800, H = 2;
    int dev = 0, ncu = 0;
    CHK(hipGetDevice(&dev));
    CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    double *V, *o0, *o1;
    const int64_t pad = argc > 2 ? std::atoll(argv[2]) : 0;
    const int64_t ldv = n + pad;
    CHK(hipMemcpyToSymbol(HIP_SYMBOL(LDV), &ldv, sizeof ldv));
    std::printf("n %lld pad %lld doubles\n", (long long)n, (long long)pad);
    CHK(hipMalloc(&V, sizeof(double) * NV * ldv));
    CHK(hipMalloc(&o0, sizeof(double) * n));
    CHK(hipMalloc(&o1, sizeof(double) * n));
    CHK(hipMemset(V, 0, sizeof(double) * NV * ldv));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const double bytes = 8.0 * n * (NV + 2);
    const int X = (int)(n / L);
    auto run = [&](const char *name, auto launch) {
        launch();
        CHK(hipDeviceSynchronize());
        std::vector<float> ts;
        for (int r = 0; r < 7; ++r) {
            CHK(hipEventRecord(e0));
            launch();
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        std::printf("%-28s %8.1f us  %7.1f GB/s\n", name, 1e3 * ts[3], bytes / (1e-3 * ts[3]) / 1e9);
        std::fflush(stdout);
    };
    const int g = ncu * 8;
    run("gridstride 8B nt", [&] { hipLaunchKernelGGL((k_rows8<true>), dim3(g), dim3(256), 0, 0, V, n, o0, o1); });
    run("gridstride 8B plain", [&] { hipLaunchKernelGGL((k_rows8<false>), dim3(g), dim3(256), 0, 0, V, n, o0, o1); });
    run("gridstride 16B nt", [&] { hipLaunchKernelGGL((k_rows16<true>), dim3(g), dim3(256), 0, 0, V, n, o0, o1); });
    run("gridstride 16B plain", [&] { hipLaunchKernelGGL((k_rows16<false>), dim3(g), dim3(256), 0, 0, V, n, o0, o1); });
    for (int wpc : {2, 4}) {
        int R = wpc * ncu / H;
        if (R > X / 2) R = X / 2;
        char nm[64];
        std::snprintf(nm, sizeof nm, "walk 8B nt T448 %d/CU", wpc);
        run(nm, [&] { hipLaunchKernelGGL((k_walk<true, 1, 448>), dim3(R * H), dim3(448), 0, 0, V, n, L, H, o0, o1); });
        std::snprintf(nm, sizeof nm, "walk 8B plain T448 %d/CU", wpc);
        run(nm, [&] { hipLaunchKernelGGL((k_walk<false, 1, 448>), dim3(R * H), dim3(448), 0, 0, V, n, L, H, o0, o1); });
        std::snprintf(nm, sizeof nm, "walk 16B nt T256 %d/CU", wpc);
        run(nm, [&] { hipLaunchKernelGGL((k_walk<true, 2, 256>), dim3(R * H), dim3(256), 0, 0, V, n, L, H, o0, o1); });
        std::snprintf(nm, sizeof nm, "walk 16B plain T256 %d/CU", wpc);
        run(nm, [&] { hipLaunchKernelGGL((k_walk<false, 2, 256>), dim3(R * H), dim3(256), 0, 0, V, n, L, H, o0, o1); });
    }
    for (int wpc : {2}) {
        const int R = wpc * ncu / H;
        run("walk 8B nt T448 rotated", [&] { hipLaunchKernelGGL((k_walk<true, 1, 448, 1>), dim3(R * H), dim3(448), 0, 0, V, n, L, H, o0, o1); });
        run("walk 8B nt T448 interleaved", [&] { hipLaunchKernelGGL((k_walk<true, 1, 448, 2>), dim3(R * H), dim3(448), 0, 0, V, n, L, H, o0, o1); });
        run("walk 16B nt T256 rotated", [&] { hipLaunchKernelGGL((k_walk<true, 2, 256, 1>), dim3(R * H), dim3(256), 0, 0, V, n, L, H, o0, o1); });
        run("walk 8B nt T448 1 barrier", [&] { hipLaunchKernelGGL((k_walk<true, 1, 448, 0, 1>), dim3(R * H), dim3(448), 0, 0, V, n, L, H, o0, o1); });
        run("walk 8B nt T448 3 barriers", [&] { hipLaunchKernelGGL((k_walk<true, 1, 448, 0, 3>), dim3(R * H), dim3(448), 0, 0, V, n, L, H, o0, o1); });
        run("walk 8B nt T448 chunk 8", [&] { hipLaunchKernelGGL((k_walk<true, 1, 448, 8>), dim3(R * H), dim3(448), 0, 0, V, n, L, H, o0, o1); });
        run("walk 8B nt T448 chunk 16", [&] { hipLaunchKernelGGL((k_walk<true, 1, 448, 16>), dim3(R * H), dim3(448), 0, 0, V, n, L, H, o0, o1); });
        run("walk 8B nt T448 chunk 32", [&] { hipLaunchKernelGGL((k_walk<true, 1, 448, 32>), dim3(R * H), dim3(448), 0, 0, V, n, L, H, o0, o1); });
        run("walk 8B nt T448 chunk 48", [&] { hipLaunchKernelGGL((k_walk<true, 1, 448, 48>), dim3(R * H), dim3(448), 0, 0, V, n, L, H, o0, o1); });
        run("walk 16B nt T256 interleaved", [&] { hipLaunchKernelGGL((k_walk<true, 2, 256, 2>), dim3(R * H), dim3(256), 0, 0, V, n, L, H, o0, o1); });
    }
    CHK(hipFree(V));
    CHK(hipFree(o0));
    CHK(hipFree(o1));
    return 0;
}
