// probe_c4.hip — where the C4 SpMV time goes.  Synthetic uniform-width SELL-64 (W entries per
// row, column = row + off[k], offsets compile-time, no code words) with fp32 or fp64 values;
// x padded by the largest offset on both sides (no periodic wrap).  Times y = A x for several
// offset sets: the 4D Vlasov stencil (0, +-1, +-40, +-2000, +-250000), the same with the far
// couplings made local, and a purely local 9-point band; 1 or 2 rows per lane.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe_c4.hip -o tools/bin/probe_c4
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int NT = 256;

struct Offs { int o[16]; };

// one lane per row (RPL = 1) or two rows per lane (RPL = 2: rows 128q + lane and 128q + 64 + lane)
template <typename VT, int W, int RPL, int SWZ>
__global__ __launch_bounds__(NT) void k_probe(const VT *__restrict__ val, const double *__restrict__ x,
                                              double *__restrict__ y, int64_t nch, Offs of) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t ngroups = nch / (4 * RPL);
    for (int64_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
        int64_t gg = g;
        if (SWZ) {   // XCD-contiguous: WGs on one XCD (b mod 8) walk a contiguous range of groups
            const int64_t per = (ngroups + 7) / 8;
            const int64_t it = g / gridDim.x, b = g % gridDim.x;
            const int64_t slot = it * (gridDim.x / 8) + b / 8;
            gg = (b % 8) * per + slot;
            if (gg >= ngroups) continue;
        }
#pragma unroll
        for (int r = 0; r < RPL; ++r) {
            const int64_t q = (gg * 4 + wv) * RPL + r;
            const int64_t row = 64 * q + lane;
            const VT *vv = val + q * 64 * W + lane;
            double d[W], xv[W];
#pragma unroll
            for (int k = 0; k < W; ++k) d[k] = (double)__builtin_nontemporal_load(vv + 64 * k);
#pragma unroll
            for (int k = 0; k < W; ++k) xv[k] = x[row + of.o[k]];
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < W; ++k) s += d[k] * xv[k];
            __builtin_nontemporal_store(s, y + row);
        }
    }
}

// column forms of the library's SELL chunks: CODED = 4-bit codes (ceil(W/8) words per lane)
// decoded through the chunk's 16-entry dictionary by ds_bpermute; DIAG = the dictionary's sorted
// offsets read by scalar loads (wave-uniform), one presence-mask word per lane, column = row +
// offset (slot k of every row holds offset dict[k])
template <typename VT, int W, int FORM>
__global__ __launch_bounds__(NT) void k_form(const VT *__restrict__ val, const uint32_t *__restrict__ pk,
                                             const int *__restrict__ dict, const double *__restrict__ x,
                                             double *__restrict__ y, int64_t nch) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t ngroups = nch / 4;
    for (int64_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
        const int q = __builtin_amdgcn_readfirstlane((int)(g * 4 + wv));
        const int64_t row = 64 * (int64_t)q + lane;
        const VT *vv = val + (int64_t)q * 64 * W + lane;
        double d[W], xv[W];
        double s = 0.0;
        if constexpr (FORM == 0) {   // CODED
            constexpr int NWD = (W + 7) / 8;
            uint32_t wd[NWD];
#pragma unroll
            for (int u = 0; u < NWD; ++u) wd[u] = __builtin_nontemporal_load(pk + (int64_t)q * 64 * NWD + u * 64 + lane);
            const int dv = lane < 16 ? dict[(int64_t)q * 16 + lane] : 0;
            int c[W];
#pragma unroll
            for (int k = 0; k < W; ++k) {
                const int code = (int)((wd[k >> 3] >> (4 * (k & 7))) & 15u);
                const int off = __shfl(dv, code, 64);
                c[k] = code != 15 ? (int)row + off : -1;
            }
#pragma unroll
            for (int k = 0; k < W; ++k) d[k] = (double)__builtin_nontemporal_load(vv + 64 * k);
#pragma unroll
            for (int k = 0; k < W; ++k) xv[k] = c[k] >= 0 ? x[c[k]] : 0.0;
#pragma unroll
            for (int k = 0; k < W; ++k)
                if (c[k] >= 0) s += d[k] * xv[k];
        } else {   // DIAG
            const uint32_t m = __builtin_nontemporal_load(pk + (int64_t)q * 64 + lane);
            const int *dq = dict + (int64_t)q * 16;
            int off[W];
#pragma unroll
            for (int k = 0; k < W; ++k) off[k] = __builtin_amdgcn_readfirstlane(dq[k]);
#pragma unroll
            for (int k = 0; k < W; ++k) d[k] = (double)__builtin_nontemporal_load(vv + 64 * k);
#pragma unroll
            for (int k = 0; k < W; ++k) xv[k] = x[((m >> k) & 1u) ? row + off[k] : row];
#pragma unroll
            for (int k = 0; k < W; ++k)
                if ((m >> k) & 1u) s += d[k] * xv[k];
        }
        __builtin_nontemporal_store(s, y + row);
    }
}

template <typename VT, int W, int FORM>
static void run_form(const char *name, const int *offs, int64_t n, int64_t pad, int grid, int reps) {
    const int64_t nch = n / 64;
    constexpr int NWD = FORM == 0 ? (W + 7) / 8 : 1;
    VT *val;
    double *xb, *y;
    uint32_t *pk;
    int *dict;
    CK(hipMalloc(&val, (size_t)n * W * sizeof(VT)));
    CK(hipMalloc(&xb, (size_t)(n + 2 * pad) * sizeof(double)));
    CK(hipMalloc(&y, (size_t)n * sizeof(double)));
    CK(hipMalloc(&pk, (size_t)n * NWD * sizeof(uint32_t)));
    CK(hipMalloc(&dict, (size_t)nch * 16 * sizeof(int)));
    CK(hipMemset(val, 0, (size_t)n * W * sizeof(VT)));
    CK(hipMemset(xb, 0, (size_t)(n + 2 * pad) * sizeof(double)));
    {
        std::vector<int> dh((size_t)nch * 16, 0);
        for (int64_t q = 0; q < nch; ++q)
            for (int k = 0; k < W; ++k) dh[(size_t)q * 16 + k] = offs[k];
        CK(hipMemcpy(dict, dh.data(), dh.size() * sizeof(int), hipMemcpyHostToDevice));
        uint32_t w0 = 0;   // CODED: code k in slot k; DIAG: every slot present
        if (FORM == 0) {
            std::vector<uint32_t> ph((size_t)n * NWD);
            for (int u = 0; u < NWD; ++u) {
                uint32_t w = 0xFFFFFFFFu;
                for (int k = 8 * u; k < W && k < 8 * u + 8; ++k) w = (w & ~(15u << (4 * (k & 7)))) | ((uint32_t)k << (4 * (k & 7)));
                for (int64_t q = 0; q < nch; ++q)
                    for (int l = 0; l < 64; ++l) ph[(size_t)q * 64 * NWD + u * 64 + l] = w;
            }
            CK(hipMemcpy(pk, ph.data(), ph.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        } else {
            w0 = (1u << W) - 1;
            std::vector<uint32_t> ph((size_t)n, w0);
            CK(hipMemcpy(pk, ph.data(), ph.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        }
    }
    const double *x = xb + pad;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_form<VT, W, FORM>), dim3(grid), dim3(NT), 0, 0, val, pk, dict, x, y, nch);
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_form<VT, W, FORM>), dim3(grid), dim3(NT), 0, 0, val, pk, dict, x, y, nch);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    const double bytes = (double)n * W * sizeof(VT) + 16.0 * n + 4.0 * n * NWD + 64.0 * nch;
    printf("%-28s W=%d %s %s grid=%5d: %8.1f us  %7.0f GB/s (val+codes+x+y)\n", name, W,
           sizeof(VT) == 4 ? "f32" : "f64", FORM == 0 ? "CODED" : "DIAG ", grid, us, bytes / us / 1e3);
    CK(hipFree(val));
    CK(hipFree(xb));
    CK(hipFree(y));
    CK(hipFree(pk));
    CK(hipFree(dict));
}

// the real 4D row structure (wraps replaced by the padded x): rows at the
// velocity boundaries (jvy = 0 / 39, jvx = 0 / 49) lack their -1 / +1 / -40 / +40 entries, so in
// the stored-order SELL layout the later entries of those lanes shift by one slot (CODED: their
// gathers leave the chunk's contiguous 512-B run); DIAG keeps slot k = offset k, absent = mask bit
template <typename VT, int FORM>
static void run_real(const char *name, int64_t n, int64_t pad, int grid, int reps) {
    constexpr int W = 9;
    const int64_t nch = n / 64;
    constexpr int NWD = FORM == 0 ? 2 : 1;
    const int offs[9] = {-250000, -2000, -40, -1, 0, 1, 40, 2000, 250000};
    std::vector<uint32_t> ph((size_t)n * NWD);
    std::vector<int> dh((size_t)nch * 16, 0);
    for (int64_t q = 0; q < nch; ++q) {
        for (int k = 0; k < 9; ++k) dh[(size_t)q * 16 + k] = offs[k];
        for (int l = 0; l < 64; ++l) {
            const int64_t r = 64 * q + l;
            const int jvy = (int)(r % 40), jvx = (int)((r / 40) % 50);
            bool pres[9];
            for (int k = 0; k < 9; ++k) pres[k] = true;
            pres[3] = jvy > 0; pres[5] = jvy < 39; pres[2] = jvx > 0; pres[6] = jvx < 49;
            if (FORM == 0) {
                uint32_t w[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};
                int e = 0;
                for (int k = 0; k < 9; ++k) {
                    if (!pres[k]) continue;
                    w[e >> 3] = (w[e >> 3] & ~(15u << (4 * (e & 7)))) | ((uint32_t)k << (4 * (e & 7)));
                    ++e;
                }
                ph[(size_t)q * 64 * 2 + l] = w[0];
                ph[(size_t)q * 64 * 2 + 64 + l] = w[1];
            } else {
                uint32_t m = 0;
                for (int k = 0; k < 9; ++k) m |= pres[k] ? 1u << k : 0u;
                ph[(size_t)q * 64 + l] = m;
            }
        }
    }
    VT *val;
    double *xb, *y;
    uint32_t *pk;
    int *dict;
    CK(hipMalloc(&val, (size_t)n * W * sizeof(VT)));
    CK(hipMalloc(&xb, (size_t)(n + 2 * pad) * sizeof(double)));
    CK(hipMalloc(&y, (size_t)n * sizeof(double)));
    CK(hipMalloc(&pk, ph.size() * sizeof(uint32_t)));
    CK(hipMalloc(&dict, dh.size() * sizeof(int)));
    CK(hipMemset(val, 0, (size_t)n * W * sizeof(VT)));
    CK(hipMemset(xb, 0, (size_t)(n + 2 * pad) * sizeof(double)));
    CK(hipMemcpy(pk, ph.data(), ph.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    CK(hipMemcpy(dict, dh.data(), dh.size() * sizeof(int), hipMemcpyHostToDevice));
    const double *x = xb + pad;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_form<VT, W, FORM>), dim3(grid), dim3(NT), 0, 0, val, pk, dict, x, y, nch);
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_form<VT, W, FORM>), dim3(grid), dim3(NT), 0, 0, val, pk, dict, x, y, nch);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    const double bytes = (double)n * W * sizeof(VT) + 16.0 * n + 4.0 * n * NWD + 64.0 * nch;
    printf("%-28s W=%d %s %s grid=%5d: %8.1f us  %7.0f GB/s (val+codes+x+y)\n", name, W,
           sizeof(VT) == 4 ? "f32" : "f64", FORM == 0 ? "CODED" : "DIAG ", grid, us, bytes / us / 1e3);
    CK(hipFree(val));
    CK(hipFree(xb));
    CK(hipFree(y));
    CK(hipFree(pk));
    CK(hipFree(dict));
}

template <typename VT, int W, int RPL, int SWZ>
static void run(const char *name, const Offs &of, int64_t n, int64_t pad, int grid, int reps) {
    const int64_t nch = n / 64;
    VT *val;
    double *xb, *y;
    CK(hipMalloc(&val, (size_t)n * W * sizeof(VT)));
    CK(hipMalloc(&xb, (size_t)(n + 2 * pad) * sizeof(double)));
    CK(hipMalloc(&y, (size_t)n * sizeof(double)));
    CK(hipMemset(val, 0, (size_t)n * W * sizeof(VT)));
    CK(hipMemset(xb, 0, (size_t)(n + 2 * pad) * sizeof(double)));
    const double *x = xb + pad;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_probe<VT, W, RPL, SWZ>), dim3(grid), dim3(NT), 0, 0, val, x, y, nch, of);
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_probe<VT, W, RPL, SWZ>), dim3(grid), dim3(NT), 0, 0, val, x, y, nch, of);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    const double bytes = (double)n * W * sizeof(VT) + 16.0 * n;
    printf("%-28s W=%d %s RPL=%d SWZ=%d grid=%5d: %8.1f us  %7.0f GB/s (val+x+y)\n", name, W,
           sizeof(VT) == 4 ? "f32" : "f64", RPL, SWZ, grid, us, bytes / us / 1e3);
    CK(hipFree(val));
    CK(hipFree(xb));
    CK(hipFree(y));
}

int main(int argc, char **argv) {
    const int64_t n = 50'000'000 / 512 * 512;   // whole groups of 2 x 4 x 64 rows
    const int64_t pad = 262144;
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    const Offs c4{{-250000, -2000, -40, -1, 0, 1, 40, 2000, 250000}};
    const Offs c4near{{-2048, -2000, -40, -1, 0, 1, 40, 2000, 2048}};
    const Offs band{{-4, -3, -2, -1, 0, 1, 2, 3, 4}};
    const Offs diag{{0, 0, 0, 0, 0, 0, 0, 0, 0}};
    const Offs c3{{-800, -1, 0, 1, 800}};
    const int c4o[9] = {-250000, -2000, -40, -1, 0, 1, 40, 2000, 250000};
    const int c3o[5] = {-800, -1, 0, 1, 800};
    for (int grid : {1024, 2048}) {
        run_real<float, 0>("c4 real rows", n, pad, grid, reps);
        run_real<float, 1>("c4 real rows", n, pad, grid, reps);
    }
    if (argc > 2) return 0;
    for (int grid : {1024, 2048}) {
        run_form<float, 9, 0>("c4 stencil", c4o, n, pad, grid, reps);
        run_form<float, 9, 1>("c4 stencil", c4o, n, pad, grid, reps);
        run_form<double, 5, 0>("c3 stencil (n=50M)", c3o, n, pad, grid, reps);
        run_form<double, 5, 1>("c3 stencil (n=50M)", c3o, n, pad, grid, reps);
    }
    for (int grid : {1024, 2048, 4096}) {
        run<float, 9, 1, 0>("c4 stencil", c4, n, pad, grid, reps);
    }
    run<float, 9, 1, 1>("c4 stencil", c4, n, pad, 2048, reps);
    run<float, 9, 2, 0>("c4 stencil", c4, n, pad, 2048, reps);
    run<float, 9, 1, 0>("c4, far -> +-2048", c4near, n, pad, 2048, reps);
    run<float, 9, 1, 0>("9-band", band, n, pad, 2048, reps);
    run<float, 9, 1, 0>("9 x diagonal", diag, n, pad, 2048, reps);
    run<double, 9, 1, 0>("c4 stencil", c4, n, pad, 2048, reps);
    run<double, 9, 1, 0>("9-band", band, n, pad, 2048, reps);
    run<double, 5, 1, 0>("c3 stencil (n=50M)", c3, n, pad, 2048, reps);
    run<float, 5, 1, 0>("c3 stencil (n=50M)", c3, n, pad, 2048, reps);
    return 0;
}
