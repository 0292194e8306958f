// probe_scalar.hip — where the DCGS2 scalar step's time goes (vtk_scalar.hpp dc_scalar_body, the
// k_dc_scalar launch of every Arnoldi step): per step index j, the kernel's in-kernel phase times
// (wall_clock64 marks from thread 0) and the launch-to-launch time, on synthetic but well-formed
// state (orthonormal-ish partial sums, a committed / uncommitted previous column).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I vt-precondition_amd/csrc \
//         tools/probe_scalar.hip -o /tmp/probe_scalar && /tmp/probe_scalar [cnt] [reps]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

#include "vtk_scalar.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

using namespace vtk;

struct Marks {
    long long *t;
    __device__ __forceinline__ void mark(int i) const {
        if (threadIdx.x == 0) t[i] = wall_clock64();
    }
};

__global__ __launch_bounds__(1024) void k_probe(const double *part, int cnt, const double *scal, int j, int m,
                                                double *Hraw, double *H, double *S, double *giv, DcCoef *cf,
                                                GmresState *st, long long *t) {
    __shared__ DcScalarLds sl;
    for (int i = threadIdx.x; i < 9; i += blockDim.x) t[i] = 0;
    __syncthreads();
    dc_scalar_body<false, 3, Marks>(sl, part, cnt, scal, j, m, 0, Hraw, H, S, giv, cf, st, nullptr, Marks{t});
}

// launch geometry variants of the plain scalar kernel (no marks): NTH threads, QW quantities per
// wave per round -- back-to-back launch time is what the solver's chain pays
template <int NTH, int QW>
__global__ __launch_bounds__(NTH) void k_geo(const double *part, int cnt, const double *scal, int j, int m,
                                             double *Hraw, double *H, double *S, double *giv, DcCoef *cf,
                                             GmresState *st) {
    __shared__ DcScalarLds sl;
    dc_scalar_body<false, QW>(sl, part, cnt, scal, j, m, 0, Hraw, H, S, giv, cf, st, nullptr);
}

int main(int argc, char **argv) {
    const int cnt = argc > 1 ? std::atoi(argv[1]) : 512, reps = argc > 2 ? std::atoi(argv[2]) : 50;
    const int m = 20, M1 = m + 1;
    double *part, *scal, *Hraw, *H, *S, *giv;
    DcCoef *cf;
    GmresState *st;
    long long *t;
    CK(hipMalloc(&part, sizeof(double) * DC_NQ * GMAX));
    CK(hipMalloc(&scal, sizeof(double) * 256));
    CK(hipMalloc(&Hraw, sizeof(double) * M1 * M1));
    CK(hipMalloc(&H, sizeof(double) * M1 * M1));
    CK(hipMalloc(&S, sizeof(double) * (M1 + 1)));
    CK(hipMalloc(&giv, sizeof(double) * 2 * M1));
    CK(hipMalloc(&cf, sizeof(DcCoef)));
    CK(hipMalloc(&st, sizeof(GmresState)));
    CK(hipMalloc(&t, sizeof(long long) * 32));
    // partials: s_k small, z_k small, alpha ~ 1, beta, gamma ~ 1 (r, nu well away from cancellation)
    std::vector<double> hp((size_t)DC_NQ * GMAX, 0.0);
    for (int q = 0; q < DC_NQ; ++q)
        for (int b = 0; b < cnt; ++b) {
            double v = 1e-3 / cnt * (1.0 + 0.01 * ((q * 7 + b) % 13));
            if (q == 2 * DC_MAXJ) v = 1.0 / cnt;
            if (q == 2 * DC_MAXJ + 1) v = 0.3 / cnt;
            if (q == 2 * DC_MAXJ + 2) v = 1.0 / cnt;
            hp[(size_t)q * GMAX + b] = v;
        }
    std::vector<double> hH((size_t)M1 * M1), hS(M1 + 1, 0.0), hg(2 * M1);
    for (int i = 0; i < M1 * M1; ++i) hH[i] = 0.1 + 0.01 * (i % 7);
    hS[0] = 1.0;
    for (int k = 0; k < M1; ++k) { hg[2 * k] = std::cos(0.1 * k); hg[2 * k + 1] = std::sin(0.1 * k); }
    for (int k = 1; k < M1; ++k) hS[k] = 0.5 * hS[k - 1];
    DcCoef hc;
    std::memset(&hc, 0, sizeof hc);
    hc.nu = 0.9;
    hc.q = 1.1;
    for (int k = 0; k <= DC_MAXJ; ++k) { hc.h0[k] = 1.0; hc.e[k] = 0.01; hc.committed[k] = 0; }
    GmresState hs;
    std::memset(&hs, 0, sizeof hs);
    hs.ptol = 1e-300;
    hs.stop_col = BIG_COL;
    hs.xup_tag = -1;
    CK(hipMemcpy(part, hp.data(), hp.size() * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::printf("cnt %d reps %d; per j: median in-kernel phase times (us) a=stop_col load, b=quantities+state "
                "loads, c=B1, d=B2 (finalise col j-1), e=C, f=D head, g=trial, h=commit; tot; launch-to-launch\n", cnt, reps);
    for (int j = 0; j < m; ++j) {
        for (int committed = 0; committed < 2; ++committed) {
            std::vector<std::vector<double>> ph(9);
            float ms_sum = 0.f;
            for (int r = 0; r < reps; ++r) {
                hc.committed[j > 0 ? j - 1 : 0] = committed;
                CK(hipMemcpy(Hraw, hH.data(), hH.size() * 8, hipMemcpyHostToDevice));
                CK(hipMemcpy(H, hH.data(), hH.size() * 8, hipMemcpyHostToDevice));
                CK(hipMemcpy(S, hS.data(), hS.size() * 8, hipMemcpyHostToDevice));
                CK(hipMemcpy(giv, hg.data(), hg.size() * 8, hipMemcpyHostToDevice));
                CK(hipMemcpy(cf, &hc, sizeof hc, hipMemcpyHostToDevice));
                CK(hipMemcpy(st, &hs, sizeof hs, hipMemcpyHostToDevice));
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(k_probe, dim3(1), dim3(1024), 0, 0, part, cnt, scal, j, m, Hraw, H, S, giv, cf, st, t);
                hipLaunchKernelGGL(k_probe, dim3(1), dim3(1024), 0, 0, part, cnt, scal, j, m, Hraw, H, S, giv, cf, st, t + 9);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                ms_sum += ms;
                long long ht[18];
                CK(hipMemcpy(ht, t, sizeof ht, hipMemcpyDeviceToHost));
                for (int i = 1; i < 9; ++i) ph[i].push_back(ht[i] > 0 && ht[i - 1] > 0 ? (ht[i] - ht[i - 1]) * 0.01 : -1.0);
                ph[0].push_back(ht[8] > 0 ? (ht[8] - ht[0]) * 0.01 : (ht[6] - ht[0]) * 0.01);
            }
            std::printf("j %2d committed %d:", j, committed);
            for (int i = 1; i < 9; ++i) {
                std::sort(ph[i].begin(), ph[i].end());
                std::printf(" %6.2f", ph[i][ph[i].size() / 2]);
            }
            std::sort(ph[0].begin(), ph[0].end());
            std::printf(" | tot %6.2f | 2 launches %6.2f us\n", ph[0][ph[0].size() / 2], 1000.f * ms_sum / reps);
        }
    }
    // back-to-back launches (state reset once per batch; the path taken stays the uncommitted
    // one only for the first launch of a batch -- the later ones find column j-1 committed)
    std::printf("back-to-back: us per launch (100 launches), j: 1024x3  256x3  256x11  64x22\n");
    for (int j = 0; j < m; j += 3) {
        float us[4];
        for (int v = 0; v < 4; ++v) {
            hc.committed[j > 0 ? j - 1 : 0] = 0;
            CK(hipMemcpy(cf, &hc, sizeof hc, hipMemcpyHostToDevice));
            CK(hipMemcpy(st, &hs, sizeof hs, hipMemcpyHostToDevice));
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            for (int r = 0; r < 100; ++r) {
                if (v == 0) hipLaunchKernelGGL((k_geo<1024, 3>), dim3(1), dim3(1024), 0, 0, part, cnt, scal, j, m, Hraw, H, S, giv, cf, st);
                if (v == 1) hipLaunchKernelGGL((k_geo<256, 3>), dim3(1), dim3(256), 0, 0, part, cnt, scal, j, m, Hraw, H, S, giv, cf, st);
                if (v == 2) hipLaunchKernelGGL((k_geo<256, 11>), dim3(1), dim3(256), 0, 0, part, cnt, scal, j, m, Hraw, H, S, giv, cf, st);
                if (v == 3) hipLaunchKernelGGL((k_geo<64, 22>), dim3(1), dim3(64), 0, 0, part, cnt, scal, j, m, Hraw, H, S, giv, cf, st);
            }
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            us[v] = 10.f * ms;
        }
        std::printf("j %2d: %7.2f %7.2f %7.2f %7.2f\n", j, us[0], us[1], us[2], us[3]);
    }
    return 0;
}
