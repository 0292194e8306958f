// vtk_scalar.hpp — the DCGS2 scalar step (SciPy's Givens / stop logic on the reduced dots) as a
// device function: run by k_dc_scalar (one 1024-thread workgroup) and by the last-arriving
// workgroup of the line-band step ("scalar step in the band step's tail").
// Built with -ffp-contract=off in every translation unit: the same bits either way.
#pragma once
#include <hip/hip_runtime.h>

#include <float.h>

#include "vtk_device.hpp"

namespace vtk {

// ------------------------------------------------------------------------------------------
// LAPACK 3.10+ dlartg (the lartg SciPy calls, iterative.py:779)
// ------------------------------------------------------------------------------------------
static __device__ void d_lartg(double f, double g, double &c, double &s, double &r) {
    const double safmin = DBL_MIN;
    const double safmax = 1.0 / DBL_MIN;
    const double rtmin = __builtin_sqrt(safmin);
    const double rtmax = __builtin_sqrt(safmax / 2.0);
    const double f1 = __builtin_fabs(f), g1 = __builtin_fabs(g);
    if (g == 0.0) {
        c = 1.0; s = 0.0; r = f;
    } else if (f == 0.0) {
        c = 0.0; s = __builtin_copysign(1.0, g); r = g1;
    } else if (f1 > rtmin && f1 < rtmax && g1 > rtmin && g1 < rtmax) {
        const double d = __builtin_sqrt(f * f + g * g);
        c = f1 / d;
        r = __builtin_copysign(d, f);
        s = g / r;
    } else {
        double u = f1 > g1 ? f1 : g1;
        if (u < safmin) u = safmin;
        if (u > safmax) u = safmax;
        const double fs = f / u, gs = g / u;
        const double d = __builtin_sqrt(fs * fs + gs * gs);
        c = __builtin_fabs(fs) / d;
        const double rr = __builtin_copysign(d, f);
        s = gs / rr;
        r = rr * u;
    }
}

// the scalar step's LDS (k_dc_scalar: static; the band step: carved from its sweep buffers)
struct DcScalarLds {
    double q[DC_NQ];
    double hr_s[(DC_MAXJ + 1) * (DC_MAXJ + 1)];
    double giv_s[2 * DC_MAXJ];
    double S_s[DC_MAXJ + 2], hc_s[DC_MAXJ + 2], hj[DC_MAXJ + 2], e_s[DC_MAXJ + 2];
    double sc[8];   // ptol, nu(prev), h0(prev), r, sz
    int flags[2];   // committed(prev), done
};

// the quantities of step j (s_k, z_k k < j; alpha, beta, gamma; j + 1 of them when closing) from
// the G partials in the launch_dc_dots layout: each quantity by one wave, lane-strided partial
// sums in a fixed order then the wave's butterfly -- the same bits for any workgroup size.  A
// wave takes QW quantities per round and issues all their loads before any add.  SC1: the
// partials were handed over by agent-scope (sc1) stores of other workgroups of the same launch
// (the band step's tail); load them the same way
template <bool SC1, int QW>
__device__ __forceinline__ void dc_sum_partials(double *q, const double *part, int cnt, int j, int with_w) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int nq = with_w ? 2 * j + 3 : j + 1;
    auto qslot = [&](int b) {
        if (b < j) return b;
        if (with_w && b < 2 * j) return DC_MAXJ + (b - j);
        return 2 * DC_MAXJ + (b - (with_w ? 2 * j : j));
    };
    constexpr int PL = GMAX / 64;
    for (int b0 = wv; b0 < nq; b0 += QW * nw) {
        double v[QW][PL];
#pragma unroll
        for (int h = 0; h < QW; ++h) {
            const int b = b0 + h * nw;
            const double *pp = part + (size_t)(b < nq ? qslot(b) : 0) * GMAX;
#pragma unroll
            for (int u = 0; u < PL; ++u) {
                const int i = lane + u * 64;
                double x = 0.0;
                if (b < nq && i < cnt) {
                    if constexpr (SC1) x = __hip_atomic_load(pp + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    else x = pp[i];
                }
                v[h][u] = x;
            }
        }
#pragma unroll
        for (int h = 0; h < QW; ++h) {
            const int b = b0 + h * nw;
            double acc = 0.0;
#pragma unroll
            for (int u = 0; u < PL; ++u) acc += v[h][u];
            acc = wave_sum(acc);
            if (b < nq && lane == 0) q[qslot(b)] = acc;
        }
    }
}

// Scalar step of DCGS2 step j (lane 0 does the O(j^2) algebra from LDS):
//  * quantities: reduced here from the G partials (one GPU) or read from scal (all-reduced);
//  * j >= 1: re-orthogonalisation scalars of p_j, finalise column j-1 (h += nu s,
//    h_{j,j-1} = nu r) unless it was already committed, SciPy's Givens/stop logic on it
//    (iterative.py:761-794);
//  * closing == 0: tentative column j and the update-pass coefficients; the column is committed
//    at once (Givens, stop test) when its estimate is numerically safe — no cancellation in
//    nu (nu > 1e-3 ||Bv||) and presid not within 1e-8 of ptol — or it is the cycle's last
//    column; otherwise it is finalised exactly by step j+1.
// TR: phase marks for tools/probe_scalar.hip (the product's ScalarNoTrace marks nothing)
struct ScalarNoTrace {
    __device__ __forceinline__ void mark(int) const {}
};
template <bool SC1, int QW, class TR = ScalarNoTrace>
__device__ __forceinline__ void dc_scalar_body(DcScalarLds &sl, const double *part, int cnt, const double *scal,
                                               int j, int m, int closing, double *Hraw, double *H, double *S,
                                               double *giv, DcCoef *cf, GmresState *st, int *stop_map,
                                               TR tr = TR{}) {
    double *const q = sl.q, *const hr_s = sl.hr_s, *const giv_s = sl.giv_s, *const S_s = sl.S_s;
    double *const hc_s = sl.hc_s, *const hj = sl.hj, *const e_s = sl.e_s, *const sc = sl.sc;
    int *const flags = sl.flags;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    tr.mark(0);
    if (st->stop_col < j) return;
    tr.mark(1);
    // across ranks (scal all-reduced): a rank voted failure in this step's all-reduce -- every
    // rank stops the cycle here, at the same step, with no x update (vtk_gmres returns an error)
    if (!part && scal[DC_VOTE] != 0.0) {
        if (tid == 0) {
            st->breakdown = PEER_FAILED;
            st->stop_col = j - 1;
            st->xup_tag = -1;
            if (stop_map) __hip_atomic_store(stop_map, j - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return;
    }
    const int with_w = closing ? 0 : 1;
    const int nq = with_w ? 2 * j + 3 : j + 1;
    const int M1 = m + 1;
    // phase A: quantities, raw Hessenberg columns 0..j-1, rotations, S, scalars -> LDS.  A wave
    // takes up to three quantities per round and issues all their partial loads before any add
    // (one memory round trip for j <= 22 instead of one per quantity)
    auto qslot = [&](int b) {
        if (b < j) return b;
        if (with_w && b < 2 * j) return DC_MAXJ + (b - j);
        return 2 * DC_MAXJ + (b - (with_w ? 2 * j : j));
    };
    if (part) {
        dc_sum_partials<SC1, QW>(q, part, cnt, j, with_w);
    } else {
        for (int b = tid; b < nq; b += blockDim.x) q[qslot(b)] = scal[qslot(b)];
    }
    for (int e = tid; e < j * (j + 1); e += blockDim.x) {
        const int i = e / (j + 1), k = e % (j + 1);
        hr_s[i * (DC_MAXJ + 1) + k] = Hraw[(size_t)i * M1 + k];
    }
    for (int e = tid; e < 2 * j; e += blockDim.x) giv_s[e] = giv[e];
    for (int e = tid; e <= m && e < DC_MAXJ + 2; e += blockDim.x) S_s[e] = S[e];
    if (tid == 0) {
        sc[0] = st->ptol;
        sc[1] = j >= 1 ? cf->nu : 0.0;
        sc[2] = j >= 1 ? cf->h0[j - 1] : 0.0;
        flags[0] = j >= 1 ? cf->committed[j - 1] : 1;
        flags[1] = 0;
    }
    __syncthreads();
    tr.mark(2);
    const double *sv = q, *zv = q + DC_MAXJ;
    const double alpha = q[2 * DC_MAXJ], beta = q[2 * DC_MAXJ + 1], gamma = q[2 * DC_MAXJ + 2];
    const double ptol = sc[0];
    // Givens + stop test on the LDS column hc_s (rows 0..c+1), SciPy's order; the rotated
    // column, S and the rotation go to global memory once
    auto rotate_commit = [&](int c, bool brk) -> bool {
        double *hc = hc_s;
        // the running element stays in a register: only the loads of hc[k+1] and the rotation
        // (independent of the chain) touch LDS
        double cur = hc[0];
#pragma unroll 4
        for (int k = 0; k < c; ++k) {
            const double cg = giv_s[2 * k], sg = giv_s[2 * k + 1];
            const double n1 = hc[k + 1];
            hc[k] = cg * cur + sg * n1;
            cur = -sg * cur + cg * n1;
        }
        hc[c] = cur;
        double cg, sg, mag;
        d_lartg(hc[c], hc[c + 1], cg, sg, mag);
        giv_s[2 * c] = cg;
        giv_s[2 * c + 1] = sg;
        giv[2 * c] = cg;
        giv[2 * c + 1] = sg;
        hc[c] = mag;
        hc[c + 1] = 0.0;
        double *hg = H + (size_t)c * M1;
        for (int k = 0; k <= c + 1; ++k) hg[k] = hc[k];
        const double t = -sg * S_s[c];
        S_s[c] = cg * S_s[c];
        S_s[c + 1] = t;
        S[c] = S_s[c];
        S[c + 1] = t;
        const double presid = __builtin_fabs(t);
        st->presid = presid;
        st->inner += 1;
        if (presid <= ptol || brk) {
            st->breakdown = brk ? 1 : 0;
            st->stop_col = c;
            if (!closing) st->xup_tag = j;   // this step's update pass does the x update
            if (stop_map) __hip_atomic_store(stop_map, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return true;
        }
        return false;
    };
    // phase B1 (wave 0, lane k): r and column j-1 final (h += nu s, h_{j,j-1} = nu r) in parallel;
    // the dots as butterfly sums (fixed tree, the same bits in every lane)
    const bool fin_prev = j >= 1 && !flags[0];
    if (wv == 0) {
        const double svk = lane < j ? sv[lane] : 0.0, zvk = lane < j ? zv[lane] : 0.0;
        const double ss = wave_allsum(svk * svk), sz = wave_allsum(svk * zvk);
        double r = 1.0;
        if (j >= 1) {
            const double r2 = alpha - ss;
            r = __builtin_sqrt(r2 > 0.0 ? r2 : alpha);
        }
        if (lane == 0) {
            sc[3] = r;
            sc[4] = sz;
        }
        if (fin_prev && lane <= j) {
            const int c = j - 1;
            double *hr = hr_s + c * (DC_MAXJ + 1);
            const double v = lane < j ? hr[lane] + sc[1] * sv[lane] : sc[1] * r;
            hr[lane] = v;
            Hraw[(size_t)c * M1 + lane] = v;
            hc_s[lane] = v;
        }
    }
    __syncthreads();
    tr.mark(3);
    // phase B2 (lane 0): breakdown test, Givens and stop test of column j-1
    if (tid == 0) {
        if (fin_prev) {
            const int c = j - 1;
            const bool brk = hc_s[j] <= DBL_EPSILON * sc[2];
            if (brk) hc_s[j] = 0.0;
            cf->committed[c] = 1;
            if (rotate_commit(c, brk)) flags[1] = 1;
        }
        if (closing) flags[1] = 1;
    }
    __syncthreads();
    tr.mark(4);
    if (flags[1]) return;
    // phase C (lanes k <= j): tentative column j, c'_k = (e_k - (H_j s)_k) / r, with the raw
    // columns i < j final; row k of column i is nonzero for i >= k-1
    const double r = sc[3];
    if (tid <= j) {
        const int k = tid;
        const double e = k < j ? zv[k] : (beta - sc[4]) / r;
        double g = 0.0;
        for (int i = (k > 0 ? k - 1 : 0); i < j; ++i) g += hr_s[i * (DC_MAXJ + 1) + k] * sv[i];
        const double h = (e - g) / r;
        e_s[k] = e;
        hj[k] = h;
        Hraw[(size_t)j * M1 + k] = h;
        cf->e_prev[k] = cf->e[k];   // the line-band step's recompute of p_j (DcCoef::e_prev)
        cf->e[k] = e;
        if (k < j) cf->s[k] = sv[k];
    }
    __syncthreads();
    tr.mark(5);
    if (wv != 0) return;
    const double ek = lane <= j ? e_s[lane] : 0.0;
    const double ee = wave_allsum(ek * ek);
    if (lane != 0) return;
    // phase D (lane 0): nu_{j+1}, update-pass scalars, early commit when unambiguous
    cf->rinv = 1.0 / r;
    const double gn = __builtin_sqrt(gamma) / r;
    const double nu2 = gamma - ee;
    double nu = nu2 > 0.0 ? __builtin_sqrt(nu2) / r : 0.0;
    const bool safe = nu > 1e-3 * gn;
    if (!(nu > 1e-8 * gn)) nu = gn > 0.0 ? gn : 1.0;   // heavy cancellation: step j+1's r corrects
    cf->nu = nu;
    cf->h0[j] = gn;
    cf->q_prev = cf->q;
    cf->q = 1.0 / (r * nu);
    cf->committed[j] = 0;
    tr.mark(6);
    if (!safe) return;
    // trial rotation of the tentative column (only the last rotated entry is needed)
    double a0 = hj[0];
    for (int k = 0; k < j; ++k) a0 = -giv_s[2 * k + 1] * a0 + giv_s[2 * k] * hj[k + 1];
    double cg, sg, mag;
    d_lartg(a0, nu, cg, sg, mag);
    const double pres_t = __builtin_fabs(-sg * S_s[j]);
    const bool last = j == m - 1;
    if (!(last || pres_t <= ptol * (1.0 - 1e-8))) return;   // above or ambiguous: finalise exactly
    tr.mark(7);
    for (int k = 0; k <= j; ++k) hc_s[k] = hj[k];
    hc_s[j + 1] = nu;
    cf->committed[j] = 1;
    if (!rotate_commit(j, false) && last) {
        st->stop_col = j;   // cycle complete: later kernels of this cycle are no-ops
        st->xup_tag = j;
        if (stop_map) __hip_atomic_store(stop_map, j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    tr.mark(8);
}

}  // namespace vtk
