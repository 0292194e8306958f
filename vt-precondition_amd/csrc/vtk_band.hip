// vtk_band.hip — the line-band DCGS2 step and its ghost-line exchange and
// structure checks, gfx950.  Built with -ffp-contract=off like vtk_kernels.hip: the update,
// SpMV and block-Jacobi arithmetic is bit-identical to k_dc_update / k_sell.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "vtk_device.hpp"

namespace vtk {

// ------------------------------------------------------------------------------------------
// Line-band DCGS2 step.  For an operator whose rows form x-lines of L rows
// (row = x L + v) with every column in lines x-1, x, x+1 (periodic in x) at v-1..v+1 -- the 2D
// Vlasov operators, L = Nv -- the update pass of step j and the fused SpMV + BJ + dots of step
// j+1 run as ONE sweep.  Workgroup (range r, part h) owns rows v0 <= v < v0 + LP (LP = L / H)
// of the lines [xa, xb) of range r and walks them in order; at line x it
//   1. updates line x+1 on its rows plus one v-halo row on each side: recomputes p_j exactly as
//      step j-1 formed it, p_j = (w_{j-1} - sum_k e'_k V_k) q' (the previous step's scalars e',
//      q' in DcCoef::e_prev / q_prev; p_0 = v_0), then v_j and p_{j+1} as k_dc_update, and puts
//      p_{j+1}(x+1) into an LDS ring of 4 lines,
//   2. computes w(x) = M^-1 A p_{j+1} on its rows of line x from the ring (the SELL entries in
//      stored order and the tridiagonal BJ solve exactly as k_sell: w is bit-identical),
//   3. accumulates step j+1's dots s = V_{j+1}^T p_{j+1}, z = V_{j+1}^T w, |p|^2, p.w, |w|^2
//      from LDS: the line's basis rows were staged there by step 1 one line earlier.
// The basis is read from HBM once per step instead of twice (update pass + dots), p_{j+1} is
// neither stored (except by the last band step, whose successor is k_dc_update) nor re-read
// for the SpMV gathers, and one launch replaces two.  Rows another workgroup owns are
// recomputed from that row's own V_k, w_{j-1}, w_j: the x-halo lines xa-1 and xb and the v-halo
// rows v0-1, v0+LP -- no per-step boundary copies between workgroups.  w cycles through three
// buffers (w_{j-1}, w_j read, w_{j+1} written).  7 waves; lane tid <-> row v = v0 - 16 + tid
// (8-row BJ blocks stay lane-aligned); ~79 KB LDS: two workgroups per CU, whose update / SpMV /
// dots phases overlap.
// ------------------------------------------------------------------------------------------
// canonical line-band rows: canon_order (vtk_device.hpp)

// geometry: half lines (LP <= BAND_LP = 400 rows, 7 waves, ~79 KB LDS, two workgroups per CU).
// Quarter lines with the staged basis double-buffered and every step's next line prefetched
// (4 waves, 2-4 workgroups per CU by LDS) measured 2-10 % slower per step (round 5).
#define VTK_BAND_DOTS_UNROLL 2   // (a #pragma unroll literal) the dots' 64-row passes issued together
constexpr int BAND_XUP_XB = 4;     // the cycle's x update inlined into k_band_step, basis loads in batches of
                                   // this many (C3 x update 648-653 -> 641-643 us)
constexpr int BAND_PF = 12;        // j <= this: next line's update operands prefetched across SpMV + dots
                                   // (round 3: 10: 567-570 us; 8: 570; 12: 567; 18: 624, spills; with
                                   // the fused multiply-adds j <= 12 fits 124 VGPRs)

// VMODE 1 (LSV): the matrix values from the line-separable tables (vtk_csr::d_lsv: the diagonal
// per row, x +- 1 couplings per position v -- held in registers for the lane's v --, v +- 1
// couplings per line) instead of the SELL copy's 5 values per row; VMODE 2 (also canonical
// rows, vtk_csr::lsv_canon): the entries' kinds and order from canon_order instead of the SELL
// codes and dictionary.  The same values in the same order either way
// OPT bit 0 (SPF): with the next-line prefetch (J <= BAND_PF) and canonical rows, the SpMV
// operands of a line (D, m, the line's v couplings) travel in the same prefetch as the update
// operands, one line ahead.  Loaded at the head of their own iteration they made the wait for the
// prefetched update operands a wait for everything (s_waitcnt vmcnt(0): the loads sit in
// exec-masked blocks, so the counter cannot be tracked per load): one exposed memory round trip
// per line.
// OPT bit 1 (WPC3): registers capped for 3 workgroups per CU (6 waves per SIMD) -- the low-J
// launches, whose LDS (ring + (J + 1) staged basis rows) leaves room for a third workgroup and
// whose serial line walks are latency-bound; the host plans 1.5x the line ranges for them.
// The update's sums and the dots are fused multiply-adds (one rounding per term, half the f64
// VALU instructions of the separate multiply and add; C3 solve -1 %, round 5); p_j's recompute
// (here and in the x update's) is the same fused chain, so step j forms p_j exactly as step j-1
// did.  (k_dc_update keeps the unfused operations of the oracle's sequence.)
template <int OPT> constexpr int band_wpe() { return (OPT & 2) ? 6 : 4; }
// OPT bit 2 (XCDP, a runtime bit): the two parts of a line range on ONE XCD.  Each part updates
// one v-halo row on either side, which lies in the other part's rows: read alone, that row drags
// its whole 128-B line from HBM (the band step's PMC fetch is ~9 % over its algorithmic bytes at
// j >= 9).  Workgroups are dealt to the XCDs round-robin (blockIdx mod 8), so blockIdx b and b + 8
// share an XCD's L2: logical block (range, part) = (8 (b / 16) + b mod 8, (b / 8) mod 2).  The
// logical index also names the workgroup's partial slot, so the dots' sums keep their bits.
__device__ __forceinline__ int band_block(int opt, int H) {
    const int b = blockIdx.x;
    if (!(opt & 4) || H != 2 || (gridDim.x & 15) != 0) return b;
    return (((b >> 4) << 3) + (b & 7)) * 2 + ((b >> 3) & 1);
}
__device__ __forceinline__ double band_msub(double acc, double a, double b) { return __builtin_fma(-a, b, acc); }
__device__ __forceinline__ double band_madd(double acc, double a, double b) { return __builtin_fma(a, b, acc); }
// OPT bit 3 (L2PF): the global rows a later line iteration reads -- its update's basis and w rows, its
// SpMV's D and m rows -- are touched ahead of time by LDS-DMA loads (global_load_lds_dword, one lane
// per 128-B segment, into a scratch word nobody reads): no VGPR holds them, so the walk keeps more
// bytes in flight than the register prefetch alone (two lines ahead with it, one without it, J >
// BAND_PF).  The barriers then are bare s_barriers after lgkmcnt(0): __syncthreads' release fence
// would wait for the DMA (vmcnt(0)) at every barrier.  Only LDS is shared inside the kernel, so
// lgkmcnt(0) + s_barrier orders everything the barrier has to.
template <int OPT> __device__ __forceinline__ void band_sync() {
    if constexpr (OPT & 8) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else __syncthreads();
}
// lane tid <-> row v0 - BAND_OFF + tid: 16 rows (128 B) ahead of the part's first row, so that a
// wave's 64 rows are one aligned 512-B run of every row vector (four cache lines; with 8, the BJ
// blocks' minimum, five: round 6), the 8-row BJ blocks lane-aligned, the v-halo rows at tid
// BAND_OFF - 1 and BAND_OFF + LP (LP + 2 BAND_OFF <= BAND_T)
constexpr int BAND_OFF = 16;
static_assert(BAND_LP + 2 * BAND_OFF <= BAND_T && BAND_OFF % 8 == 0, "band geometry");
template <int WU, int J, int VMODE = 0, bool GH = true, int OPT = 0>
__global__ __launch_bounds__(BAND_T) __attribute__((amdgpu_waves_per_eu(band_wpe<OPT>()))) void k_band_step(BandK a) {
    constexpr int BAND_RS = BAND_T;
    constexpr int BAND_W = BAND_T / 64, BAND_IT = (J + 2 + BAND_W - 1) / BAND_W;   // dot items per wave
    __shared__ double vbuf[(J + 1) * BAND_LP];
    __shared__ double ring[4 * BAND_RS];
    __shared__ double wbuf[BAND_LP];
    __shared__ double red[DC_NQ];
    __shared__ double cs[BAND_JV], ce[BAND_JV], cp[BAND_JV];
    __shared__ int pf_sink[64];   // L2PF: the DMA's destination (never read)
    constexpr int j = J;
    if (__builtin_nontemporal_load(&a.st->xup_tag) == j) {   // the cycle's x update
        dc_xupdate_body<BAND_XUP_XB, true>(a.V, a.ld, j, __builtin_nontemporal_load(&a.st->stop_col), a.n, a.cf, a.x,
                                           a.H, a.S, a.m, a.w_prev);
        return;
    }
    if (stopped(&a.st->stop_col, j)) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int L = a.L, X = a.X, H = a.H_parts, LP = L / H;
    const int b = band_block(a.opt, H), R = (int)gridDim.x / H, rb = b / H, h = b % H, v0 = h * LP;
    const int xa = (int)((int64_t)rb * X / R), xb = (int)((int64_t)(rb + 1) * X / R);
    const int v = v0 - BAND_OFF + tid;
    const int wrapL = (X - 1) * L;   // |column - row| of a periodic x-coupling across the wrap
    const bool own = tid >= BAND_OFF && tid < BAND_OFF + LP;
    const bool upd = tid >= BAND_OFF - 1 && tid <= LP + BAND_OFF && v >= 0 && v < L;   // owned rows and the v-halo rows
    constexpr bool LSV = VMODE >= 1, CANON = VMODE == 2;
    const int ii = lane & 7;
    // LSV: the lane's x-coupling values (position v in every line)
    double tx0 = 0.0, tx1 = 0.0;
    if constexpr (LSV) {
        if (v >= 0 && v < L) {
            tx0 = a.lsv[a.n + v];
            tx1 = a.lsv[a.n + L + v];
        }
    }
    for (int k = tid; k < j; k += BAND_T) {
        cs[k] = a.cf->s[k];
        ce[k] = a.cf->e[k];
        cp[k] = a.cf->e_prev[k];
    }
    const double rinv = a.cf->rinv, qc = a.cf->q, ej = a.cf->e[j], qp = a.cf->q_prev;
    band_sync<OPT>();
    double vreg[J + 1];
    double acc[BAND_IT][3];
#pragma unroll
    for (int u = 0; u < BAND_IT; ++u) acc[u][0] = acc[u][1] = acc[u][2] = 0.0;
    // line of iteration it (it = 0: the x-halo line before xa; it = nl + 1: the one after xb - 1;
    // kind 1 / 2, recomputed, nothing stored)
    const int nl = xb - xa;
    const int xhm = xa == 0 ? X - 1 : xa - 1, xhp = xb == X ? 0 : xb;   // the x-halo lines (mod X)
    // opt bit 4 (ALT): odd line ranges walk their lines backwards, so that the two workgroups on
    // either side of every range boundary read the boundary's two lines (each one's own line and
    // the other's x-halo line) at the same time, at the start or at the end of both walks: the
    // second read finds the line in the Infinity Cache instead of HBM.  (The dots then sum an
    // odd range's lines in reverse order: not the bits of the forward walk, within the DCGS2 bars.)
    const bool rev = (a.opt & 16) && (rb & 1);
    // kind 1 / 2: the left / right x-halo line (a forward walk's first / last iteration)
    auto line_of = [&](int it, int &kind) {
        if (rev) {
            kind = it == 0 ? 2 : (it == nl + 1 ? 1 : 0);
            return it == 0 ? xhp : (it == nl + 1 ? xhm : xb - it);
        }
        kind = it == 0 ? 1 : (it == nl + 1 ? 2 : 0);
        return it == 0 ? xhm : (it == nl + 1 ? xhp : xa - 1 + it);
    };
    // the owned line whose SpMV and dots iteration it (>= 2) runs: the line updated one iteration
    // before, whose x-neighbours are both in the ring now
    auto spmv_line = [&](int it) { return rev ? xb + 1 - it : xa - 2 + it; };
    // software pipeline (J <= BAND_PF, as the registers allow): the next line's update
    // operands are loaded during this line's SpMV and dots.  (A partial prefetch of 4 basis rows
    // for larger J measured slower: 1234 vs 1254 it/s, spills)
    // (round 6: the prefetch for every J -- spilling a few values past BAND_PF -- measured j13
    // 758 -> 755, j16 880 -> 944, j18 989 -> 1087 us in process; not kept)
    constexpr bool PF = J <= BAND_PF;
    constexpr bool SPF = PF && CANON && (OPT & 1);
    // update operands of iteration it's line on the lane's row: V_k (k < j), w_{j-1} (j = 0: v_0)
    // and w_j
    struct Ld {
        double v[J > 0 ? J : 1];
        double wm, wj;
        double drow, mrow, tv0, tv1;   // SPF: the SpMV operands of the iteration's line x
    };
    auto load = [&](int it, Ld &o) {
        int kind;
        const int y = line_of(it, kind);
        if constexpr (SPF) {
            // line x = y - 1 of iteration it (owned when it >= 2): D, m on the lane's row, the
            // line's v couplings (the same loads the iteration head issues without SPF)
            o.drow = 0.0;
            o.mrow = 1.0;
            o.tv0 = o.tv1 = 0.0;
            if (it >= 2) {
                const int xs = spmv_line(it);
                const int64_t rs = (int64_t)xs * L + (own ? v : v0);
                if (own) {
                    o.drow = __builtin_nontemporal_load(a.lsv + rs);
                    o.mrow = __builtin_nontemporal_load(a.mtri + rs);
                }
                o.tv0 = a.lsv[a.n + 2 * L + xs];
                o.tv1 = a.lsv[a.n + 2 * L + X + xs];
            }
        }
        const int64_t row = (int64_t)y * L + (upd ? v : 0);
        o.wm = 0.0;
        o.wj = 0.0;
        // a rank's first / last line range: the x-halo line is a neighbour rank's line, whose
        // V_k (k < j), w_j and w_{j-1} arrived in the ghost buffer (slots k, m + (j & 1),
        // m + ((j - 1) & 1); v_0 in slot 0 at j = 0)
        const double *gh = (GH && a.ghost && ((kind == 1 && rb == 0) || (kind == 2 && rb == R - 1)))
                               ? a.ghost + (size_t)(kind == 1 ? 0 : 1) * (a.m + 2) * L : nullptr;
        if (upd) {
            if (gh) {
                o.wj = gh[(size_t)(a.m + (j & 1)) * L + v];
                o.wm = gh[(size_t)(j == 0 ? 0 : a.m + ((j + 1) & 1)) * L + v];
            } else {
                o.wj = __builtin_nontemporal_load(a.w_in + row);
                o.wm = __builtin_nontemporal_load((j == 0 ? a.V : a.w_prev) + row);
            }
        }
        if (gh) {
#pragma unroll
            for (int k = 0; k < J; ++k) o.v[k] = upd ? gh[(size_t)k * L + v] : 0.0;
        } else {
            // one lane pointer stepped by ld (per-k scalar bases would spill SGPRs: readlanes)
            const double *pv = a.V + row;
#pragma unroll
            for (int k = 0; k < J; ++k) {
                o.v[k] = upd ? __builtin_nontemporal_load(pv) : 0.0;
                pv += a.ld;
            }
        }
    };
    // the update itself: p_j as step j-1's update formed it, then k_dc_update's operations;
    // stores v_j on owned lines (and p_{j+1} at the last band step); vreg = V_k, v_j
    auto update = [&](int it, const Ld &o) -> double {
        int kind;
        const int y = line_of(it, kind);
        const int64_t row = (int64_t)y * L + (upd ? v : 0);
#pragma unroll
        for (int k = 0; k < J; ++k) vreg[k] = o.v[k];
        double pj = o.wm;   // j = 0: p_0 = v_0
        if (j >= 1) {
            double tp = o.wm;
#pragma unroll
            for (int k = 0; k < J; ++k) tp = band_msub(tp, cp[k], vreg[k]);
            pj = tp * qp;
        }
        double av = pj, tv = o.wj;
#pragma unroll
        for (int k = 0; k < J; ++k) {
            const double sk = cs[k], ek = ce[k];
            av = band_msub(av, sk, vreg[k]);
            tv = band_msub(tv, ek, vreg[k]);
        }
        double vj = pj;
        if (j >= 1) vj = av * rinv;
        tv = band_msub(tv, ej, vj);
        const double pn = tv * qc;
        vreg[J] = vj;
        if (kind == 0 && own) {
            if (j >= 1) {
                st_wt(a.V + (size_t)j * a.ld + row, vj);
            }
            if (j == a.m - 2) st_wt(a.V + (size_t)(j + 1) * a.ld + row, pn);
        }
        return pn;
    };
    auto stage = [&](double *vb) {
        if (own) {
#pragma unroll
            for (int k = 0; k <= J; ++k) vb[k * BAND_LP + tid - BAND_OFF] = vreg[k];
        }
    };
    auto slot = [&](int y) { return ((y - xa + 1) & 3) * BAND_RS; };
    // L2PF: touch the rows iteration itp reads (its line's rows v0 - 1 .. v0 + LP of the J basis
    // vectors, w_j and w_{j-1} (v_0 at j = 0); D and m of its SpMV line), 128-B segments, the
    // rows spread over the waves.  Ghost lines (a neighbour rank's) come from the ghost buffer: skipped
    constexpr int PF_ROWS = J + 2 + (CANON ? 2 : 0);
    auto l2_prefetch = [&](int itp) {
        if constexpr ((OPT & 8) != 0) {
            if (itp > nl + 1) return;
            int kind;
            const int y = line_of(itp, kind);
            const bool ghostl = GH && a.ghost && ((kind == 1 && rb == 0) || (kind == 2 && rb == R - 1));
            const int xs = spmv_line(itp);   // its SpMV line (owned when itp >= 2)
            const int vlo = v0 > 0 ? v0 - 1 : 0, vhi = v0 + LP < L ? v0 + LP + 1 : L;
            // (round 6: capping the prefetch at 10 basis rows -- a line's J + 4 rows of ~3.3 KB per
            // workgroup, 64 workgroups per XCD, overflow the 4 MB L2 past ~14 rows: PMC fetch 1.07x at
            // j = 13, 1.19x at j = 18 -- made j13-j18 11-33 us slower in process: not kept)
            for (int r = wv; r < PF_ROWS; r += BAND_W) {   // wave-uniform
                const double *vec;
                int64_t r0, r1;
                if (r < J + 2) {
                    if (ghostl) continue;
                    vec = r < J ? a.V + (size_t)r * a.ld : (r == J ? a.w_in : (j == 0 ? a.V : a.w_prev));
                    r0 = (int64_t)y * L + vlo;
                    r1 = (int64_t)y * L + vhi;
                } else {
                    if (itp < 2) continue;
                    vec = r == J + 2 ? a.lsv : a.mtri;
                    r0 = (int64_t)xs * L + v0;
                    r1 = r0 + LP;
                }
                const int64_t s0 = r0 >> 4, ns = ((r1 - 1) >> 4) - s0 + 1;   // 16 doubles = 128 B
                if (lane < ns)
                    __builtin_amdgcn_global_load_lds(vec + ((s0 + lane) << 4), (__attribute__((address_space(3))) void *)pf_sink,
                                                     4, 0, 0);
            }
        }
    };
    // iteration it updates line y = xa - 1 + it (ALT, odd ranges: xb - it) and, from it = 2 on,
    // runs the SpMV and dots of line y - 1 (ALT, odd ranges: y + 1)
    Ld nx;
    if constexpr (PF) load(0, nx);
    l2_prefetch(PF ? 1 : 0);   // (L2PF only)
    for (int it = 0; it <= nl + 1; ++it) {
        // y: the updated line's logical index (xa - 1 .. xb, unwrapped: its ring slot), x: the
        // SpMV line (owned when it >= 2)
        const int y = rev ? xb - it : xa - 1 + it, x = spmv_line(it);
        const bool work = it >= 2;   // line x = y - 1 is owned: SpMV + dots
        const int64_t lrow = (int64_t)(work ? x : xa) * L;
        const int64_t row = lrow + (own ? v : v0);
        // the SpMV operands of line x (independent of the update): codes, dictionary, values, m
        const int64_t q = row >> 6, q0 = (lrow + v0 - BAND_OFF + 64 * wv) >> 6;
        const int l64 = (int)(row & 63);
        uint32_t word = 0u;
        int dv = 0;
        double d[LSV ? 1 : WU];
        double mrow = 1.0, drow = 0.0, tv0 = 0.0, tv1 = 0.0;
        if (work && !SPF) {
            if constexpr (!CANON) {
                word = __builtin_nontemporal_load(a.pk + q * 64 + l64);
                const int64_t qd = q0 + (lane >> 4);
                dv = (lane < 32 && qd >= 0 && qd * 64 < a.n) ? a.dict[qd * 16 + (lane & 15)] : 0;
            }
            if constexpr (LSV) {
                if (own) drow = __builtin_nontemporal_load(a.lsv + row);
                tv0 = a.lsv[a.n + 2 * L + x];
                tv1 = a.lsv[a.n + 2 * L + X + x];
            } else {
#pragma unroll
                for (int k = 0; k < WU; ++k) d[k] = __builtin_nontemporal_load(a.val + q * 64 * WU + 64 * k + l64);
            }
            if (own) mrow = __builtin_nontemporal_load(a.mtri + row);
        }
        // 1. update of line y
        {
            Ld cu;
            if constexpr (PF) cu = nx;
            else load(it, cu);
            if constexpr (SPF) {
                drow = cu.drow;
                mrow = cu.mrow;
                tv0 = cu.tv0;
                tv1 = cu.tv1;
            }
            const double pn = update(it, cu);
            if (upd) ring[slot(y) + tid] = pn;
            if constexpr (PF) {
                if (it <= nl) load(it + 1, nx);
            }
            l2_prefetch(PF ? it + 2 : it + 1);   // (L2PF only)
        }
        band_sync<OPT>();
        if (work) {
            // 2. w = M^-1 A p_{j+1} on the part's rows of line x, gathers from the ring
            double sacc = 0.0, sub = 0.0, sup = 0.0;
            if constexpr (CANON) {
                // the line's stored order of the five kinds (the same for every lane of the line)
                int64_t cxm, cxp;
                const int ord = __builtin_amdgcn_readfirstlane(
                    canon_order_xv(x, 0, a.n, L, X, GH && a.ghost ? a.left_blk : -1, cxm, cxp, a.xord));
                const int sx = ((x - xa + 1) & 3) * BAND_RS - v0 + BAND_OFF;   // ring offset of line x
                // the three orders the lines take (interior / first line / last line of one rank),
                // straight-line: every lane reads its five operands (a clamped row off its own
                // rows), the absent v -+ 1 terms are skipped by selects -- the same additions in
                // the same order as the loop below, without its per-entry exec-mask branches
                constexpr int P_MID = 0 | 1 << 3 | 2 << 6 | 3 << 9 | 4 << 12;
                constexpr int P_FIRST = 1 | 2 << 3 | 3 << 6 | 4 << 9 | 0 << 12;
                constexpr int P_LAST = 4 | 0 << 3 | 1 << 6 | 2 << 9 | 3 << 12;
                const bool sl = a.canon == 2 && (ord == P_MID || ord == P_FIRST || ord == P_LAST);   // uniform
                if (sl) {
                    const int vv = own ? v : v0;
                    const double t0 = tx0 * ring[((x - xa) & 3) * BAND_RS - v0 + BAND_OFF + vv];
                    const double t4 = tx1 * ring[((x - xa + 2) & 3) * BAND_RS - v0 + BAND_OFF + vv];
                    const double t2 = drow * ring[sx + vv];
                    const double t1 = tv0 * ring[sx + vv - 1];
                    const double t3 = tv1 * ring[sx + vv + 1];
                    const bool h1 = vv > 0, h3 = vv < L - 1;
                    double sa = 0.0;
                    if (ord == P_MID) {
                        sa = sa + t0;
                        sa = h1 ? sa + t1 : sa;
                        sa = sa + t2;
                        sa = h3 ? sa + t3 : sa;
                        sa = sa + t4;
                    } else if (ord == P_FIRST) {
                        sa = h1 ? sa + t1 : sa;
                        sa = sa + t2;
                        sa = h3 ? sa + t3 : sa;
                        sa = sa + t4;
                        sa = sa + t0;
                    } else {
                        sa = sa + t4;
                        sa = sa + t0;
                        sa = h1 ? sa + t1 : sa;
                        sa = sa + t2;
                        sa = h3 ? sa + t3 : sa;
                    }
                    sacc = own ? sa : 0.0;
                    sub = (own && h1 && ii > 0) ? 0.0 + tv0 : 0.0;
                    sup = (own && h3 && ii < 7) ? 0.0 + tv1 : 0.0;
                }
#pragma unroll
                for (int e = 0; e < 5; ++e) {
                    const int kind = (ord >> (3 * e)) & 7;   // uniform
                    if (!sl && own) {
                        if (kind == 0) sacc += tx0 * ring[((x - xa) & 3) * BAND_RS - v0 + BAND_OFF + v];
                        else if (kind == 4) sacc += tx1 * ring[((x - xa + 2) & 3) * BAND_RS - v0 + BAND_OFF + v];
                        else if (kind == 2) sacc += drow * ring[sx + v];
                        else if (kind == 1) {
                            if (v > 0) {
                                sacc += tv0 * ring[sx + v - 1];
                                if (ii > 0) sub = sub + tv0;
                            }
                        } else if (v < L - 1) {
                            sacc += tv1 * ring[sx + v + 1];
                            if (ii < 7) sup = sup + tv1;
                        }
                    }
                }
            } else {
                const int sel = (int)(q - q0) * 16;
#pragma unroll
                for (int k = 0; k < WU; ++k) {
                    const int code = (int)((word >> (4 * k)) & 15u);
                    const int off = __shfl(dv, (sel + code) & 63, 64);
                    if (own && code != PK_CODES) {
                        // the column's line relative to x and its position in that line, by range
                        // tests (vtk_csr_set_line_band checked: lines x-1..x+1, or the periodic wrap)
                        const int t = v + off;
                        int rel, vc;
                        const int c = x * L + t;
                        if (a.ghost && c >= (int)a.n) {   // halo column: a neighbour rank's line
                            const int kk = c - (int)a.n, blk = kk >= L ? 1 : 0;
                            rel = blk == a.left_blk ? -1 : 1;
                            vc = kk - blk * L;
                        } else if (t >= 0 && t < L) { rel = 0; vc = t; }
                        else if (t >= L && t < 2 * L) { rel = 1; vc = t - L; }
                        else if (t < 0 && t >= -L) { rel = -1; vc = t + L; }
                        else if (t >= L) { rel = -1; vc = t - wrapL; }   // column in line X-1, row in line 0
                        else { rel = 1; vc = t + wrapL; }                // column in line 0, row in line X-1
                        const double xv = ring[((x - xa + 1 + rel) & 3) * BAND_RS + vc - v0 + BAND_OFF];
                        double dk;
                        if constexpr (LSV) dk = rel != 0 ? (rel > 0 ? tx1 : tx0) : (vc == v ? drow : (vc > v ? tv1 : tv0));
                        else dk = d[k];
                        sacc += dk * xv;
                        if (off == -1 && ii > 0) sub = sub + dk;
                        if (off == 1 && ii < 7) sup = sup + dk;
                    }
                }
            }
            const double z = bj_trim_group<8>(own ? sacc : 0.0, lane, sub, sup, mrow);
            if (own) {
                st_wt(a.w_out + row, z);
                wbuf[tid - BAND_OFF] = z;
            }
            band_sync<OPT>();
            // 3. dots of the part's rows of line x: wave wv owns items wv, wv + 7, wv + 14 (item
            //    k <= j: s_k, z_k; j + 1: |p|^2, p.w, |w|^2), lanes stride the rows.  Items
            //    outer: each item's loop streams one basis row against p and w (rows outer with
            //    p, w read once per row for all items measured slower: 1268-1285 vs 1296 it/s)
            const double *pr = ring + slot(x) + BAND_OFF;
#pragma unroll
            for (int u = 0; u < BAND_IT; ++u) {
                const int itm = wv + BAND_W * u;
                if (itm <= j) {
                    const double *vk = vbuf + itm * BAND_LP;
#pragma unroll VTK_BAND_DOTS_UNROLL
                    for (int t = lane; t < LP; t += 64) {
                        const double vv = vk[t];
                        acc[u][0] = band_madd(acc[u][0], vv, pr[t]);
                        acc[u][1] = band_madd(acc[u][1], vv, wbuf[t]);
                    }
                } else if (itm == j + 1) {
#pragma unroll VTK_BAND_DOTS_UNROLL
                    for (int t = lane; t < LP; t += 64) {
                        const double pv = pr[t], wq = wbuf[t];
                        acc[u][0] = band_madd(acc[u][0], pv, pv);
                        acc[u][1] = band_madd(acc[u][1], pv, wq);
                        acc[u][2] = band_madd(acc[u][2], wq, wq);
                    }
                }
            }
            band_sync<OPT>();
        }
        if (it >= 1 && it <= nl) stage(vbuf);   // line y is owned: its basis rows for the dots one line on
    }
    // per-workgroup partials in launch_dc_dots' layout for step j+1
#pragma unroll
    for (int u = 0; u < BAND_IT; ++u) {
        const int itm = wv + BAND_W * u;
        if (itm <= j + 1) {   // wave-uniform
            const double t0 = wave_allsum(acc[u][0]), t1 = wave_allsum(acc[u][1]), t2 = wave_allsum(acc[u][2]);
            if (lane == 0) {
                if (itm <= j) {
                    red[itm] = t0;
                    red[DC_MAXJ + itm] = t1;
                } else {
                    red[2 * DC_MAXJ] = t0;
                    red[2 * DC_MAXJ + 1] = t1;
                    red[2 * DC_MAXJ + 2] = t2;
                }
            }
        }
    }
    __syncthreads();
    const int jn = j + 1;
    for (int qq = tid; qq < DC_NQ; qq += BAND_T) {
        const bool used = qq < jn || (qq >= DC_MAXJ && qq < DC_MAXJ + jn) || qq >= 2 * DC_MAXJ;
        if (used) a.part[(size_t)qq * GMAX + b] = red[qq];
    }
}

// the one-rank production instantiations (canonical rows, line-separable values) with the
// variant bits of a.opt; WPC3 only where the LDS of three workgroups fits (J <= BAND_J3)
// SPF (bit 0) only at the step indices where it measured faster: in-process A/B, round 6, on the
// final kernels (profiles/r06_band_bits_ab.json): j = 0 -12 us, j = 3, 4 -3 us each at C3; j = 1, 2
// +2 / +5 us, j = 6-12 +6 ... +20 us each (the operands' registers held across the SpMV + dots);
// the same signs on C2 and the C3 slabs
template <int J> constexpr bool band_spf_j() { return J == 0 || J == 3 || J == 4; }
template <int J> static void launch_band_one_rank(const BandK &a0, int grid, hipStream_t s) {
    BandK a = a0;
    if constexpr (!band_spf_j<J>()) a.opt &= ~1;
    const dim3 g(grid), blk(BAND_T);
    // L2PF where the registers hold no next line (J > BAND_PF).  In-process A/B (C3, round 6): j13-j17
    // 745-925 -> 709-875 us, j18 991 -> 970; with the register prefetch (J <= 12, two lines ahead)
    // it cost 11-35 us per launch
    if constexpr (J > BAND_PF) {
        if (a.opt & 8) { hipLaunchKernelGGL((k_band_step<5, J, 2, false, 9>), g, blk, 0, s, a); return; }
    }
    if constexpr (J <= BAND_J3) {
        if ((a.opt & 3) == 3) { hipLaunchKernelGGL((k_band_step<5, J, 2, false, 3>), g, blk, 0, s, a); return; }
        if ((a.opt & 3) == 2) { hipLaunchKernelGGL((k_band_step<5, J, 2, false, 2>), g, blk, 0, s, a); return; }
    }
    if (a.opt & 1) hipLaunchKernelGGL((k_band_step<5, J, 2, false, 1>), g, blk, 0, s, a);
    else hipLaunchKernelGGL((k_band_step<5, J, 2, false>), g, blk, 0, s, a);
}

// across ranks (ghost lines, canonical rows, line-separable values): the same variants as one rank
// -- until round 6 the distributed band step ran OPT 0 only (no SpMV operands in the prefetch, no
// third workgroup per CU at low j, no LDS-DMA prefetch at high j), which the one-rank slab
// projections (--comm-solo: no ghost lines) did not see.  The ghost lines' update operands come from
// the ghost buffer in load(); the DMA prefetch skips them (l2_prefetch's ghostl)
template <int J> static void launch_band_ghost(const BandK &a0, int grid, hipStream_t s) {
    BandK a = a0;
    if constexpr (!band_spf_j<J>()) a.opt &= ~1;
    const dim3 g(grid), blk(BAND_T);
    if constexpr (J > BAND_PF) {
        if (a.opt & 8) { hipLaunchKernelGGL((k_band_step<5, J, 2, true, 9>), g, blk, 0, s, a); return; }
    }
    if constexpr (J <= BAND_J3) {
        if ((a.opt & 3) == 3) { hipLaunchKernelGGL((k_band_step<5, J, 2, true, 3>), g, blk, 0, s, a); return; }
        if ((a.opt & 3) == 2) { hipLaunchKernelGGL((k_band_step<5, J, 2, true, 2>), g, blk, 0, s, a); return; }
    }
    if constexpr (J > BAND_J3 && J <= BAND_PF) {
        if (a.opt & 1) { hipLaunchKernelGGL((k_band_step<5, J, 2, true, 1>), g, blk, 0, s, a); return; }
    }
    hipLaunchKernelGGL((k_band_step<5, J, 2>), g, blk, 0, s, a);
}

hipError_t launch_band_step(const BandK &a, int grid, int wu, hipStream_t s) {
    if (wu != 5 || a.H_parts < 1 || a.L % a.H_parts != 0 || a.L / a.H_parts > BAND_LP || (a.L / a.H_parts) % 8 != 0 ||
        a.j + 1 > BAND_JV || grid < a.H_parts || grid > GMAX || grid % a.H_parts != 0 || grid / a.H_parts > a.X ||
        a.n > INT32_MAX / 2)
        return hipErrorInvalidValue;
    switch (a.j) {
#define VTK_BAND_J(J_)                                                                                           \
    case J_:                                                                                                     \
        if (a.lsv && a.canon && !a.ghost) launch_band_one_rank<J_>(a, grid, s); \
        else if (a.lsv && a.canon) launch_band_ghost<J_>(a, grid, s); \
        else if (a.lsv) hipLaunchKernelGGL((k_band_step<5, J_, 1>), dim3(grid), dim3(BAND_T), 0, s, a); \
        else hipLaunchKernelGGL((k_band_step<5, J_>), dim3(grid), dim3(BAND_T), 0, s, a); \
        break;
        VTK_BAND_J(0) VTK_BAND_J(1) VTK_BAND_J(2) VTK_BAND_J(3) VTK_BAND_J(4) VTK_BAND_J(5) VTK_BAND_J(6)
        VTK_BAND_J(7) VTK_BAND_J(8) VTK_BAND_J(9) VTK_BAND_J(10) VTK_BAND_J(11) VTK_BAND_J(12) VTK_BAND_J(13)
        VTK_BAND_J(14) VTK_BAND_J(15) VTK_BAND_J(16) VTK_BAND_J(17) VTK_BAND_J(18)
#undef VTK_BAND_J
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ghost exchange of the distributed band step: pack the rank's first / last line
// of v_{j-1} (V[j-1]; V[0] at j = 0) and w_j into send pieces of BAND_GHOST_VECS L, unpack the
// received pieces into the ghost slots (v_{j-1} -> slot j-1, v_0 -> slot 0 at j = 0, w_j ->
// m + (j & 1): step j-1's w stays in the other slot for the recompute of p_j)
__global__ __launch_bounds__(NT) void k_ghost_pack(const double *__restrict__ V, int64_t ld, int j,
                                                   const double *__restrict__ w, int64_t n, int L,
                                                   double *__restrict__ sbuf, int64_t off_first, int64_t off_last) {
    constexpr int NV = BAND_GHOST_VECS;
    for (int i = blockIdx.x * NT + threadIdx.x; i < 2 * NV * L; i += gridDim.x * NT) {
        const int side = i / (NV * L), r = i % (NV * L), vec = r / L, t = r % L;
        const int64_t off = side == 0 ? off_first : off_last;
        if (off < 0) continue;
        const int64_t row = (side == 0 ? 0 : n - L) + t;
        sbuf[off + r] = vec == 0 ? V[(size_t)(j >= 1 ? j - 1 : 0) * ld + row] : w[row];
    }
}

__global__ __launch_bounds__(NT) void k_ghost_unpack(const double *__restrict__ rbuf, int64_t off_left, int64_t off_right,
                                                     int j, int m, int L, double *__restrict__ ghost) {
    constexpr int NV = BAND_GHOST_VECS;
    for (int i = blockIdx.x * NT + threadIdx.x; i < 2 * NV * L; i += gridDim.x * NT) {
        const int side = i / (NV * L), r = i % (NV * L), vec = r / L, t = r % L;
        const int64_t off = side == 0 ? off_left : off_right;
        if (off < 0) continue;
        const int slot = vec == 0 ? (j >= 1 ? j - 1 : 0) : m + (j & 1);
        ghost[((size_t)side * (m + 2) + slot) * L + t] = rbuf[off + r];
    }
}

hipError_t launch_ghost_pack(const double *V, int64_t ld, int j, const double *w, int64_t n, int L, double *sbuf,
                             int64_t off_first, int64_t off_last, hipStream_t s) {
    hipLaunchKernelGGL(k_ghost_pack, dim3((2 * BAND_GHOST_VECS * L + NT - 1) / NT), dim3(NT), 0, s, V, ld, j, w, n, L, sbuf, off_first,
                       off_last);
    return hipGetLastError();
}

hipError_t launch_ghost_unpack(const double *rbuf, int64_t off_left, int64_t off_right, int j, int m, int L,
                               double *ghost, hipStream_t s) {
    hipLaunchKernelGGL(k_ghost_unpack, dim3((2 * BAND_GHOST_VECS * L + NT - 1) / NT), dim3(NT), 0, s, rbuf, off_left, off_right, j, m, L,
                       ghost);
    return hipGetLastError();
}

// distributed form of the check (local column numbering; the halo is exactly two neighbour lines,
// halo block lblk the left one): an owned column within lines x-1..x+1 of the row's line without
// wrap, a halo column only from the first (left block) or last (right block) local line
__global__ __launch_bounds__(NT) void k_band_check_dist(const int32_t *__restrict__ indptr,
                                                        const int32_t *__restrict__ indices, int64_t n, int L,
                                                        int lblk, int *bad) {
    const int64_t X = n / L;
    for (int64_t r = (int64_t)blockIdx.x * NT + threadIdx.x; r < n; r += (int64_t)gridDim.x * NT) {
        const int64_t x = r / L, vr = r % L;
        bool ok = true, vloc = true;
        for (int k = indptr[r]; k < indptr[r + 1]; ++k) {
            const int64_t c = indices[k];
            int64_t vc;
            if (c < 0 || c >= n + 2 * L) { ok = false; break; }
            if (c < n) {
                const int64_t rel = c / L - x;
                if (rel < -1 || rel > 1) { ok = false; break; }
                vc = c % L;
            } else {
                const int64_t kk = c - n, blk = kk / L;
                if ((blk == lblk && x != 0) || (blk != lblk && x != X - 1)) { ok = false; break; }
                vc = kk % L;
            }
            if (vc - vr < -1 || vc - vr > 1) vloc = false;
        }
        if (!ok) atomicOr(bad, 1);
        if (!vloc) atomicOr(bad, 2);
    }
}

hipError_t launch_band_check_dist(const int32_t *indptr, const int32_t *indices, int64_t n, int L, int lblk, int *bad,
                                  hipStream_t s) {
    int64_t g = (n + NT - 1) / NT;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    hipLaunchKernelGGL(k_band_check_dist, dim3((unsigned)g), dim3(NT), 0, s, indptr, indices, n, L, lblk, bad);
    return hipGetLastError();
}

// line-separable values: the table slot of entry (r, c) -- 0 the diagonal D[r], 1 TX[dir][v]
// (line x +- 1 at the row's position v), 2 TV[dir][x] (v +- 1 in the row's line) -- or -1
__device__ __forceinline__ int lsv_slot(int64_t r, int64_t c, int64_t n, int L, int X, int lblk, int64_t &idx) {
    const int64_t x = r / L, v = r % L;
    int64_t dx, vc;
    if (c < n) {
        dx = c / L - x;
        vc = c % L;
        if (lblk < 0) {   // one rank: periodic in x (X >= 3)
            if (dx == X - 1) dx = -1;
            else if (dx == -(X - 1)) dx = 1;
        }
    } else {
        const int64_t kk = c - n, blk = kk / L;
        dx = blk == lblk ? -1 : 1;
        vc = kk % L;
    }
    if (dx == 0) {
        if (vc == v) { idx = r; return 0; }
        if (vc == v - 1 || vc == v + 1) { idx = (int64_t)n + 2 * L + (vc > v ? X : 0) + x; return 2; }
        return -1;
    }
    if ((dx == 1 || dx == -1) && vc == v) { idx = (int64_t)n + (dx > 0 ? L : 0) + v; return 1; }
    return -1;
}

// pass 0: write every entry into its slot (entries sharing a table slot write the same bits when
// the operator is separable; the check pass decides); pass 1: compare every entry bit for bit
__global__ __launch_bounds__(NT) void k_lsv_build(const int32_t *__restrict__ indptr, const int32_t *__restrict__ indices,
                                                  const double *__restrict__ data, int64_t n, int L, int lblk,
                                                  int xord, double *__restrict__ lsv, int *bad, int pass) {
    const int X = (int)(n / L);
    for (int64_t r = (int64_t)blockIdx.x * NT + threadIdx.x; r < n; r += (int64_t)gridDim.x * NT) {
        for (int k = indptr[r]; k < indptr[r + 1]; ++k) {
            int64_t idx;
            if (lsv_slot(r, indices[k], n, L, X, lblk, idx) < 0) {
                atomicOr(bad, 1);
                break;
            }
            if (pass == 0) lsv[idx] = data[k];
            else if (__double_as_longlong(lsv[idx]) != __double_as_longlong(data[k])) atomicOr(bad, 1);
        }
        if (pass == 1) {
            // |= 2: the row is not canonical (its stored columns differ from canon_order's)
            int64_t cxm, cxp;
            const int ord = canon_order(r, n, L, X, lblk, cxm, cxp, xord);
            const int64_t v = r % L;
            int k = indptr[r];
            bool ok = true;
            for (int e = 0; e < 5 && ok; ++e) {
                const int kind = (ord >> (3 * e)) & 7;
                if ((kind == 1 && v == 0) || (kind == 3 && v == L - 1)) continue;
                const int64_t c = kind == 0 ? cxm : (kind == 4 ? cxp : r + kind - 2);
                ok = k < indptr[r + 1] && indices[k] == c;
                ++k;
            }
            if (!ok || k != indptr[r + 1]) atomicOr(bad, 2);
        }
    }
}

hipError_t launch_lsv_build(const int32_t *indptr, const int32_t *indices, const double *data, int64_t n, int L,
                            int lblk, int xord, double *lsv, int *bad, hipStream_t s) {
    if (L <= 0 || n % L != 0 || n / L < 2) return hipErrorInvalidValue;
    int64_t g = (n + NT - 1) / NT;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    for (int pass = 0; pass < 2; ++pass) {
        hipLaunchKernelGGL(k_lsv_build, dim3((unsigned)g), dim3(NT), 0, s, indptr, indices, data, n, L, lblk, xord, lsv, bad, pass);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// 4D grid rows (vtk::Grid4): pass 0 writes every entry's value into its table slot (D[r] for
// the diagonal), pass 1 compares every entry with its slot bit for bit; either pass flags a row
// whose stored columns are not the grid kinds in ascending order.  Rows writing different values
// into one slot leave one of them there, so pass 1 catches every disagreement.
template <typename VT>
__global__ __launch_bounds__(NT) void k_grid4_build(const int32_t *__restrict__ indptr, const int32_t *__restrict__ indices,
                                                    const VT *__restrict__ data, int64_t n, Grid4 g,
                                                    double *__restrict__ tab, VT *__restrict__ D, int *bad, int pass) {
    for (int64_t r = (int64_t)blockIdx.x * NT + threadIdx.x; r < n; r += (int64_t)gridDim.x * NT) {
        const G4Row q = g4_coords(r, g);
        int64_t c[9];
        bool p[9];
        g4_cols(r, q, g, n, c, p);
        int64_t key[9];   // stored-order positions (halo planes: Grid4::xord)
        for (int k = 0; k < 9; ++k) key[k] = k == 0 || k == 8 ? g4_key(c[k], k, n, g) : c[k];
        int ord[9], m = 0;
        for (int k = 0; k < 9; ++k)
            if (p[k]) ord[m++] = k;
        for (int i = 1; i < m; ++i)   // ascending global columns (the stored order of a canonical CSR)
            for (int t = i; t > 0 && key[ord[t]] < key[ord[t - 1]]; --t) {
                const int s = ord[t];
                ord[t] = ord[t - 1];
                ord[t - 1] = s;
            }
        const int k0 = indptr[r];
        bool ok = indptr[r + 1] - k0 == m;
        for (int e = 0; e < m && ok; ++e) {
            const int kind = ord[e];
            if ((int64_t)indices[k0 + e] != c[kind] || (e > 0 && c[ord[e]] == c[ord[e - 1]])) { ok = false; break; }
            const VT dv = data[k0 + e];
            if (kind == 4) {
                if (pass == 0) D[r] = dv;
            } else {
                const int sl = g4_slot(kind, q, g);
                if (pass == 0) tab[sl] = (double)dv;
                else if (__double_as_longlong(tab[sl]) != __double_as_longlong((double)dv)) ok = false;
            }
        }
        if (!ok) atomicOr(bad, 1);
    }
}

hipError_t launch_grid4_build(const int32_t *indptr, const int32_t *indices, const void *data, int fp32, int64_t n,
                              const Grid4 &g, double *tab, void *D, int *bad, hipStream_t s) {
    const int64_t S4 = (int64_t)g.Ny * g.Nvx * g.Nvy;
    if (g.Ny < 3 || g.Nvx < 2 || g.Nvy < 2 || S4 <= 0 || n % S4 != 0 || n / S4 != g.X || n > INT32_MAX / 2 ||
        (g.lblk < 0 && g.X < 3))
        return hipErrorInvalidValue;
    int64_t gr = (n + NT - 1) / NT;
    if (gr > 4096) gr = 4096;
    if (gr < 1) gr = 1;
    for (int pass = 0; pass < 2; ++pass) {
        if (fp32) hipLaunchKernelGGL(k_grid4_build<float>, dim3((unsigned)gr), dim3(NT), 0, s, indptr, indices,
                                     (const float *)data, n, g, tab, (float *)D, bad, pass);
        else hipLaunchKernelGGL(k_grid4_build<double>, dim3((unsigned)gr), dim3(NT), 0, s, indptr, indices,
                                (const double *)data, n, g, tab, (double *)D, bad, pass);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// y = A x from the line-separable tables and the SELL codes (one wave per 64-row chunk, lane per
// row): k_sell's plain SpMV -- entries in stored order, padding skipped -- reading 12 B of
// matrix per row instead of 44.  lblk < 0: one rank (x couplings periodic); else the halo
// block of the left neighbour line (HALO: the halo columns read from halo[])
// CANON (every row canonical, vtk_csr::lsv_canon): the columns and values from canon_row -- no
// code word or dictionary loaded, the gathers issue with the diagonal
template <bool HALO, bool CANON = false>
__global__ __launch_bounds__(NT) void k_lsv_spmv(const uint32_t *__restrict__ pk, const int32_t *__restrict__ dict,
                                                 const double *__restrict__ lsv, const double *__restrict__ x,
                                                 const double *__restrict__ halo, double *__restrict__ y, int n, int L,
                                                 int lblk, int xord, const int *stop_col, int col) {
    if (stopped(stop_col, col)) return;
    const int lane = threadIdx.x & 63;
    const int X = n / L, nch = (n + 63) >> 6;
    for (int q = (int)(((int64_t)blockIdx.x * NT + threadIdx.x) >> 6); q < nch; q += (int)((int64_t)gridDim.x * NT >> 6)) {
        const int r = 64 * q + lane;
        const bool act = r < n;
        // the row's line and position: the chunk's first row by one division, then the lane
        int xl = (64 * q) / L, v = 64 * q - xl * L + lane;
        while (v >= L) {
            v -= L;
            ++xl;
        }
        const double drow = act ? __builtin_nontemporal_load(lsv + r) : 0.0;
        double s = 0.0;
        if constexpr (CANON) {
            if (act) {
                int c[5];
                double d[5];
                canon_row(lsv, n, L, lblk, xl, v, drow, c, d, xord);
                double xv[5];
#pragma unroll
                for (int k = 0; k < 5; ++k) {
                    const int cc = c[k] >= 0 ? c[k] : r;
                    xv[k] = (HALO && cc >= n) ? halo[cc - n] : x[cc];
                }
#pragma unroll
                for (int k = 0; k < 5; ++k)
                    if (c[k] >= 0) s += d[k] * xv[k];
                __builtin_nontemporal_store(s, y + r);
            }
            continue;
        }
        const uint32_t word = act ? __builtin_nontemporal_load(pk + (size_t)q * 64 + lane) : ~0u;
        const int dv = lane < 16 ? dict[(size_t)q * 16 + lane] : 0;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const int code = (int)((word >> (4 * k)) & 15u);
            const int off = __shfl(dv, code, 64);
            if (act && code != PK_CODES) {
                const int c = r + off;
                double val;
                if (off == 0) val = drow;
                else if (off == 1 || off == -1) val = lsv[(size_t)n + 2 * L + (off > 0 ? X : 0) + xl];
                else {
                    const bool up = (HALO && c >= n) ? ((c - n) / L != lblk) : (off == L || (lblk < 0 && off == -(X - 1) * L));
                    val = lsv[(size_t)n + (up ? L : 0) + v];
                }
                const double xv = (HALO && c >= n) ? halo[c - n] : x[c];
                s += val * xv;
            }
        }
        if (act) __builtin_nontemporal_store(s, y + r);
    }
}

// The same SpMV with the x vector staged through LDS (one rank, canonical rows): workgroup (range
// rb, part h) walks the lines of its range in order, loads each line's x rows v0-8 .. v0+LP+7 once
// (coalesced, prefetched one line ahead in registers) into a ring of 4 lines, and forms row v of
// line x from the ring -- x-1 and x+1 at v, x at v-1..v+1 -- with canon_order's straight-line
// sum (the same products added in the same order as k_lsv_spmv<CANON>: bit-identical).  HBM
// reads x once (+2 halo lines per range) instead of gathering it three times from L2/MALL.
__global__ __launch_bounds__(BAND_T) void k_lsv_ring(const double *__restrict__ lsv, const double *__restrict__ x,
                                                     double *__restrict__ y, int n, int L, int H, const int *stop_col,
                                                     int col) {
    __shared__ double ring[4 * BAND_T];
    if (stopped(stop_col, col)) return;
    const int tid = threadIdx.x, X = n / L, LP = L / H;
    const int b = blockIdx.x, R = (int)gridDim.x / H, rb = b / H, h = b % H, v0 = h * LP;
    const int xa = (int)((int64_t)rb * X / R), xb = (int)((int64_t)(rb + 1) * X / R), nl = xb - xa;
    const int v = v0 - 8 + tid;
    const bool inl = v >= 0 && v < L && tid < LP + 16;   // a row of the line (own or v-halo)
    const bool own = tid >= 8 && tid < 8 + LP;
    const double tx0 = own ? lsv[n + v] : 0.0, tx1 = own ? lsv[n + L + v] : 0.0;
    auto line_of = [&](int it) { return it == 0 ? (xa == 0 ? X - 1 : xa - 1) : (it == nl + 1 ? (xb == X ? 0 : xb) : xa - 1 + it); };
    auto slot = [&](int it) { return (it & 3) * BAND_T; };
    // prefetch: x of line_of(it) on the lane's row, D of line it - 1 (computed at iteration it)
    double nxv = inl ? __builtin_nontemporal_load(x + (int64_t)line_of(0) * L + v) : 0.0, nd = 0.0;
    for (int it = 0; it <= nl + 1; ++it) {
        ring[slot(it) + tid] = nxv;
        const double drow = nd;
        if (it <= nl) {
            nxv = inl ? __builtin_nontemporal_load(x + (int64_t)line_of(it + 1) * L + v) : 0.0;
            nd = own && it + 1 >= 2 ? __builtin_nontemporal_load(lsv + (int64_t)(xa + it - 1) * L + v) : 0.0;
        }
        __syncthreads();
        if (it >= 2) {
            const int xl = xa + it - 2;   // line x: ring slots it-2 (x-1), it-1 (x), it (x+1)
            const double tv0 = lsv[n + 2 * L + xl], tv1 = lsv[n + 2 * L + X + xl];
            int64_t cxm, cxp;
            const int ord = __builtin_amdgcn_readfirstlane(canon_order_xv(xl, 0, n, L, X, -1, cxm, cxp));
            constexpr int P_MID = 0 | 1 << 3 | 2 << 6 | 3 << 9 | 4 << 12;
            constexpr int P_FIRST = 1 | 2 << 3 | 3 << 6 | 4 << 9 | 0 << 12;
            const int sx = slot(it - 1);
            const double t0 = tx0 * ring[slot(it - 2) + tid];
            const double t4 = tx1 * ring[slot(it) + tid];
            const double t2 = drow * ring[sx + tid];
            const double t1 = tv0 * ring[sx + tid - (tid > 0 ? 1 : 0)];
            const double t3 = tv1 * ring[sx + tid + (tid < BAND_T - 1 ? 1 : 0)];
            const bool h1 = v > 0, h3 = v < L - 1;
            double sa = 0.0;
            if (ord == P_MID) {
                sa = sa + t0;
                sa = h1 ? sa + t1 : sa;
                sa = sa + t2;
                sa = h3 ? sa + t3 : sa;
                sa = sa + t4;
            } else if (ord == P_FIRST) {   // line 0: x-1 wraps to line X-1, last
                sa = h1 ? sa + t1 : sa;
                sa = sa + t2;
                sa = h3 ? sa + t3 : sa;
                sa = sa + t4;
                sa = sa + t0;
            } else {                        // line X-1: x+1 wraps to line 0, first
                sa = sa + t4;
                sa = sa + t0;
                sa = h1 ? sa + t1 : sa;
                sa = sa + t2;
                sa = h3 ? sa + t3 : sa;
            }
            if (own) st_nt<2>(y + (int64_t)xl * L + v, sa);
        }
    }
}

// 4D grid rows (vtk::Grid4) with x staged through LDS: w = M^-1 A p for the tridiagonal BJ(8)
// (the split DCGS2 step of the 4D operators).  A workgroup of 256 lanes (one row
// each) walks a contiguous range of 256-row groups; an LDS ring of RL doubles holds x over
// [g0 - S3, g0 + 256 + S3) (S3 = Nvx Nvy, the y-line), so the vy, vx and y couplings read LDS, and
// the window slides by one group per step.  Every global operand of a group -- the window's next
// 256 rows, the x -+ 1 plane rows (S4 away: contiguous 256-row blocks), the y-wrap row, m and D --
// is loaded one group ahead into registers, all loads unconditional (clamped rows, the
// halo chosen by address): no exec-masked load, so the wait for a group's operands does not wait
// for the groups behind it.  Coordinates advance by 256 in the mixed radix (no division per row),
// ring slots by 256 modulo RL.  Terms summed in the stored order (as k_sell's grid rows), the BJ
// solve of bj_trim_group: bit-identical to k_sell<EPI_PREC, 8, tri> on the same operator.
// RL: ring length (>= 2 S3 + 512): 4608 (36 KB, four workgroups per CU) when the y-line allows
// (C4: S3 = 2000), else 8192 (64 KB); the tables TX | TY | TVX | TVY (<= G4TAB doubles) in LDS
// too: three workgroups per CU at C4.
// MODE (G4Dots::mode): 0 w = M^-1 A x; 2 DCGS2 step 0 (j = 0: |p|^2, p.w, |w|^2, each lane over
// its own rows); 3 the cycle-start residual r = b - A x, w = M^-1 r, |r|^2, |w|^2 (partials p0,
// p1) -- k_sell<EPI_RESID_PREC>'s operations.  Modes 2-3: one partial per workgroup, lanes ->
// waves -> workgroup in a fixed order.  (Round 5 removed mode 1, the later steps' dots fused in:
// 215.6 vs 201.5 ms per C4 solve)
template <typename VT, bool HALO, int RL, int MODE, int GR>
__global__ __launch_bounds__(GR) __attribute__((amdgpu_waves_per_eu(GR == 512 && RL <= 5120 ? 6 : 1))) void k_g4_ring(Grid4 g, const double *__restrict__ x, const double *__restrict__ halo,
                                                const double *__restrict__ mtri, double *__restrict__ w, int n,
                                                int ngroups_per_wg, int g_lo, int g_hi, G4Dots dd, const int *stop_col,
                                                int col, int fast) {
    constexpr bool RES = MODE == 3;
    // the ring with G4RM-slot mirrors of its ends (slot t < G4RM also at RL + t, t >= RL - G4RM
    // also at t - RL): the +-1 and +-Nvy reads need no wrap
    __shared__ double ring_m[G4RM + RL + G4RM];
    double *const ring = ring_m + G4RM;
    __shared__ double tb[G4TAB];
    __shared__ double red3[3][MODE >= 2 ? GR / 64 : 1];
    double e0 = 0.0, e1 = 0.0, e2 = 0.0;   // MODE 2 / 3: the lane's sums over its rows
    if (stopped(stop_col, col)) return;
    const int tid = threadIdx.x, lane = tid & 63, ii = lane & 7;
    const int Nvy = g.Nvy, Nvx = g.Nvx, Ny = g.Ny;
    const int S2 = Nvy, S3 = Nvx * Nvy, S4 = Ny * S3;
    const int gb = g_lo + blockIdx.x * ngroups_per_wg, ge = min(g_hi, gb + ngroups_per_wg);
    const int pslot = dd.part_off + blockIdx.x;   // this workgroup's partial slot
    if (gb >= ge) {   // (no work: zero partials, so that the slots' consumers need no count)
        if (MODE >= 1 && threadIdx.x < DC_NQ) {
            const int q = threadIdx.x;
            if (MODE == 3) { if (q == 0) dd.p0[pslot] = 0.0; if (q == 1) dd.p1[pslot] = 0.0; }
            else if (q >= 2 * DC_MAXJ) dd.part[(size_t)q * GMAX + pslot] = 0.0;
        }
        return;
    }
    const int oy = 2 * Nvx, ovx = oy + 2 * Nvy, ovy = ovx + 2 * g.X;
    const int lb = g.lblk;
    // the value tables in LDS (a table load in the row loop would be a global load issued after
    // the queue's prefetch: waiting for it would wait for the whole queue)
    for (int i = tid; i < ovy + 2 * Ny; i += GR) tb[i] = g.tab[i];
    // the window's initial rows [gb GR - S3, gb GR + GR + S3), clamped to [0, n)
    for (int r = gb * GR - S3 + tid; r < gb * GR + GR + S3; r += GR)
        if (r >= 0 && r < n) {
            const int t = r % RL;
            const double v = x[r];
            ring[t] = v;
            if (t < G4RM) ring[RL + t] = v;
            if (t >= RL - G4RM) ring[t - RL] = v;
        }
    // GR in the mixed radix (Nvy, Nvx, Ny, X)
    const int a0 = GR % Nvy, q0 = GR / Nvy, a1 = q0 % Nvx, q1 = q0 / Nvx, a2 = q1 % Ny, a3 = q1 / Ny;
    struct Co {
        int jvy, jvx, iy, ix;
    };
    auto adv = [&](Co &c) {
        c.jvy += a0;
        int cy = c.jvy >= Nvy;
        c.jvy -= cy ? Nvy : 0;
        c.jvx += a1 + cy;
        cy = c.jvx >= Nvx;
        c.jvx -= cy ? Nvx : 0;
        c.iy += a2 + cy;
        cy = c.iy >= Ny;
        c.iy -= cy ? Ny : 0;
        c.ix += a3 + cy;
    };
    // the x -+ 1 plane columns of row rc (one rank: periodic inside the slab; else halo planes)
    auto xcols = [&](int rc, int &cm, int &cp) {
        if (!HALO) {
            cm = rc >= S4 ? rc - S4 : rc + (n - S4);
            cp = rc < n - S4 ? rc + S4 : rc - (n - S4);
        } else {
            cm = rc >= S4 ? rc - S4 : n + lb * S4 + rc;
            cp = rc < n - S4 ? rc + S4 : (1 - lb) * S4 + rc + S4;
        }
    };
    // element i of a kernel-argument array through a 32-bit byte offset (i < 2^28): the load
    // takes the array base in SGPRs and the offset in one VGPR (no 64-bit address per lane)
    auto at = [](const auto *base, int i) {
        using T = std::remove_cv_t<std::remove_pointer_t<decltype(base)>>;
        return *reinterpret_cast<const T *>(reinterpret_cast<const char *>(base) + (uint32_t)i * (uint32_t)sizeof(T));
    };
    auto atn = [](const auto *base, int i) {   // (non-temporal: the streamed operands)
        using T = std::remove_cv_t<std::remove_pointer_t<decltype(base)>>;
        return __builtin_nontemporal_load(
            reinterpret_cast<const T *>(reinterpret_cast<const char *>(base) + (uint32_t)i * (uint32_t)sizeof(T)));
    };
    auto xat = [&](int c) { return HALO ? *(c >= n ? halo + (c - n) : x + c) : at(x, c); };
    struct Ld {
        double xn, xm, xp, xw, m, d, b;
        Co c;
    };
    Co lead;
    {
        const int r = gb * GR + tid;
        lead.jvy = r % Nvy;
        const int t1 = r / Nvy;
        lead.jvx = t1 % Nvx;
        const int t2 = t1 / Nvx;
        lead.iy = t2 % Ny;
        lead.ix = t2 / Ny;
    }
    auto load = [&](int gl, Ld &o) {
        const int r = gl * GR + tid;
        const int rc = min(r, n - 1);
        o.xn = at(x, min(r + GR + S3, n - 1));
        int cm, cp;
        xcols(rc, cm, cp);
        o.xm = xat(cm);
        o.xp = xat(cp);
        const int cw = lead.iy == 0 ? rc + (Ny - 1) * S3 : (lead.iy == Ny - 1 ? rc - (Ny - 1) * S3 : rc);
        o.xw = at(x, min(max(cw, 0), n - 1));
        o.m = atn(mtri, rc);
        o.d = (double)atn(static_cast<const VT *>(g.D), rc);
        o.b = RES ? atn(dd.b, rc) : 0.0;
        o.c = lead;
        adv(lead);
    };
    Ld nx;
    load(gb, nx);
    int sb = (gb * GR + tid) % RL;   // ring slot of the lane's row
    auto slotp = [&](int off) {   // sb + off, 0 <= off < RL
        const int t = sb + off;
        return t >= RL ? t - RL : t;
    };
    auto slotm = [&](int off) {   // sb - off, 0 <= off < RL
        const int t = sb - off;
        return t < 0 ? t + RL : t;
    };
    __syncthreads();
    for (int gi = gb; gi < ge; ++gi) {
        const Ld cu = nx;
        // the next group's operands; across ranks not past the range's last group: the interior
        // launch runs while the comm stream writes the halo planes, which a group beyond its
        // range would read (the value was never used, the read still raced the write)
        load(HALO ? min(gi + 1, ge - 1) : gi + 1, nx);
        const int r = gi * GR + tid;
        const bool act = r < n;
        const int rc = act ? r : n - 1;
        const int jvy = cu.c.jvy, jvx = cu.c.jvx, iy = cu.c.iy, ix = cu.c.ix;
        const bool pvm = jvx > 0, pvp = jvx < Nvx - 1, pym = jvy > 0, pyp = jvy < Nvy - 1;
        const double xvm = ring[sb - S2], xvp = ring[sb + S2];   // (mirrored ends)
        const double xwm = ring[sb - 1], xwp = ring[sb + 1];
        const double x0 = ring[sb];
        const int jx = min(jvx, Nvx - 1), jy = min(jvy, Nvy - 1), kx = min(ix, g.X - 1), ky = min(iy, Ny - 1);
        const double t0 = tb[jx] * cu.xm, t8 = tb[Nvx + jx] * cu.xp;
        const double d2 = tb[ovx + kx], d6 = tb[ovx + g.X + kx], d3 = tb[ovy + ky], d5 = tb[ovy + Ny + ky];
        const double t2v = d2 * xvm, t6 = d6 * xvp, t3 = d3 * xwm, t5 = d5 * xwp, t4 = cu.d * x0;
        double s = 0.0;
        // a wave whose rows all sit inside the slab's x range and the y range (no periodic wrap, no
        // halo plane): the stored order is x-1, y-1, vx-1, vy-1, diag, vy+1, vx+1, y+1, x+1 -- the
        // general form's select chains below reduce to it term for term (the same adds in the same
        // order), without the column keys (C4: the waves off a y-line's or a slab's edge, ~95 %)
        const bool inner = act && rc >= S4 && rc < n - S4 && iy > 0 && iy < Ny - 1;
        if (fast && __builtin_amdgcn_ballot_w64(!inner) == 0) {
            const double t1y = tb[oy + jy] * ring[slotm(S3)], t7 = tb[oy + Nvy + jy] * ring[slotp(S3)];
            s = s + t0;
            s = s + t1y;
            s = pvm ? s + t2v : s;
            s = pym ? s + t3 : s;
            s = s + t4;
            s = pyp ? s + t5 : s;
            s = pvp ? s + t6 : s;
            s = s + t7;
            s = s + t8;
        } else {
            // in-plane neighbours from the ring (y wraps from the queue)
            const int cym = iy == 0 ? rc + (Ny - 1) * S3 : rc - S3;
            const int cyp = iy == Ny - 1 ? rc - (Ny - 1) * S3 : rc + S3;
            const double xym = iy == 0 ? cu.xw : ring[slotm(S3)];
            const double xyp = iy == Ny - 1 ? cu.xw : ring[slotp(S3)];
            const double t1y = tb[oy + jy] * xym, t7 = tb[oy + Nvy + jy] * xyp;
            int cm, cp;
            xcols(rc, cm, cp);
            const int64_t km = g4_key(cm, 0, n, g), kp = g4_key(cp, 8, n, g);   // stored-order positions
            auto add2 = [&](bool pa, int64_t ca, double ta, bool pb, int64_t cb, double tb2) {
                const bool sw = pa && pb && cb < ca;
                const double u1 = sw ? tb2 : ta, u2 = sw ? ta : tb2;
                const bool p1 = sw ? pb : pa, p2 = sw ? pa : pb;
                s = p1 ? s + u1 : s;
                s = p2 ? s + u2 : s;
            };
            add2(km < rc, km, t0, kp < rc, kp, t8);
            add2(cym < rc, cym, t1y, cyp < rc, cyp, t7);
            s = pvm ? s + t2v : s;
            s = pym ? s + t3 : s;
            s = s + t4;
            s = pyp ? s + t5 : s;
            s = pvp ? s + t6 : s;
            add2(cym > rc, cym, t1y, cyp > rc, cyp, t7);
            add2(km > rc, km, t0, kp > rc, kp, t8);
        }
        const double sub = (pym && ii > 0) ? 0.0 + d3 : 0.0, sup = (pyp && ii < 7) ? 0.0 + d5 : 0.0;
        // BJ, store and sums; ALL: every lane of the wave holds a row (all but the last group's
        // waves), so no lane needs the inactive-lane selects
        auto epi = [&](const bool all) {
            const bool on = all || act;
            double sv = s;
            if constexpr (RES) {   // r = b - A x (iterative.py:816)
                sv = on ? cu.b - s : 0.0;
                e0 += sv * sv;
            }
            const double z = bj_trim_group<8>(on ? sv : 0.0, lane, on ? sub : 0.0, on ? sup : 0.0, on ? cu.m : 1.0);
            if (on) st_nt<2>(reinterpret_cast<double *>(reinterpret_cast<char *>(w) + (uint32_t)r * 8u), z);
            if constexpr (RES) {
                if (on) e1 += z * z;
            } else if constexpr (MODE == 2) {
                if (on) {
                    e0 += x0 * x0;
                    e1 += x0 * z;
                    e2 += z * z;
                }
            }
        };
        if (__builtin_amdgcn_ballot_w64(!act) == 0) epi(true);
        else epi(false);
        // slide the window: the rows of group gi + 1's upper edge (their slots held rows the
        // remaining groups no longer read; the ring is > 2 S3 + 512 long)
        if (r + GR + S3 < n) {
            const int t = slotp(GR + S3);
            ring[t] = cu.xn;
            if (t < G4RM) ring[RL + t] = cu.xn;
            if (t >= RL - G4RM) ring[t - RL] = cu.xn;
        }
        sb = slotp(GR);
        __syncthreads();
    }
    if constexpr (MODE >= 2) {
        const int wid = tid >> 6;
        const double t0 = wave_sum(e0), t1 = wave_sum(e1), t2 = wave_sum(e2);
        if (lane == 0) {
            red3[0][wid] = t0;
            red3[1][wid] = t1;
            red3[2][wid] = t2;
        }
        __syncthreads();
        if (tid < 3) {
            double sum = 0.0;
#pragma unroll
            for (int wv = 0; wv < GR / 64; ++wv) sum += red3[tid][wv];
            if constexpr (MODE == 2) dd.part[(size_t)(2 * DC_MAXJ + tid) * GMAX + pslot] = sum;
            else if (tid == 0) dd.p0[pslot] = sum;
            else if (tid == 1) dd.p1[pslot] = sum;
        }
    }
}

hipError_t launch_g4_ring(const Grid4 &g, const double *x, const double *halo, const double *mtri, double *w, int64_t n,
                          int fp32, int wgs, int gr, const G4Dots *dots, int *grid_out, const int *stop_col,
                          int col, hipStream_t s, int g_lo, int g_hi, int per_in, int fast) {
    // gr: rows per group = lanes per workgroup (256 or 512)
    const int mode = dots ? dots->mode : 0;
    const int G = g4_ring_group(gr);
    const int64_t S3 = (int64_t)g.Nvx * g.Nvy, S4 = S3 * g.Ny;
    if (!g.tab || !g.D || !g4_ring_fits(g, n, gr) || S4 <= 0 || n % S4 || (halo == nullptr) != (g.lblk < 0))
        return hipErrorInvalidValue;
    // the ring: the window 2 S3 + G plus the next group's rows
    const bool small = 2 * S3 + 2 * G <= (G == 256 ? 4608 : 5120);
    const int64_t ng = (n + G - 1) / G;
    int64_t per = g4_ring_per(ng, S4, G, wgs);
    // the fused reductions write one partial per workgroup: at most GMAX workgroups
    if (mode) per = std::max<int64_t>(per, (ng + GMAX - 1) / GMAX);
    // a group range [g_lo, g_hi) of the launch (the interior / boundary planes of a rank's slab
    // around the halo exchange), groups per workgroup per_in > 0 as the caller planned them
    if (g_hi < 0) g_hi = (int)ng;
    if (per_in > 0) per = per_in;
    if (g_lo < 0 || g_lo > g_hi || g_hi > ng) return hipErrorInvalidValue;
    const int64_t span = std::max<int64_t>(1, g_hi - g_lo);
    const dim3 grid((unsigned)((span + per - 1) / per)), blk(G);
    if (mode && (dots->part_off < 0 || dots->part_off + (int64_t)grid.x > GMAX)) return hipErrorInvalidValue;
    if (mode == 1 || mode < 0 || mode > 3 || (mode == 2 && !dots->part) ||
        (mode == 3 && (!dots->b || !dots->p0 || !dots->p1)))
        return hipErrorInvalidValue;
    if (grid_out) *grid_out = (int)grid.x;
    const G4Dots dd = dots ? *dots : G4Dots{};
#define VTK_G4R(VT_, H_, RL_, M_, GR_) \
    hipLaunchKernelGGL((k_g4_ring<VT_, H_, RL_, M_, GR_>), grid, blk, 0, s, g, x, halo, mtri, w, (int)n, (int)per, g_lo, \
                       g_hi, dd, stop_col, col, fast)
#define VTK_G4R_M(VT_, H_, RL_, GR_) \
    do { \
        if (mode == 2) VTK_G4R(VT_, H_, RL_, 2, GR_); \
        else if (mode == 3) VTK_G4R(VT_, H_, RL_, 3, GR_); \
        else VTK_G4R(VT_, H_, RL_, 0, GR_); \
    } while (0)
#define VTK_G4R_PD(VT_, H_) \
    do { \
        if (G == 512) { if (small) VTK_G4R_M(VT_, H_, 5120, 512); else VTK_G4R_M(VT_, H_, 8192, 512); } \
        else if (small) VTK_G4R_M(VT_, H_, 4608, 256); \
        else VTK_G4R_M(VT_, H_, 8192, 256); \
    } while (0)
    if (fp32) {
        if (halo) VTK_G4R_PD(float, true);
        else VTK_G4R_PD(float, false);
    } else {
        if (halo) VTK_G4R_PD(double, true);
        else VTK_G4R_PD(double, false);
    }
#undef VTK_G4R_PD
#undef VTK_G4R_M
#undef VTK_G4R
    return hipGetLastError();
}

// k_lsv_ring with the solver's epilogues (one rank, canonical rows): the row sum
// exactly as k_lsv_ring / k_sell's canonical rows, then
//   EPI_RESID       r = b - A x -> y, |r|^2                         (cycle start, line path)
//   EPI_RESID_PREC  r = b - A x, z = M^-1 r -> y, |r|^2, |z|^2      (cycle start, BJ(8))
//   EPI_PREC_DC     z = M^-1 A x -> y, |x|^2, x.z, |z|^2            (DCGS2 step 0, BJ(8))
// with M^-1 the tridiagonal BJ(8) of bj_trim_group (the same operations as k_sell's TRIM
// epilogue).  The reductions: per lane over its rows in line order, then wave_sum, then the
// waves in order -- one partial per workgroup (PREC_DC: launch_dc_dots' layout).
// halo (distributed, vtk_csr::band_ghost): the two neighbour lines (blocks lblk = left and
// 1 - lblk = right of L doubles, after halo_exchange), xord their place in the stored order
struct LsvEpiK {
    const double *lsv, *x, *b, *mtri;
    double *y, *p0, *p1, *dcpart;
    int n, L, H;
    const int *stop_col;
    int col;
    const double *halo;
    int lblk, xord;
};
template <int EPI>
__global__ __launch_bounds__(BAND_T) void k_lsv_ring_epi(LsvEpiK a) {
    __shared__ double ring[4 * BAND_T];
    __shared__ double red[3][BAND_T / 64];
    if (stopped(a.stop_col, a.col)) return;
    const double *__restrict__ lsv = a.lsv;
    const double *__restrict__ x = a.x;
    const int n = a.n, L = a.L, H = a.H;
    const int tid = threadIdx.x, lane = tid & 63, ii = lane & 7, X = n / L, LP = L / H;
    const int b = blockIdx.x, R = (int)gridDim.x / H, rb = b / H, h = b % H, v0 = h * LP;
    const int xa = (int)((int64_t)rb * X / R), xb = (int)((int64_t)(rb + 1) * X / R), nl = xb - xa;
    const int v = v0 - 8 + tid;
    const bool inl = v >= 0 && v < L && tid < LP + 16;
    const bool own = tid >= 8 && tid < 8 + LP;
    const double tx0 = own ? lsv[n + v] : 0.0, tx1 = own ? lsv[n + L + v] : 0.0;
    auto line_of = [&](int it) { return it == 0 ? (xa == 0 ? X - 1 : xa - 1) : (it == nl + 1 ? (xb == X ? 0 : xb) : xa - 1 + it); };
    // the rows of iteration it's line: x, or a neighbour rank's line (the slab's x-halo) in halo
    const double *hal = a.halo;
    auto line_ptr = [&](int it) -> const double * {
        if (hal && it == 0 && xa == 0) return hal + (int64_t)a.lblk * L;
        if (hal && it == nl + 1 && xb == X) return hal + (int64_t)(1 - a.lblk) * L;
        return x + (int64_t)line_of(it) * L;
    };
    auto slot = [&](int it) { return (it & 3) * BAND_T; };
    constexpr bool BJ = EPI == EPI_RESID_PREC || EPI == EPI_PREC_DC;
    constexpr bool HB = EPI == EPI_RESID || EPI == EPI_RESID_PREC;
    double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
    // prefetch: x of line_of(it), and D (m, b) of line it - 1 (computed at iteration it)
    double nxv = inl ? __builtin_nontemporal_load(line_ptr(0) + v) : 0.0, nd = 0.0, nm = 1.0, nb = 0.0;
    for (int it = 0; it <= nl + 1; ++it) {
        ring[slot(it) + tid] = nxv;
        const double drow = nd, mrow = nm, brow = nb;
        if (it <= nl) {
            nxv = inl ? __builtin_nontemporal_load(line_ptr(it + 1) + v) : 0.0;
            if (own && it + 1 >= 2) {
                const int64_t rr = (int64_t)(xa + it - 1) * L + v;
                nd = __builtin_nontemporal_load(lsv + rr);
                if constexpr (BJ) nm = __builtin_nontemporal_load(a.mtri + rr);
                if constexpr (HB) nb = __builtin_nontemporal_load(a.b + rr);
            }
        }
        __syncthreads();
        if (it >= 2) {
            const int xl = xa + it - 2;
            const double tv0 = lsv[n + 2 * L + xl], tv1 = lsv[n + 2 * L + X + xl];
            int64_t cxm, cxp;
            const int ord = __builtin_amdgcn_readfirstlane(canon_order_xv(xl, 0, n, L, X, hal ? a.lblk : -1, cxm, cxp, a.xord));
            constexpr int P_MID = 0 | 1 << 3 | 2 << 6 | 3 << 9 | 4 << 12;
            constexpr int P_FIRST = 1 | 2 << 3 | 3 << 6 | 4 << 9 | 0 << 12;
            const int sx = slot(it - 1);
            const double t0 = tx0 * ring[slot(it - 2) + tid];
            const double t4 = tx1 * ring[slot(it) + tid];
            const double xr = ring[sx + tid];
            const double t2 = drow * xr;
            const double t1 = tv0 * ring[sx + tid - (tid > 0 ? 1 : 0)];
            const double t3 = tv1 * ring[sx + tid + (tid < BAND_T - 1 ? 1 : 0)];
            const bool h1 = v > 0, h3 = v < L - 1;
            double sa = 0.0;
            if (ord == P_MID) {
                sa = sa + t0;
                sa = h1 ? sa + t1 : sa;
                sa = sa + t2;
                sa = h3 ? sa + t3 : sa;
                sa = sa + t4;
            } else if (ord == P_FIRST) {
                sa = h1 ? sa + t1 : sa;
                sa = sa + t2;
                sa = h3 ? sa + t3 : sa;
                sa = sa + t4;
                sa = sa + t0;
            } else {
                sa = sa + t4;
                sa = sa + t0;
                sa = h1 ? sa + t1 : sa;
                sa = sa + t2;
                sa = h3 ? sa + t3 : sa;
            }
            const int64_t row = (int64_t)xl * L + v;
            double out = sa;
            if constexpr (HB) {
                out = own ? brow - sa : 0.0;   // r = b - A x
                acc0 += out * out;
            }
            if constexpr (BJ) {
                const double sub = (own && h1 && ii > 0) ? 0.0 + tv0 : 0.0;
                const double sup = (own && h3 && ii < 7) ? 0.0 + tv1 : 0.0;
                const double z = bj_trim_group<8>(own ? out : 0.0, lane, sub, sup, own ? mrow : 1.0);
                if constexpr (EPI == EPI_RESID_PREC) {
                    if (own) acc1 += z * z;
                } else {
                    if (own) {
                        acc0 += xr * xr;
                        acc1 += xr * z;
                        acc2 += z * z;
                    }
                }
                out = z;
            }
            if (own) st_nt<2>(a.y + row, out);
        }
    }
    const int wid = tid >> 6;
    const double t0 = wave_sum(acc0), t1 = wave_sum(acc1), t2 = wave_sum(acc2);
    if (lane == 0) {
        red[0][wid] = t0;
        red[1][wid] = t1;
        red[2][wid] = t2;
    }
    __syncthreads();
    if (tid < 3) {
        double sum = 0.0;
#pragma unroll
        for (int w = 0; w < BAND_T / 64; ++w) sum += red[tid][w];
        if constexpr (EPI == EPI_PREC_DC) a.dcpart[(size_t)(2 * DC_MAXJ + tid) * GMAX + b] = sum;
        else if (tid == 0) a.p0[b] = sum;
        else if (tid == 1 && EPI == EPI_RESID_PREC) a.p1[b] = sum;
    }
}

hipError_t launch_lsv_ring_epi(int epi, const double *lsv, const double *x, const double *b, const double *mtri,
                               double *y, double *p0, double *p1, double *dcpart, int64_t n, int L, int ring_wgs,
                               const int *stop_col, int col, int *grid_out, hipStream_t s, const double *halo, int lblk,
                               int xord) {
    const int H = band_parts(L);
    const int64_t X = L > 0 ? n / L : 0;
    if (n <= 0 || n > INT32_MAX / 2 || L <= 0 || n % L != 0 || H < 1 || X < (halo ? 2 : 3) || ring_wgs < 1 ||
        (halo && (lblk < 0 || lblk > 1)))
        return hipErrorInvalidValue;
    const bool bj = epi == EPI_RESID_PREC || epi == EPI_PREC_DC;
    if ((bj && !mtri) || ((epi == EPI_RESID || epi == EPI_RESID_PREC) && (!b || !p0)) ||
        (epi == EPI_RESID_PREC && !p1) || (epi == EPI_PREC_DC && !dcpart) || L % 8 != 0)
        return hipErrorInvalidValue;
    // one partial per workgroup: at most GMAX
    const int64_t R = std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(ring_wgs / H, X / 2), GMAX / H));
    LsvEpiK a{lsv, x, b, mtri, y, p0, p1, dcpart, (int)n, L, H, stop_col, col, halo, halo ? lblk : -1, halo ? xord : 0};
    const dim3 g((unsigned)(R * H)), blk(BAND_T);
    if (grid_out) *grid_out = (int)g.x;
    switch (epi) {
        case EPI_RESID: hipLaunchKernelGGL(k_lsv_ring_epi<EPI_RESID>, g, blk, 0, s, a); break;
        case EPI_RESID_PREC: hipLaunchKernelGGL(k_lsv_ring_epi<EPI_RESID_PREC>, g, blk, 0, s, a); break;
        case EPI_PREC_DC: hipLaunchKernelGGL(k_lsv_ring_epi<EPI_PREC_DC>, g, blk, 0, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_lsv_spmv(const uint32_t *pk, const int32_t *dict, const double *lsv, const double *x,
                           const double *halo, double *y, int64_t n, int L, int lblk, const int *stop_col, int col,
                           hipStream_t s, int canon, int grid_cap, int ring_wgs, int xord) {
    if (n <= 0 || n > INT32_MAX / 2 || L <= 0 || n % L != 0 || (halo && lblk < 0)) return hipErrorInvalidValue;
    if (ring_wgs > 0 && canon && !halo) {   // the LDS-staged form (one rank, canonical rows)
        const int H = band_parts(L);
        const int64_t X = n / L;
        if (H >= 1 && X >= 3) {
            const int64_t R = std::max<int64_t>(1, std::min<int64_t>(ring_wgs / H, X / 2));
            hipLaunchKernelGGL(k_lsv_ring, dim3((unsigned)(R * H)), dim3(BAND_T), 0, s, lsv, x, y, (int)n, L, H, stop_col, col);
            return hipGetLastError();
        }
    }
    const int64_t nch = (n + 63) / 64;
    // grid_cap: 8192 workgroups by default (vtk::Tuning::lsv_spmv_cap; C3 line solve, in-process
    // A/B: 8.69 ms vs 8.73 at 2048 and 8.85 with one chunk per wave; an XCD swizzle of the chunks
    // 8.81 vs 8.70)
    const int64_t cap = grid_cap > 0 ? grid_cap : 8192;
    const int64_t g = std::max<int64_t>(1, std::min<int64_t>((nch + 3) / 4, cap));
    if (canon && halo) hipLaunchKernelGGL((k_lsv_spmv<true, true>), dim3((unsigned)g), dim3(NT), 0, s, pk, dict, lsv, x, halo, y, (int)n, L, lblk, xord, stop_col, col);
    else if (canon) hipLaunchKernelGGL((k_lsv_spmv<false, true>), dim3((unsigned)g), dim3(NT), 0, s, pk, dict, lsv, x, halo, y, (int)n, L, lblk, xord, stop_col, col);
    else if (halo) hipLaunchKernelGGL(k_lsv_spmv<true>, dim3((unsigned)g), dim3(NT), 0, s, pk, dict, lsv, x, halo, y, (int)n, L, lblk, xord, stop_col, col);
    else hipLaunchKernelGGL(k_lsv_spmv<false>, dim3((unsigned)g), dim3(NT), 0, s, pk, dict, lsv, x, halo, y, (int)n, L, lblk, xord, stop_col, col);
    return hipGetLastError();
}

// *bad |= 1 when a column lies outside lines x-1..x+1 (mod X) of its row's line x; |= 2 when it
// lies more than one row off the row's position v within its line
__global__ __launch_bounds__(NT) void k_band_check(const int32_t *__restrict__ indptr, const int32_t *__restrict__ indices,
                                                   int64_t n, int L, int X, int *bad) {
    for (int64_t r = (int64_t)blockIdx.x * NT + threadIdx.x; r < n; r += (int64_t)gridDim.x * NT) {
        const int64_t x = r / L, vr = r % L;
        bool ok = true, vloc = true;
        for (int k = indptr[r]; k < indptr[r + 1]; ++k) {
            const int64_t c = indices[k];
            if (c < 0 || c >= n) { ok = false; break; }
            int64_t rel = c / L - x;
            if (rel > 1) rel -= X;
            else if (rel < -1) rel += X;
            if (rel < -1 || rel > 1) { ok = false; break; }
            const int64_t dv = c % L - vr;
            if (dv < -1 || dv > 1) vloc = false;
        }
        if (!ok) atomicOr(bad, 1);
        if (!vloc) atomicOr(bad, 2);
    }
}

hipError_t launch_band_check(const int32_t *indptr, const int32_t *indices, int64_t n, int L, int X, int *bad,
                             hipStream_t s) {
    int64_t g = (n + NT - 1) / NT;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    hipLaunchKernelGGL(k_band_check, dim3((unsigned)g), dim3(NT), 0, s, indptr, indices, n, L, X, bad);
    return hipGetLastError();
}

}  // namespace vtk
