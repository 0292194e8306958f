// vtk_device.hpp — device helpers shared by the gfx950 kernel translation units
// (vtk_kernels.hip, vtk_band.hip): deterministic wave / workgroup reductions, DPP lane moves,
// non-temporal load/store wrappers, the tridiagonal block-Jacobi group solves, the Hessenberg
// back substitution and the DCGS2 x update.  Device code only; not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <float.h>

#include "vtk_internal.hpp"

namespace vtk {

// canonical line-band row (every row of the 2D Vlasov operators): the couplings to lines x - 1
// (kind 0) and x + 1 (4), to v - 1 (1, absent at v = 0) and v + 1 (3, absent at v = L - 1) and
// the diagonal (2), stored in ascending column order.  The columns of x -+ 1 in local numbering:
// one rank periodic ((x -+ 1) mod X) L + v; across ranks the first / last line's outer
// neighbour is a halo line (n + block L + v).  VM, D, VP are always in that order; the x
// couplings sort before them ("small") or after them by their GLOBAL column (the stored CSR
// order): locally numbered lines by position; across ranks the left halo line before the row
// (a lower rank's line) and the right one after it, except where the slab starts at global line
// 0 (xord bit 0: its left neighbour is the last line, after the row) or ends at the last line
// (bit 1: its right neighbour is line 0, before the row).  Two couplings on the same side sort
// x + 1 first (one rank: the wrapped line; across ranks: the lower global line).  The same for
// every v of a line.  Returns the 5 kinds in stored order, 3 bits each.
__device__ __forceinline__ int canon_order_xv(int64_t x, int64_t v, int64_t n, int L, int X, int lblk, int64_t &cxm,
                                              int64_t &cxp, int xord = 0) {
    const int64_t r = x * L + v;
    bool ms, ps;   // "small": stored before the line's own entries
    if (lblk < 0) {   // (x -+ 1) mod X for 0 <= x < X, by selects (no 64-bit division)
        cxm = (x == 0 ? X - 1 : x - 1) * L + v;
        cxp = (x == X - 1 ? 0 : x + 1) * L + v;
        ms = cxm < r;
        ps = cxp < r;
    } else {
        cxm = x >= 1 ? r - L : n + (int64_t)lblk * L + v;
        cxp = x <= X - 2 ? r + L : n + (int64_t)(1 - lblk) * L + v;
        ms = x >= 1 || !(xord & 1);
        ps = x == X - 1 && (xord & 2);
    }
    int ord = 0, k = 0;
    auto put = [&](int kind) { ord |= kind << (3 * k++); };
    if (ms && ps) { put(4); put(0); }
    else if (ms) put(0);
    else if (ps) put(4);
    put(1);
    put(2);
    put(3);
    if (!ms && !ps) { put(4); put(0); }
    else if (!ms) put(0);
    else if (!ps) put(4);
    return ord;
}
__device__ __forceinline__ int canon_order(int64_t r, int64_t n, int L, int X, int lblk, int64_t &cxm, int64_t &cxp,
                                           int xord = 0) {
    return canon_order_xv(r / L, r % L, n, L, X, lblk, cxm, cxp, xord);
}

// the entries of canonical row (xl, v) -- row = xl L + v, local numbering, n local rows, X = n / L
// lines -- in stored order from the line-separable tables lsv = D[n] | TX[2][L] | TV[2][X]
// (vtk_band.hip k_lsv_build): column c[e] (-1: kind absent at v = 0 / L - 1) and value d[e].
// The SELL copy of the same row holds the same columns and values in the same order, padding
// after them, so a sum over these in order equals the SELL sum bit for bit
__device__ __forceinline__ void canon_row(const double *__restrict__ lsv, int n, int L, int lblk, int xl, int v,
                                          double drow, int (&c)[5], double (&d)[5], int xord = 0) {
    const int X = n / L, row = xl * L + v;
    int64_t cxm, cxp;
    const int ord = canon_order_xv(xl, v, n, L, X, lblk, cxm, cxp, xord);
#pragma unroll
    for (int e = 0; e < 5; ++e) {
        const int kind = (ord >> (3 * e)) & 7;
        if (kind == 0) { c[e] = (int)cxm; d[e] = lsv[(size_t)n + v]; }
        else if (kind == 4) { c[e] = (int)cxp; d[e] = lsv[(size_t)n + L + v]; }
        else if (kind == 2) { c[e] = row; d[e] = drow; }
        else if (kind == 1) { c[e] = v > 0 ? row - 1 : -1; d[e] = v > 0 ? lsv[(size_t)n + 2 * L + xl] : 0.0; }
        else { c[e] = v < L - 1 ? row + 1 : -1; d[e] = v < L - 1 ? lsv[(size_t)n + 2 * L + X + xl] : 0.0; }
    }
}

// ---- 4D grid rows (vtk::Grid4) -------------------------------------------------------------
// kinds in the order of a row without periodic wraps: 0 x-1, 1 y-1, 2 vx-1, 3 vy-1, 4 diagonal,
// 5 vy+1, 6 vx+1, 7 y+1, 8 x+1.  Table slot of kind k's value: tab[g4_slot(k, coordinates)]
struct G4Row {
    int ix, iy, jvx, jvy;
};
__device__ __forceinline__ G4Row g4_coords(int64_t r, const Grid4 &g) {
    G4Row q;
    q.jvy = (int)(r % g.Nvy);
    int64_t t = r / g.Nvy;
    q.jvx = (int)(t % g.Nvx);
    t /= g.Nvx;
    q.iy = (int)(t % g.Ny);
    q.ix = (int)(t / g.Ny);
    return q;
}
__device__ __forceinline__ int g4_slot(int kind, const G4Row &q, const Grid4 &g) {
    const int oy = 2 * g.Nvx, ovx = oy + 2 * g.Nvy, ovy = ovx + 2 * g.X;
    switch (kind) {
        case 0: return q.jvx;
        case 8: return g.Nvx + q.jvx;
        case 1: return oy + q.jvy;
        case 7: return oy + g.Nvy + q.jvy;
        case 2: return ovx + q.ix;
        case 6: return ovx + g.X + q.ix;
        case 3: return ovy + q.iy;
        default: return ovy + g.Ny + q.iy;   // 5
    }
}
// the nine kinds' columns of local row r (n local rows) and whether the row has them (vx, vy
// Dirichlet); x neighbours periodic inside the slab on one rank (lblk < 0), else halo planes
__device__ __forceinline__ void g4_cols(int64_t r, const G4Row &q, const Grid4 &g, int64_t n, int64_t (&c)[9],
                                        bool (&p)[9]) {
    const int64_t S2 = g.Nvy, S3 = (int64_t)g.Nvx * g.Nvy, S4 = (int64_t)g.Ny * S3;
    const int64_t rest = r - (int64_t)q.ix * S4;
    if (g.lblk < 0) {
        c[0] = (int64_t)(q.ix == 0 ? g.X - 1 : q.ix - 1) * S4 + rest;
        c[8] = (int64_t)(q.ix == g.X - 1 ? 0 : q.ix + 1) * S4 + rest;
    } else {
        c[0] = q.ix >= 1 ? r - S4 : n + (int64_t)g.lblk * S4 + rest;
        c[8] = q.ix <= g.X - 2 ? r + S4 : n + (int64_t)(1 - g.lblk) * S4 + rest;
    }
    c[1] = q.iy == 0 ? r + (int64_t)(g.Ny - 1) * S3 : r - S3;
    c[7] = q.iy == g.Ny - 1 ? r - (int64_t)(g.Ny - 1) * S3 : r + S3;
    c[2] = r - S2;
    c[6] = r + S2;
    c[3] = r - 1;
    c[5] = r + 1;
    c[4] = r;
#pragma unroll
    for (int k = 0; k < 9; ++k) p[k] = true;
    p[2] = q.jvx > 0;
    p[6] = q.jvx < g.Nvx - 1;
    p[3] = q.jvy > 0;
    p[5] = q.jvy < g.Nvy - 1;
}

// a grid column's position in the row's stored order: local columns as they are; a halo plane's
// column (k = 0: the x - 1 plane, 8: x + 1) before or after every local one (Grid4::xord)
__device__ __forceinline__ int64_t g4_key(int64_t c, int k, int64_t n, const Grid4 &g) {
    if (c < n) return c;
    constexpr int64_t BIG = (int64_t)1 << 40;
    const bool after = k == 0 ? (g.xord & 1) != 0 : (g.xord & 2) == 0;
    return after ? BIG + c : c - BIG;
}

// Bijective XCD swizzle (cdna_hip_programming.md T1): workgroups are dealt round-robin over the
// 8 XCDs, so b and b + 8 share an L2.  The logical id gives the blocks sharing an XCD one
// contiguous id range; with the grid-stride tile loop an XCD then works on a contiguous window
// of tiles at a time and neighbouring tiles' x halos (+-nv rows on the 2D operator) hit its L2.
// Speed only: the partial of workgroup b stays at index b, every mapping is fixed.
__device__ __forceinline__ int xcd_swizzle(int b, int g) {
    constexpr int NX = 8;
    const int q = g / NX, r = g % NX, x = b % NX;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / NX;
}

// ------------------------------------------------------------------------------------------
// reductions
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ double wave_allsum(double v);
__device__ __forceinline__ double wave_sum(double v) {
    return wave_allsum(v);  // (every lane; callers read lane 0)
}

// every thread of the workgroup returns the same total (fixed order)
__device__ __forceinline__ double block_sum(double v, double *red) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) s += red[i];
    return s;
}

// sum of p[i0], p[i0+STRIDE], ... (< cnt <= U*STRIDE) in that order, with every load issued
// before the first add (a rolled loop paid one L2 round trip per element)
template <int U, int STRIDE>
__device__ __forceinline__ double strided_sum(const double *p, int cnt, int i0) {
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int i = i0 + u * STRIDE;
        v[u] = i < cnt ? p[i] : 0.0;
    }
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
    return acc;
}
static_assert(GMAX <= 4 * NT && GMAX <= 16 * 64, "partial-sum unroll bounds");

__device__ __forceinline__ double reduce_red(Red r, double *red) {
    return block_sum(strided_sum<GMAX / NT, NT>(r.p, r.cnt, threadIdx.x), red);
}

__device__ __forceinline__ bool stopped(const int *stop_col, int col) {
    // wave-uniform: one scalar load
    return stop_col != nullptr && __builtin_nontemporal_load(stop_col) < col;
}

// The basis vector an MGS step subtracts (and the basis read by the x update) is loaded
// non-temporal, 16 B per lane, so that w stays resident in the 256 MB Infinity Cache across
// the chain of MGS kernels: on C3 (20M rows) an MGS step went from 122 us to 98 us
// (tools/probe_mgs.hip).  Narrow (4/8 B) nt loads are slow on gfx950; the SpMV keeps plain loads.
typedef double d2v __attribute__((ext_vector_type(2)));
template <typename T>
__device__ __forceinline__ T ldnt(const T *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ d2v ldnt2(const double *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const d2v *>(p));
}
// cache policy per operand class ("Cache policy"): non-temporal vector stores of
// streamed-out results re-read only by a later kernel (NT_STORES bits: 1 scale0 / x update --
// neutral, off; 2 SpMV epilogues, plain SpMV 243 -> 223 us; 4 line apply, line solve +0.8 %) and
// non-temporal loads of operands read once per kernel (NT_LOADS bits: 1 fused BJ m, +2.5 % on
// the C3 BJ path; 4 dots p/w and 8 line apply r/m, +1 % on the line path)
constexpr int NT_STORES = 6, NT_LOADS = 13;
// write-through (sc1) store of a streamed-out result: the line leaves the XCD's L2 with the store,
// so the release at the kernel's end finds no dirty lines to write back (plain and nt stores keep
// them: MI355X_MICROARCH.md, store flavours).  The band step's v_j / w stores: C3/8 slab
// 9 811 -> 9 971 it/s, C3 +0.5 % (round 5)
__device__ __forceinline__ void st_wt(double *p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int BIT>
__device__ __forceinline__ double ld_nt(const double *p) {
    if constexpr ((NT_LOADS & BIT) != 0) return __builtin_nontemporal_load(p);
    else return *p;
}
template <int BIT>
__device__ __forceinline__ double2 ld_nt2(const double *p) {
    if constexpr ((NT_LOADS & BIT) != 0) {
        const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v *>(p));
        return make_double2(v.x, v.y);
    } else {
        return *reinterpret_cast<const double2 *>(p);
    }
}
template <int BIT>
__device__ __forceinline__ void st_nt(double *p, double v) {
    if constexpr ((NT_STORES & BIT) != 0) __builtin_nontemporal_store(v, p);
    else *p = v;
}
template <int BIT>
__device__ __forceinline__ void st_nt2(double *p, double x, double y) {
    if constexpr ((NT_STORES & BIT) != 0) __builtin_nontemporal_store(d2v{x, y}, reinterpret_cast<d2v *>(p));
    else *reinterpret_cast<double2 *>(p) = make_double2(x, y);
}


// ------------------------------------------------------------------------------------------
// DPP lane moves (CDNA row-level data-parallel primitives: 16-lane rows, a VALU modifier
// instead of an LDS-crossbar ds_bpermute).  Lanes whose source falls outside their row read 0.
// Only the transport changes: a scan written with these moves does the same IEEE operations.
// ------------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}
constexpr int DPP_ROW_SHL = 0x100;   // + n: lane i <- lane i + n of its row
constexpr int DPP_ROW_SHR = 0x110;   // + n: lane i <- lane i - n of its row
// __shfl_up / __shfl_down within groups of W <= 16 lanes (W divides 16): the lanes a group
// would take from outside itself are exactly those the callers mask off
template <int W>
__device__ __forceinline__ double grp_up(double v, int off) {
    if constexpr (W <= 16) {
        switch (off) {
            case 1: return dpp_mov<DPP_ROW_SHR + 1>(v);
            case 2: return dpp_mov<DPP_ROW_SHR + 2>(v);
            case 4: return dpp_mov<DPP_ROW_SHR + 4>(v);
            default: return dpp_mov<DPP_ROW_SHR + 8>(v);
        }
    } else {
        return __shfl_up(v, off, W);
    }
}
template <int W>
__device__ __forceinline__ double grp_down(double v, int off) {
    if constexpr (W <= 16) {
        switch (off) {
            case 1: return dpp_mov<DPP_ROW_SHL + 1>(v);
            case 2: return dpp_mov<DPP_ROW_SHL + 2>(v);
            case 4: return dpp_mov<DPP_ROW_SHL + 4>(v);
            default: return dpp_mov<DPP_ROW_SHL + 8>(v);
        }
    } else {
        return __shfl_down(v, off, W);
    }
}

// Block-Jacobi apply with tridiagonal blocks, BS lanes per block (one row each): the LU solve
// L d = y, U z = d as two affine scans over the group (log2 BS shuffle steps each):
//   d_i = y_i - l_i d_{i-1},   z_i = m_i d_i - g_i z_{i+1}   (m_i = 1/u_i, g_i = sup_i / u_i)
// Same M^-1 as the inverse rows to rounding; 24 B per row instead of 8 BS.
template <int BS>
__device__ __forceinline__ double bj_tri_group(double y, bool act, int64_t row, int lane, const double *tri,
                                               int64_t ld) {
    const int ii = lane & (BS - 1);
    double l = 0.0, m = 1.0, g = 0.0;
    if (act) {
        l = tri[row];
        m = tri[ld + row];
        g = tri[2 * ld + row];
    }
    double A = y, B = -l;
#pragma unroll
    for (int off = 1; off < BS; off <<= 1) {
        const double Ap = grp_up<BS>(A, off), Bp = grp_up<BS>(B, off);
        if (ii >= off) {
            A = A + B * Ap;
            B = B * Bp;
        }
    }
    A = m * A;
    B = -g;
#pragma unroll
    for (int off = 1; off < BS; off <<= 1) {
        const double An = grp_down<BS>(A, off), Bn = grp_down<BS>(B, off);
        if (ii + off < BS) {
            A = A + B * An;
            B = B * Bn;
        }
    }
    return A;
}

// The same solve from m alone (SELL kernels): the lane has its row's block sub/super-diagonal
// entries from the SpMV loop (duplicates summed in stored order, as in the setup), so
// l_i = sub_i m_{i-1} (m_{i-1} from the neighbour lane) and g_i = sup_i m_i: 8 B per row.
template <int BS>
__device__ __forceinline__ double bj_trim_group(double y, int lane, double sub, double sup, double m) {
    const int ii = lane & (BS - 1);
    const double mprev = grp_up<BS>(m, 1);
    const double l = ii > 0 ? sub * mprev : 0.0;
    const double g = sup * m;
    double A = y, B = -l;
#pragma unroll
    for (int off = 1; off < BS; off <<= 1) {
        const double Ap = grp_up<BS>(A, off), Bp = grp_up<BS>(B, off);
        if (ii >= off) {
            A = A + B * Ap;
            B = B * Bp;
        }
    }
    A = m * A;
    B = -g;
#pragma unroll
    for (int off = 1; off < BS; off <<= 1) {
        const double An = grp_down<BS>(A, off), Bn = grp_down<BS>(B, off);
        if (ii + off < BS) {
            A = A + B * An;
            B = B * Bn;
        }
    }
    return A;
}

// ------------------------------------------------------------------------------------------
// wave reductions by DPP moves and readlanes
__device__ __forceinline__ double readlane_f64(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}
// sum over the wavefront, the same bits in every lane: xor-1/xor-2 quad permutes, half-row and
// row mirrors (each step adds a lane pair that both end up equal, a + b = b + a), then the four
// row sums in a fixed order.  DPP moves and readlanes: no LDS traffic.
__device__ __forceinline__ double wave_allsum(double v) {
    v = v + dpp_mov<0xB1>(v);    // quad_perm [1,0,3,2]
    v = v + dpp_mov<0x4E>(v);    // quad_perm [2,3,0,1]
    v = v + dpp_mov<0x141>(v);   // row_half_mirror
    v = v + dpp_mov<0x140>(v);   // row_mirror
    return (readlane_f64(v, 0) + readlane_f64(v, 16)) + (readlane_f64(v, 32) + readlane_f64(v, 48));
}

// ------------------------------------------------------------------------------------------
// x += y @ V[0..col] with y from the (m+1) x m Hessenberg least squares
// (iterative.py:799-814).  Workgroup-redundant triangular solve on lane 0, into LDS.
// ------------------------------------------------------------------------------------------
// y = H^-1 S over columns 0..col (lane 0 of a workgroup, into LDS ys; iterative.py:799-812)
__device__ inline void hess_solve(const double *__restrict__ H, const double *__restrict__ S, int m, int col,
                                  double *ys) {
    const int M1 = m + 1;
    for (int k = 0; k <= col; ++k) ys[k] = S[k];
    if (H[(size_t)col * M1 + col] == 0.0) ys[col] = 0.0;
    for (int k = col; k > 0; --k) {
        if (ys[k] != 0.0) {
            ys[k] = ys[k] / H[(size_t)k * M1 + k];
            const double t = ys[k];
            for (int i = 0; i < k; ++i) ys[i] = ys[i] - t * H[(size_t)k * M1 + i];
        }
    }
    if (ys[0] != 0.0) ys[0] = ys[0] / H[0];
}

// v_j = (p_j - sum_k s_k v_k) / r  (in place, j >= 1);  p_{j+1} = (w - sum_k e_k v_k - e_j v_j) * q
// (the update pass stores v_j and p_{j+1} non-temporal: A/B +2.6 % it/s)
// The cycle's x update in the update pass of the step whose scalar kernel stopped it (xup_tag):
// c = stop_col is j-1 (column j-1 finalised in step j: V[0..j-1] all stored) or j (column j
// committed early: v_j = (p_j - V_j s) / r formed here exactly as the normal pass would store
// it).  Same operations and order as k_xupdate, so x is bit-identical to the unfused path.
// FM: p_j's recompute and v_j's formation as fused multiply-adds (k_band_step's form)
template <int XB, bool FM = false>
static __device__ __forceinline__ void dc_xupdate_body(const double *__restrict__ V, int64_t ld, int j, int c,
                                                       int64_t n, const DcCoef *cf, double *__restrict__ x,
                                                       const double *__restrict__ H, const double *__restrict__ S,
                                                       int m, const double *__restrict__ wprev,
                                                       const double *__restrict__ pj_at = nullptr) {
    __shared__ double ys[DC_MAXJ + 1], cs[DC_MAXJ], ep[DC_MAXJ];
    __shared__ double rinv_s, qp_s;
    // wprev (line-band step): p_j is not stored; recompute it as step j-1 formed it
    const bool rec = c == j && j >= 1 && wprev != nullptr;
    if (threadIdx.x == 0) {
        hess_solve(H, S, m, c, ys);
        rinv_s = cf->rinv;
        qp_s = cf->q_prev;
    }
    if (c == j)
        for (int k = threadIdx.x; k < j; k += blockDim.x) {
            cs[k] = cf->s[k];
            ep[k] = cf->e_prev[k];
        }
    __syncthreads();
    const double rinv = rinv_s, qp = qp_s;
    // p_j: V[j] (the update pass stores it there), or pj_at (the line sweep keeps p apart)
    const double *pj = pj_at ? pj_at : V + (size_t)j * ld;
    const int kv = c == j ? j : c + 1;   // stored basis vectors in the sum
    const int64_t stride = 2 * (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = 2 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x); i < n; i += stride) {
        if (i + 1 < n) {
            double ax = 0.0, ay = 0.0;
            double2 a = make_double2(0.0, 0.0);
            // XB > 1: the basis rows in batches of XB loads issued together; the sums in ascending
            // k either way
            if (rec) {
                const d2v wp = ldnt2(wprev + i);
                double tx = wp.x, ty = wp.y;
                int k = 0;
                if constexpr (XB > 1)
                for (; k + XB <= j; k += XB) {
                    d2v v[XB];
#pragma unroll
                    for (int u = 0; u < XB; ++u) v[u] = ldnt2(V + (size_t)(k + u) * ld + i);
#pragma unroll
                    for (int u = 0; u < XB; ++u) {
                        tx = FM ? __builtin_fma(-ep[k + u], v[u].x, tx) : tx - ep[k + u] * v[u].x;
                        ty = FM ? __builtin_fma(-ep[k + u], v[u].y, ty) : ty - ep[k + u] * v[u].y;
                    }
                }
                for (; k < j; ++k) {
                    const d2v v = ldnt2(V + (size_t)k * ld + i);
                    tx = FM ? __builtin_fma(-ep[k], v.x, tx) : tx - ep[k] * v.x;
                    ty = FM ? __builtin_fma(-ep[k], v.y, ty) : ty - ep[k] * v.y;
                }
                a = make_double2(tx * qp, ty * qp);
            } else if (c == j) {
                const d2v pp = ldnt2(pj + i);
                a = make_double2(pp.x, pp.y);
            }
            auto acc1 = [&](int k, const d2v &v) {
                ax += ys[k] * v.x;
                ay += ys[k] * v.y;
                if (c == j) {
                    const double sk = cs[k];
                    a.x = FM ? __builtin_fma(-sk, v.x, a.x) : a.x - sk * v.x;
                    a.y = FM ? __builtin_fma(-sk, v.y, a.y) : a.y - sk * v.y;
                }
            };
            int k = 0;
            if constexpr (XB > 1)
            for (; k + XB <= kv; k += XB) {
                d2v v[XB];
#pragma unroll
                for (int u = 0; u < XB; ++u) v[u] = ldnt2(V + (size_t)(k + u) * ld + i);
#pragma unroll
                for (int u = 0; u < XB; ++u) acc1(k + u, v[u]);
            }
            for (; k < kv; ++k) acc1(k, ldnt2(V + (size_t)k * ld + i));
            if (c == j) {
                const double vx = j >= 1 ? a.x * rinv : a.x, vy = j >= 1 ? a.y * rinv : a.y;
                ax += ys[j] * vx;
                ay += ys[j] * vy;
            }
            double2 xv = *reinterpret_cast<const double2 *>(x + i);
            xv.x = xv.x + ax;
            xv.y = xv.y + ay;
            st_wt(x + i, xv.x);   // (write-through: C3 x update 652 -> 630 us, C4 1 615 -> 1 558 us)
            st_wt(x + i + 1, xv.y);
        } else {
            double ax = 0.0, a = c == j ? pj[i] : 0.0;
            if (rec) {
                double t = wprev[i];
                for (int k = 0; k < j; ++k) t = FM ? __builtin_fma(-ep[k], V[(size_t)k * ld + i], t) : t - ep[k] * V[(size_t)k * ld + i];
                a = t * qp;
            }
            for (int k = 0; k < kv; ++k) {
                const double v = V[(size_t)k * ld + i];
                ax += ys[k] * v;
                if (c == j) a = FM ? __builtin_fma(-cs[k], v, a) : a - cs[k] * v;
            }
            if (c == j) ax += ys[j] * (j >= 1 ? a * rinv : a);
            x[i] = x[i] + ax;
        }
    }
}


}  // namespace vtk
