// vtk_kernels.hip — hand-written gfx950 (MI355X, CDNA4) kernels of the preconditioned-Krylov
// path.  Built with -ffp-contract=off: every + - * / is one IEEE-rounded operation, so the
// SpMV row sums (serial, ascending column order — scipy sparsetools csr_matvec), the BJ
// apply (serial over the block row) and the BJ setup (Gauss-Jordan, partial pivoting) are
// bit-identical to the CPU restatement in oracle/vtk_oracle.c.
//
// Reductions are deterministic: each workgroup of a fixed grid (G <= GMAX, a function of n
// only) writes one partial; every consumer workgroup sums the G partials in one fixed order,
// so all workgroups (and all runs) see the same scalar.  No float atomics anywhere.
//
// Wavefront = 64 lanes.  Geometry and rooflines: DESIGN.md §3.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <float.h>

#include <climits>
#include <type_traits>
#include <cstdlib>

#include "vtk_internal.hpp"
#include "vtk_vlasov.hpp"
#include "vtk_device.hpp"
#include "vtk_scalar.hpp"

namespace vtk {

// ------------------------------------------------------------------------------------------
// CSR SpMV, CSR-stream tiles: a workgroup stages one tile's products val*x[col] in LDS with
// fully coalesced reads of data/indices, then one lane per row sums its products serially.
// Rows longer than TILE_NNZ form single-row tiles reduced by the whole workgroup.
// ------------------------------------------------------------------------------------------
template <typename VT, bool HALO>
struct SpmvK {
    const int32_t *indptr, *indices;
    const VT *data;
    const int32_t *tile_row, *tile_end;   // tile_end null: tile t ends where t+1 starts
    int ntiles, n_local;
    const double *x, *halo;
    double *y;
    const double *b, *inv, *v0;
    double *part0, *part1;
    const int *stop_col;
    int col;
    const double *tri;   // TRI: l | m | g factors of tridiagonal blocks, stride tri_ld
    int64_t tri_ld;
    const double *V;   // EPI_PREC_DC: basis, leading dimension, step, partials
    int64_t ld;
    int j;
    double *dcpart;
    // SELL-64 layout (k_sell): chunk q = rows 64q..64q+63, entry k of row 64q+l at
    // sell_off[q] + 64k + l, col -1 = padding; groups of 4 chunks (256 rows), optional list
    const int64_t *sell_off;
    const int32_t *sell_col;
    const VT *sell_val;
    const int32_t *group_list;
    int ngroups;
    // dictionary-coded columns (Sell::d_pk; null: int32 columns everywhere)
    const uint32_t *pk;
    const int64_t *pk_off;
    const int32_t *dict;
    int sell_uw;   // Sell::uniform_w (0: read the offsets)
    // line-separable values (vtk_csr::d_lsv, solver launches only; null: the SELL values): the
    // entry's value from its column -- the same value, so the same sums
    const double *lsv;
    int lsv_L, lsv_lblk;
    int lsv_xord;   // across ranks: where the halo lines sort in the stored order (canon_order_xv)
    int canon;   // with lsv: every row canonical (vtk_csr::lsv_canon): columns from canon_row
    int swz;     // XCD-aware group order (xcd_swizzle; vtk::Tuning::sell_swz)
    Grid4 g4;    // 4D grid rows: columns from the coordinates, values from D / tables (g4.tab null: off)
};

// value of entry (row, c) from the line-separable tables; drow = D[row], (xl, v) the row's line
// and position (vtk_band.hip k_lsv_build)
template <typename VT, bool HALO>
__device__ __forceinline__ double lsv_value(const SpmvK<VT, HALO> &a, int row, int c, double drow, int xl, int v) {
    const int off = c - row, L = a.lsv_L, X = a.n_local / L;
    if (off == 0) return drow;
    if (off == 1 || off == -1) return a.lsv[(size_t)a.n_local + 2 * L + (off > 0 ? X : 0) + xl];
    // the periodic wrap only on one rank (lblk < 0): across ranks a slab of two lines has
    // -(X - 1) L == -L, the x - 1 coupling
    const bool up = (HALO && c >= a.n_local) ? ((c - a.n_local) / L != a.lsv_lblk)
                                             : (off == L || (a.lsv_lblk < 0 && off == -(X - 1) * L));
    return a.lsv[(size_t)a.n_local + (up ? L : 0) + v];
}

template <typename VT, bool HALO>
__device__ __forceinline__ double xload(const SpmvK<VT, HALO> &a, int c) {
    if (HALO) return c < a.n_local ? a.x[c] : a.halo[c - a.n_local];
    return a.x[c];
}


template <int BS>
__device__ __forceinline__ void load_inv_row(const double *irow, double (&m)[BS]) {
    if constexpr (BS % 2 == 0) {
#pragma unroll
        for (int j = 0; j < BS; j += 2) {
            const double2 t = *reinterpret_cast<const double2 *>(irow + j);
            m[j] = t.x;
            m[j + 1] = t.y;
        }
    } else {
#pragma unroll
        for (int j = 0; j < BS; ++j) m[j] = irow[j];
    }
}


// DCGS2 dots of rows [i0, i1) of a tile, w and p staged in LDS (wt, pt): wave wv owns the basis
// vectors k = wv, wv + 4, ...; W = 2: 16-byte loads of V (the tile's first row even)
constexpr int DC_KPW = DC_MAXJ / (NT / 64);
struct DcAcc {
    double s[DC_KPW], z[DC_KPW], aa, ab, ag;
};
template <int W>
__device__ __forceinline__ void dc_rows(DcAcc &d, const double *vb, int64_t ld, int j, const double *pt,
                                        const double *wt, int nr, int lane, int wv) {
    for (int i = W * lane; i < nr; i += W * 64) {
        const bool two = W == 2 && i + 1 < nr;
        double pv[2], wv2[2];
        pv[0] = pt[i]; wv2[0] = wt[i];
        pv[1] = two ? pt[i + 1] : 0.0; wv2[1] = two ? wt[i + 1] : 0.0;
#pragma unroll
        for (int u = 0; u < DC_KPW; ++u) {
            const int k = wv + u * (NT / 64);
            if (k < j) {
                const double *vk = vb + (size_t)k * ld + i;
                double v0, v1 = 0.0;
                if (two) {   // streamed once here (re-read by the update pass, not from cache)
                    const d2v t = ldnt2(vk);
                    v0 = t.x; v1 = t.y;
                } else {
                    v0 = vk[0];
                }
                d.s[u] += v0 * pv[0];
                d.z[u] += v0 * wv2[0];
                if (W == 2) { d.s[u] += v1 * pv[1]; d.z[u] += v1 * wv2[1]; }
            }
        }
        if (wv == 0) {
#pragma unroll
            for (int h = 0; h < W; ++h) {
                d.aa += pv[h] * pv[h];
                d.ab += pv[h] * wv2[h];
                d.ag += wv2[h] * wv2[h];
            }
        }
    }
}

// per-workgroup partials in launch_dc_dots' layout (part[q * GMAX + block]); red >= DC_NQ doubles
__device__ __forceinline__ void dc_write(const DcAcc &d, int j, double *red, double *part) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int u = 0; u < DC_KPW; ++u) {
        const int k = wv + u * (NT / 64);
        const double ts = wave_sum(d.s[u]);
        const double tz = wave_sum(d.z[u]);
        if (lane == 0 && k < j) { red[k] = ts; red[DC_MAXJ + k] = tz; }
    }
    {
        const double t0 = wave_sum(d.aa), t1 = wave_sum(d.ab), t2 = wave_sum(d.ag);
        if (wv == 0 && lane == 0) { red[2 * DC_MAXJ] = t0; red[2 * DC_MAXJ + 1] = t1; red[2 * DC_MAXJ + 2] = t2; }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < DC_NQ; q += NT) {
        const bool used = q < j || (q >= DC_MAXJ && q < DC_MAXJ + j) || q >= 2 * DC_MAXJ;
        if (used) part[(size_t)q * GMAX + blockIdx.x] = red[q];
    }
}

// Epilogue of one row (both layouts): y[row] from the row sum s, per-lane partial sums.  All
// lanes of the wave call it (the BJ groups exchange values by shuffles); act = a real row.
// Returns the value written (w for the DCGS2 dots).
// TRIM: the tridiagonal solve from m and the row's sub/sup (SELL); else from l | m | g.
template <typename VT, bool HALO, int EPI, int BS, bool TRI, bool TRIM = false>
__device__ __forceinline__ double row_epilogue(const SpmvK<VT, HALO> &a, double s, int row, bool act, int lane,
                                               double &acc0, double &acc1, double sub = 0.0, double sup = 0.0,
                                               bool have_m = false, double mrow = 1.0, bool store = true,
                                               bool have_bv = false, double bv = 0.0, double v0v = 0.0) {
    constexpr bool DC = EPI == EPI_PREC_DC;
    if constexpr (EPI == EPI_PLAIN) {
        if (act) st_nt<2>(a.y + row, s);
        return s;
    } else if constexpr (EPI == EPI_RESID) {
        const double r = act ? (have_bv ? bv : a.b[row]) - s : 0.0;
        if (act) {
            st_nt<2>(a.y + row, r);
            acc0 += r * r;
        }
        return r;
    } else {
        // PREC: z = M^-1 (A x);  RESID_PREC: r = b - A x (iterative.py:816), z = M^-1 r
        double sv = s;
        if constexpr (EPI == EPI_RESID_PREC) {
            sv = act ? (have_bv ? bv : a.b[row]) - s : 0.0;
            acc0 += sv * sv;
        }
        double z = sv;
        if constexpr (BS > 0 && TRI && TRIM) {
            if (!have_m) mrow = act ? a.tri[a.tri_ld + row] : 1.0;
            z = bj_trim_group<BS>(sv, lane, sub, sup, mrow);
        } else if constexpr (BS > 0 && TRI) {
            z = bj_tri_group<BS>(sv, act, row, lane, a.tri, a.tri_ld);
        } else if constexpr (BS > 0) {
            // z_i = sum_j inv[i][j] * y_j over the BS lanes of this block
            double m[BS];
            if (act) load_inv_row<BS>(a.inv + (size_t)row * BS, m);
            const int gb = lane & ~(BS - 1);
            z = 0.0;
#pragma unroll
            for (int j = 0; j < BS; ++j) {
                const double yj = __shfl(sv, gb + j, 64);
                if (act) z += m[j] * yj;
            }
        }
        if (act) {
            if (store) {
                if constexpr (DC) __builtin_nontemporal_store(z, a.y + row);   // (A/B: fused 593 -> 582 us)
                else st_nt<2>(a.y + row, z);
            }
            if constexpr (EPI == EPI_RESID_PREC) {
                acc1 += z * z;
            } else if constexpr (!DC) {
                acc0 += z * z;
                if (a.v0) acc1 += (have_bv ? v0v : a.v0[row]) * z;
            }
        }
        return act ? z : 0.0;
    }
}

// EPI: 0 plain, 1 residual, 2 preconditioned (BS == 0: identity, else block-Jacobi of size BS),
// 3 residual + preconditioned, 4 preconditioned + DCGS2 dots
// 4 waves/SIMD = the LDS-bound occupancy (4 workgroups of 35 KB per CU): caps VGPRs at 128
template <typename VT, bool HALO, int EPI, int BS, bool TRI = false>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void k_spmv(SpmvK<VT, HALO> a) {
    __shared__ double prod[TILE_NNZ];
    __shared__ int rp[TILE_ROWS + 1];
    __shared__ double red[NT / 64];
    static_assert(2 * TILE_ROWS <= TILE_NNZ && DC_NQ <= TILE_NNZ, "DC staging in prod[]");
    if (stopped(a.stop_col, a.col)) return;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    constexpr bool DC = EPI == EPI_PREC_DC;
    double acc0 = 0.0, acc1 = 0.0;
    DcAcc dc;
    if constexpr (DC) {
#pragma unroll
        for (int u = 0; u < DC_KPW; ++u) { dc.s[u] = 0.0; dc.z[u] = 0.0; }
        dc.aa = dc.ab = dc.ag = 0.0;
    }
    for (int t = xcd_swizzle(blockIdx.x, gridDim.x); t < a.ntiles; t += gridDim.x) {
        const int r0 = a.tile_row[t], r1 = a.tile_end ? a.tile_end[t] : a.tile_row[t + 1], nr = r1 - r0;
        const int nz0 = a.indptr[r0], nnz = a.indptr[r1] - nz0;
        if (nnz <= TILE_NNZ) {
            // Plain (cached) loads here: non-temporal 4/8-byte loads ran this kernel 25% slower
            // (tools/probe_fused.hip: 603 -> 751 us on C3), and neither prefetching the BJ rows
            // nor a deeper unroll helped.
            for (int i = tid; i <= nr; i += NT) rp[i] = a.indptr[r0 + i] - nz0;
            const int32_t *ci = a.indices + nz0;
            const VT *cv = a.data + nz0;
            int e = tid;
            constexpr int U = 4;
            for (; e + (U - 1) * NT < nnz; e += U * NT) {
                int c[U];
                double d[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    c[u] = ci[e + u * NT];
                    d[u] = (double)cv[e + u * NT];
                }
#pragma unroll
                for (int u = 0; u < U; ++u) prod[e + u * NT] = d[u] * xload(a, c[u]);
            }
            for (; e < nnz; e += NT) prod[e] = (double)cv[e] * xload(a, ci[e]);
            __syncthreads();
            double zk[TILE_ROWS / NT];
#pragma unroll
            for (int u = 0; u < TILE_ROWS / NT; ++u) {
                const int base = u * NT;
                if (base >= nr) break;
                const int i = base + tid;
                const bool act = i < nr;
                double s = 0.0;
                if (act) {
                    const int k1 = rp[i + 1];
                    for (int k = rp[i]; k < k1; ++k) s += prod[k];
                }
                const int row = r0 + i;
                const double z = row_epilogue<VT, HALO, EPI, BS, TRI>(a, s, row, act, lane, acc0, acc1);
                if constexpr (DC) zk[u] = z;
            }
            __syncthreads();
            if constexpr (DC) {
                // stage the tile's w and p in the (now free) product buffer, then the dots
                double *wt = prod, *pt = prod + TILE_ROWS;
#pragma unroll
                for (int u = 0; u < TILE_ROWS / NT; ++u) {
                    const int i = u * NT + tid;
                    if (i < nr) { wt[i] = zk[u]; pt[i] = a.x[r0 + i]; }
                }
                __syncthreads();
                // fused BJ tiles start on a block boundary: even rows for even BS (16-B loads)
                constexpr int W = (BS >= 2 && BS % 2 == 0) ? 2 : 1;
                dc_rows<W>(dc, a.V + r0, a.ld, a.j, pt, wt, nr, lane, tid >> 6);
                __syncthreads();
            }
        } else if constexpr (!DC) {   // (DC: BJ-fused tiles never hold long rows)
            // long rows (each such tile is a single row): workgroup-strided products
            for (int i = 0; i < nr; ++i) {
                const int row = r0 + i;
                const int k0 = a.indptr[row], k1 = a.indptr[row + 1];
                double s = 0.0;
                for (int k = k0 + tid; k < k1; k += NT) s += (double)a.data[k] * xload(a, a.indices[k]);
                s = block_sum(s, red);
                if (tid == 0) {
                    if constexpr (EPI == EPI_PLAIN) {
                        a.y[row] = s;
                    } else if constexpr (EPI == EPI_RESID) {
                        const double r = a.b[row] - s;
                        a.y[row] = r;
                        acc0 += r * r;
                    } else if constexpr (EPI == EPI_RESID_PREC) {
                        const double r = a.b[row] - s;   // BS == 0 only (host guarantees)
                        a.y[row] = r;
                        acc0 += r * r;
                        acc1 += r * r;
                    } else {
                        a.y[row] = s;   // BS == 0 only (host guarantees)
                        acc0 += s * s;
                        if (a.v0) acc1 += a.v0[row] * s;
                    }
                }
            }
        }
    }
    if constexpr (DC) {
        dc_write(dc, a.j, prod, a.dcpart);
        return;
    }
    if constexpr (EPI != EPI_PLAIN && !DC) {
        const double t0 = block_sum(acc0, red);
        if (tid == 0) a.part0[blockIdx.x] = t0;
        if (EPI == EPI_RESID_PREC || (EPI == EPI_PREC && a.v0 != nullptr)) {
            const double t1 = block_sum(acc1, red);
            if (tid == 0) a.part1[blockIdx.x] = t1;
        }
    }
}

// ------------------------------------------------------------------------------------------
// CSR SpMV in the SELL-64 layout (built on the device from the CSR when its padding is small,
// vtk_api.cpp): one wavefront per 64-row chunk, lane l = row 64q+l, entries column-major in the
// chunk.  Every lane sums its row's products serially in stored order (padding skipped), so y
// is bit-identical to csr_matvec and to k_spmv.  No LDS and no barriers on the SpMV itself; a
// workgroup takes a group of 4 chunks (256 contiguous rows).  col/val are streamed once:
// non-temporal loads (tools/probe_sell.hip, C3: 291 us vs 348 us for the CSR-stream tiles,
// bit-identical).
//
// DCGS2 dots (EPI_PREC_DC), wave-local: each lane already holds its row's w and p, so the wave
// reads V[k][row] for every k < j itself (4 loads in flight per batch, no LDS staging, no
// barrier).  The first JB = 10 vectors accumulate per lane in registers and are reduced once
// at the end; vectors beyond are reduced per chunk with a butterfly (every lane gets the same
// bits) and lane k keeps their running sums.  C3: the LDS-staged split of the vectors over the
// waves cost 462 us + 33.4 us per vector, butterflies for every vector 320 us + 68 us, this
// ~360 us + 29 us per register vector.  Tried and measured slower on one box (A/B): 20
// register vectors at 3 waves/SIMD (-2 %), k >= 10 handed to k_dc_dots (-3 %).
// ------------------------------------------------------------------------------------------

constexpr int DC_KB = 4;   // basis vectors per load batch (fused DC step)
constexpr int DC_JB = 10;   // basis vectors with per-lane register accumulators (fused DC step)
constexpr int DC_PSW = 4;   // entries per load batch of the fused DC step (runtime widths)
// compile-time chunk width of the uniform-width SELL copies the stencil operators produce (2D
// Vlasov: 5, 4D: 9); 0 = the runtime-width loop
constexpr int DC_JB9 = 10;   // ... at width 9 (C4)
constexpr int DC_PSW9 = 9;   // DC load batch at width 9 (C4)
constexpr int SELL_WPE = 4;   // minimum waves/SIMD the SELL kernels are register-limited to
// WU > 0: every chunk is WU entries wide (Sell::uniform_w == WU, checked by the launch): the
// chunk's code words are all issued with its dictionary and the entry loop has compile-time
// bounds, so a row wider than one code word (C4: 9 entries) costs no extra dependent round trip
// for its second word and no batch boundary at the word edge.
// VAR bit 0 (plain SpMV): padding slots branch around their gather instead of gathering the
// lane's own row (the unconditional gather the 9-wide C4 rows want)
template <typename VT, bool HALO, int EPI, int BS, bool TRI = false, int PSWT = 0, int WU = 0, int VAR = 0>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(SELL_WPE))) void k_sell(SpmvK<VT, HALO> a) {
    // entries per load batch (DC: registers; PSWT: a row length the launch picked; WU without
    // PSWT: the whole row in one batch)
    constexpr int PSW = PSWT > 0 ? PSWT : (WU > 0 ? WU : (EPI == EPI_PREC_DC ? DC_PSW : 8));
    constexpr int KB = DC_KB;   // basis vectors per load batch (DC)
    // basis vectors with per-lane register accumulators (DC; the 9-wide rows hold more operands)
    constexpr int JB = WU > 8 ? DC_JB9 : DC_JB;
    constexpr bool DC = EPI == EPI_PREC_DC;
    constexpr bool HOIST = DC;
    constexpr bool HOISTE = !DC && EPI != EPI_PLAIN;   // the other epilogues (residual: -13 %)
    constexpr int NQW = 2 * DC_MAXJ + 3;      // per-wave partial record (DC)
    __shared__ double stage[(NT / 64) * NQW];
    __shared__ double red[NT / 64];
    if (stopped(a.stop_col, a.col)) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    double acc0 = 0.0, acc1 = 0.0;
    double dsl = 0.0, dzl = 0.0, daa = 0.0, dab = 0.0, dag = 0.0;   // DC
    double as_[DC ? JB : 1], az_[DC ? JB : 1];
    if constexpr (DC) {
#pragma unroll
        for (int k = 0; k < JB; ++k) { as_[k] = 0.0; az_[k] = 0.0; }
    }
    const int t0 = a.swz ? xcd_swizzle(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    for (int t = t0; t < a.ngroups; t += gridDim.x) {
        const int g = a.group_list ? a.group_list[t] : t;
        const int q = __builtin_amdgcn_readfirstlane(4 * g + wv);
        const int row = 64 * q + lane;
        const bool act = row < a.n_local;
        double s = 0.0;
        double sub = 0.0, sup = 0.0;   // TRI: the row's block sub/super-diagonal entries
        constexpr bool TRIM = TRI && BS > 0;
        [[maybe_unused]] const int ii = lane & (BS > 0 ? BS - 1 : 0);
        // HOIST: the row's own operands (BJ factor m, p, b, v0) issued ahead of the CSR loads,
        // so the epilogue does not wait a memory round trip per chunk (EPI_PREC: 352 -> ... us)
        double mrow = 1.0, pv = 0.0, bv = 0.0, v0v = 0.0;
        if constexpr (HOIST) {
            if (act) {
                if constexpr (TRIM) mrow = ld_nt<1>(a.tri + a.tri_ld + row);
                pv = a.x[row];
            }
        } else if constexpr (HOISTE) {
            if (act) {
                if constexpr (TRIM) mrow = ld_nt<1>(a.tri + a.tri_ld + row);
                if constexpr (EPI == EPI_RESID || EPI == EPI_RESID_PREC) bv = a.b[row];
                if constexpr (EPI == EPI_PREC) {
                    if (a.v0) v0v = a.v0[row];
                }
            }
        }
        // products of one batch, summed serially in stored order (padding skipped)
        auto batch = [&](const auto &c, const auto &d, auto mid) {
            constexpr int NB = sizeof(c) / sizeof(c[0]);
            double xv[NB];
#pragma unroll
            for (int u = 0; u < NB; ++u) {
                // UNCOND: padding slots gather the lane's own x[row] (the line of its diagonal
                // entry) instead of branching around the load: the gathers issue back to back
                // with no exec-mask blocks.  (x[0] for every padding slot measured 1.6x slower on
                // C4: one hot L2 line for the whole chip.)
                if constexpr (!(VAR & 1)) xv[u] = xload(a, c[u] >= 0 ? c[u] : (act ? row : 0));
                else xv[u] = c[u] >= 0 ? xload(a, c[u]) : 0.0;
            }
            mid();
#pragma unroll
            for (int u = 0; u < NB; ++u)
                if (c[u] >= 0) s += d[u] * xv[u];
            if constexpr (TRIM) {
#pragma unroll
                for (int u = 0; u < NB; ++u) {
                    if (c[u] == row - 1 && ii > 0) sub = sub + d[u];
                    if (c[u] == row + 1 && ii < BS - 1) sup = sup + d[u];
                }
            }
        };
        // canonical line-band rows with line-separable values (a.canon): every entry's column
        // and value from the row's line and position -- no code words, dictionary or values
        // loaded, so the gathers issue with the row's diagonal instead of after two dependent
        // round trips; the same entries in the same order as the SELL copy (canon_row)
        // (not in the plain SpMV: vtk_spmv, the measured standalone SpMV, never has lsv, and the
        // extra path cost its loop 249 -> 372 us on C3 through code shape alone)
        constexpr bool CANON_OK = std::is_same<VT, double>::value && (WU == 0 || WU == 5) && EPI != EPI_PLAIN;
        constexpr bool G4_OK = (WU == 0 || WU == 9) && EPI != EPI_PLAIN && (VAR & 2) == 0;
        // the line-separable tables are a solver-launch form: compiled out of the plain SpMV (its
        // per-entry value selection cost the measured kernel 222 -> 242 us on C3)
        constexpr bool LSV_OK = EPI != EPI_PLAIN;
        // 4D grid rows (vtk::Grid4, checked bit for bit at setup): the nine couplings' columns
        // from the row's coordinates, their values from D and the per-coordinate tables, summed
        // in the stored (ascending column) order -- the SELL sum, without codes or values
        auto g4_rows = [&]() {
            if (64 * q < a.n_local) {
                const Grid4 &g = a.g4;
                // coordinates: the chunk's first row by divisions (wave-uniform), then the lane
                const int r0 = 64 * q;
                int jvy = r0 % g.Nvy, t4 = r0 / g.Nvy;
                int jvx = t4 % g.Nvx;
                t4 /= g.Nvx;
                int iy = t4 % g.Ny, ix = t4 / g.Ny;
                jvy += lane;
                while (jvy >= g.Nvy) {
                    jvy -= g.Nvy;
                    if (++jvx == g.Nvx) {
                        jvx = 0;
                        if (++iy == g.Ny) {
                            iy = 0;
                            ++ix;
                        }
                    }
                }
                if (!act) ix = iy = jvx = jvy = 0;
                const G4Row qq{ix, iy, jvx, jvy};
                int64_t c9[9];
                bool p9[9];
                g4_cols(row, qq, g, a.n_local, c9, p9);
                const double *tb = g.tab;
                const int oy = 2 * g.Nvx, ovx = oy + 2 * g.Nvy, ovy = ovx + 2 * g.X;
                double d9[9];
                d9[0] = tb[jvx];
                d9[8] = tb[g.Nvx + jvx];
                d9[1] = tb[oy + jvy];
                d9[7] = tb[oy + g.Nvy + jvy];
                d9[2] = tb[ovx + ix];
                d9[6] = tb[ovx + g.X + ix];
                d9[3] = tb[ovy + iy];
                d9[5] = tb[ovy + g.Ny + iy];
                d9[4] = act ? (double)__builtin_nontemporal_load(static_cast<const VT *>(g.D) + row) : 0.0;
                double xv[9];
#pragma unroll
                for (int k = 0; k < 9; ++k) xv[k] = xload(a, act && p9[k] ? (int)c9[k] : (act ? row : 0));
                double tk[9];
#pragma unroll
                for (int k = 0; k < 9; ++k) tk[k] = d9[k] * xv[k];
                // two couplings of one direction on the same side of the row: in column order
                auto add2 = [&](bool pa, int64_t ca, double ta, bool pb, int64_t cb, double tb2) {
                    const bool sw = pa && pb && cb < ca;
                    const double t1 = sw ? tb2 : ta, t2 = sw ? ta : tb2;
                    const bool p1 = sw ? pb : pa, p2 = sw ? pa : pb;
                    s = p1 ? s + t1 : s;
                    s = p2 ? s + t2 : s;
                };
                // the x planes' positions in the stored order (halo planes: Grid4::xord)
                const int64_t k0 = g4_key(c9[0], 0, a.n_local, g), k8 = g4_key(c9[8], 8, a.n_local, g);
                if (act) {
                    // x planes before the row's plane, then y lines before its line (periodic
                    // wraps), the in-line block, the y lines and x planes after
                    add2(k0 < row, k0, tk[0], k8 < row, k8, tk[8]);
                    add2(c9[1] < row, c9[1], tk[1], c9[7] < row, c9[7], tk[7]);
                    s = p9[2] ? s + tk[2] : s;
                    s = p9[3] ? s + tk[3] : s;
                    s = s + tk[4];
                    s = p9[5] ? s + tk[5] : s;
                    s = p9[6] ? s + tk[6] : s;
                    add2(c9[1] > row, c9[1], tk[1], c9[7] > row, c9[7], tk[7]);
                    add2(k0 > row, k0, tk[0], k8 > row, k8, tk[8]);
                    if constexpr (TRIM) {
                        if (p9[3] && ii > 0) sub = sub + d9[3];
                        if (p9[5] && ii < BS - 1) sup = sup + d9[5];
                    }
                }
            }
        };
        // G4ONLY (VAR bit 1): an instantiation with the grid-row form alone (no SELL code path
        // competing for registers: the 9-wide C4 kernels spilled with both)
        if constexpr ((VAR & 2) != 0) {
            g4_rows();
        } else
        if (CANON_OK && a.canon) {
            if (64 * q < a.n_local) {
                const int L = a.lsv_L;
                int xl = (64 * q) / L, v = 64 * q - xl * L + lane;
                while (v >= L) {
                    v -= L;
                    ++xl;
                }
                int c[5];
                double d[5];
                if (act) {
                    canon_row(a.lsv, a.n_local, L, a.lsv_lblk, xl, v, __builtin_nontemporal_load(a.lsv + row), c, d, a.lsv_xord);
                } else {
#pragma unroll
                    for (int u = 0; u < 5; ++u) {
                        c[u] = -1;
                        d[u] = 0.0;
                    }
                }
                batch(c, d, [] {});
            }
        } else if (G4_OK && a.g4.tab != nullptr) {
            g4_rows();
        } else if constexpr (WU > 0) {
            if (64 * q < a.n_local) {
                constexpr int NWD = (WU + 7) / 8;   // 4-bit code words per lane
                const int64_t o0 = (int64_t)q * 64 * WU;
                const VT *vv = a.sell_val + o0 + lane;
                uint32_t wd[NWD];
                int dv = 0;
                bool wide = true;   // wave-uniform
                VT dall[WU];   // raw (fp32 values: one VGPR each until used)
                if (a.pk) {
                    const uint32_t *pw = a.pk + (int64_t)q * 64 * NWD + lane;
#pragma unroll
                    for (int u = 0; u < NWD; ++u) wd[u] = __builtin_nontemporal_load(pw + u * 64);
                    dv = lane < 16 ? a.dict[(int64_t)q * 16 + lane] : 0;
                }
                // the row's values do not depend on the column form: issued with the codes and
                // the dictionary, before the form test waits for the dictionary
                if (!(LSV_OK && a.lsv)) {
#pragma unroll
                    for (int k = 0; k < WU; ++k) dall[k] = __builtin_nontemporal_load(vv + k * 64);
                }
                // line-separable values: the row's diagonal, line and position
                double lsv_d = 0.0;
                int lsv_x = 0, lsv_v = 0;
                if (LSV_OK && a.lsv) {
                    lsv_x = (64 * q) / a.lsv_L;
                    lsv_v = 64 * q - lsv_x * a.lsv_L + lane;
                    while (lsv_v >= a.lsv_L) {
                        lsv_v -= a.lsv_L;
                        ++lsv_x;
                    }
                    if (act) lsv_d = __builtin_nontemporal_load(a.lsv + row);
                }
                if (a.pk) wide = __shfl(dv, 15, 64) != 0;
                // one copy of the unrolled entry loop per column form (no branch inside it)
                auto entries = [&](auto wide_c) {
                    constexpr bool WIDE = decltype(wide_c)::value;
                    const int32_t *cc = a.sell_col + o0 + lane;
#pragma unroll
                    for (int k0 = 0; k0 < WU; k0 += PSW) {
                        int c[PSW];
                        double d[PSW];
#pragma unroll
                        for (int u = 0; u < PSW; ++u) {
                            const int k = k0 + u;
                            if (k >= WU) {
                                c[u] = -1;
                                d[u] = 0.0;
                                continue;
                            }
                            if constexpr (WIDE) {
                                c[u] = __builtin_nontemporal_load(cc + k * 64);
                            } else {
                                const int code = (int)((wd[k >> 3] >> (4 * (k & 7))) & 15u);
                                const int off = __shfl(dv, code, 64);
                                c[u] = code != PK_CODES ? row + off : -1;
                            }
                            d[u] = (LSV_OK && a.lsv) ? (c[u] >= 0 ? lsv_value(a, row, c[u], lsv_d, lsv_x, lsv_v) : 0.0) : (double)dall[k];
                        }
                        batch(c, d, [] {});
                    }
                };
                if (wide) entries(std::true_type{});
                else entries(std::false_type{});
            }
        } else if (64 * q < a.n_local) {
            // uniform widths: offsets from q (no scalar loads ahead of the value / code loads)
            const int64_t o0 = a.sell_uw ? (int64_t)q * 64 * a.sell_uw : a.sell_off[q];
            const int w = a.sell_uw ? a.sell_uw : (int)((a.sell_off[q + 1] - o0) >> 6);
            const VT *vv = a.sell_val + o0 + lane;
            // columns: dictionary codes (one 32-bit word per 8 entries of a lane), or int32
            // for "wide" chunks / unpacked copies; wave-uniform choice, one code path
            bool wide = true;
            int dv = 0;
            // WORD_EARLY: the first code word is loaded together with the dictionary (every chunk
            // has its pk words, wide or not), not after the wide test has seen the dictionary
            const uint32_t *pw = a.pk ? a.pk + (a.sell_uw ? (int64_t)q * 64 * ((a.sell_uw + 7) / 8) : a.pk_off[q]) + lane
                                      : nullptr;
            const uint32_t word0 = (a.pk && w > 0) ? __builtin_nontemporal_load(pw) : 0u;
            if (a.pk) {   // the chunk's dictionary: one 64-B load by lanes 0..15
                dv = lane < 16 ? a.dict[(int64_t)q * 16 + lane] : 0;
                wide = __shfl(dv, 15, 64) != 0;
            }
            const int32_t *cc = a.sell_col + o0 + lane;
            double lsv_d = 0.0;
            int lsv_x = 0, lsv_v = 0;
            if (LSV_OK && a.lsv) {
                lsv_x = (64 * q) / a.lsv_L;
                lsv_v = 64 * q - lsv_x * a.lsv_L + lane;
                while (lsv_v >= a.lsv_L) {
                    lsv_v -= a.lsv_L;
                    ++lsv_x;
                }
                if (act) lsv_d = __builtin_nontemporal_load(a.lsv + row);
            }
            for (int k0 = 0; k0 < w; k0 += 8) {
                const uint32_t word = wide ? 0u
                                           : ((k0 == 0) ? word0
                                                                          : __builtin_nontemporal_load(pw + (k0 >> 3) * 64));
#pragma unroll
                for (int h = 0; h < 8; h += PSW) {
                    if (k0 + h >= w) break;   // wave-uniform
                    int c[PSW];
                    double d[PSW];
                    if (wide) {
#pragma unroll
                        for (int u = 0; u < PSW; ++u) {
                            const int k = k0 + h + u;
                            c[u] = (h + u < 8 && k < w) ? __builtin_nontemporal_load(cc + k * 64) : -1;
                        }
                    } else {
#pragma unroll
                        for (int u = 0; u < PSW; ++u) {
                            const int code = h + u < 8 ? (int)((word >> (4 * (h + u))) & 15u) : PK_CODES;
                            const int off = __shfl(dv, code, 64);
                            c[u] = code != PK_CODES ? row + off : -1;
                        }
                    }
                    // values do not wait for the codes: padding slots hold 0 and are skipped
#pragma unroll
                    for (int u = 0; u < PSW; ++u) {
                        if (LSV_OK && a.lsv) d[u] = c[u] >= 0 ? lsv_value(a, row, c[u], lsv_d, lsv_x, lsv_v) : 0.0;
                        else d[u] = (h + u < 8 && k0 + h + u < w)
                                        ? (double)__builtin_nontemporal_load(vv + (k0 + h + u) * 64) : 0.0;
                    }
                    batch(c, d, [] {});
                }
            }
        }
        const double z = row_epilogue<VT, HALO, EPI, BS, TRI, TRIM>(a, s, row, act, lane, acc0, acc1, sub, sup,
                                                                    (HOIST || HOISTE) && TRIM, mrow, true,
                                                                    HOISTE, bv, v0v);
        if constexpr (DC) {
            if constexpr (!HOIST) pv = act ? a.x[row] : 0.0;   // p_j (= the SpMV input) on this row
            daa += pv * pv;
            dab += pv * z;
            dag += z * z;
            const double *vb = a.V + row;
#pragma unroll
            for (int k0 = 0; k0 < JB; k0 += KB) {
                if (k0 >= a.j) break;   // wave-uniform
                double v[KB];
#pragma unroll
                for (int u = 0; u < KB; ++u) {
                    v[u] = (k0 + u < JB && k0 + u < a.j && act)
                               ? __builtin_nontemporal_load(vb + (size_t)(k0 + u) * a.ld) : 0.0;
                }
#pragma unroll
                for (int u = 0; u < KB; ++u) {
                    if (k0 + u < JB) {   // compile-time after unrolling: JB need not divide by KB
                        as_[k0 + u] += v[u] * pv;
                        az_[k0 + u] += v[u] * z;
                    }
                }
            }
            for (int k0 = JB; k0 < a.j; k0 += KB) {
                double v[KB];
#pragma unroll
                for (int u = 0; u < KB; ++u)
                    v[u] = (k0 + u < a.j && act) ? __builtin_nontemporal_load(vb + (size_t)(k0 + u) * a.ld) : 0.0;
#pragma unroll
                for (int u = 0; u < KB; ++u) {
                    if (k0 + u < a.j) {   // wave-uniform
                        const double ts = wave_allsum(v[u] * pv), tz = wave_allsum(v[u] * z);
                        if (lane == k0 + u) {
                            dsl += ts;
                            dzl += tz;
                        }
                    }
                }
            }
        }
    }
    if constexpr (DC) {
        // per-block partials in launch_dc_dots' layout: the 4 waves' records summed in order
        double *rec = stage + wv * NQW;
        if (lane >= JB && lane < a.j) {
            rec[lane] = dsl;
            rec[DC_MAXJ + lane] = dzl;
        }
#pragma unroll
        for (int k = 0; k < JB; ++k) {
            if (k < a.j) {   // wave-uniform
                const double ts = wave_sum(as_[k]), tz = wave_sum(az_[k]);
                if (lane == 0) {
                    rec[k] = ts;
                    rec[DC_MAXJ + k] = tz;
                }
            }
        }
        const double t0 = wave_sum(daa), t1 = wave_sum(dab), t2 = wave_sum(dag);
        if (lane == 0) {
            rec[2 * DC_MAXJ] = t0;
            rec[2 * DC_MAXJ + 1] = t1;
            rec[2 * DC_MAXJ + 2] = t2;
        }
        __syncthreads();
        for (int qq = tid; qq < DC_NQ; qq += NT) {
            const bool used = qq < a.j || (qq >= DC_MAXJ && qq < DC_MAXJ + a.j) || qq >= 2 * DC_MAXJ;
            if (used) {
                double t = 0.0;
#pragma unroll
                for (int w2 = 0; w2 < NT / 64; ++w2) t += stage[w2 * NQW + qq];
                a.dcpart[(size_t)qq * GMAX + blockIdx.x] = t;
            }
        }
        return;
    }
    if constexpr (EPI != EPI_PLAIN) {
        const double t0 = block_sum(acc0, red);
        if (tid == 0) a.part0[blockIdx.x] = t0;
        if (EPI == EPI_RESID_PREC || (EPI == EPI_PREC && a.v0 != nullptr)) {
            const double t1 = block_sum(acc1, red);
            if (tid == 0) a.part1[blockIdx.x] = t1;
        }
    }
}

// SELL-64 build: chunk q's width = its longest row; offsets = exclusive scan of 64*width
__global__ __launch_bounds__(NT) void k_sell_width(const int32_t *__restrict__ indptr, int64_t n, int64_t nch,
                                                   int64_t *__restrict__ w64) {
    for (int64_t q = (int64_t)blockIdx.x * NT + threadIdx.x; q <= nch; q += (int64_t)gridDim.x * NT) {
        int w = 0;
        if (q < nch) {
            const int64_t r1 = q * 64 + 64 < n ? q * 64 + 64 : n;
            for (int64_t r = q * 64; r < r1; ++r) w = max(w, indptr[r + 1] - indptr[r]);
        }
        w64[q] = 64 * (int64_t)w;   // w64[nch] = 0: the scan's last entry is the total
    }
}

template <typename VT>
__global__ __launch_bounds__(NT) void k_sell_fill(const int32_t *__restrict__ indptr, const int32_t *__restrict__ indices,
                                                  const VT *__restrict__ data, int64_t n, int64_t nch,
                                                  const int64_t *__restrict__ off, int32_t *__restrict__ col,
                                                  VT *__restrict__ val) {
    for (int64_t r = (int64_t)blockIdx.x * NT + threadIdx.x; r < nch * 64; r += (int64_t)gridDim.x * NT) {
        const int64_t q = r >> 6, l = r & 63;
        const int w = (int)((off[q + 1] - off[q]) >> 6);
        const int k0 = r < n ? indptr[r] : 0, len = r < n ? indptr[r + 1] - k0 : 0;
        int32_t *cc = col + off[q] + l;
        VT *vv = val + off[q] + l;
        for (int k = 0; k < w; ++k) {
            cc[(int64_t)k * 64] = k < len ? indices[k0 + k] : -1;
            vv[(int64_t)k * 64] = k < len ? data[k0 + k] : (VT)0;
        }
    }
}

hipError_t launch_sell_build(const int32_t *indptr, const int32_t *indices, const void *data, int fp32, int64_t n,
                             int64_t *off, int64_t *tmp64, void *scan_tmp, size_t scan_bytes, int32_t *col,
                             void *val, int phase, hipStream_t s) {
    const int64_t nch = (n + 63) / 64;
    if (phase == 0) {   // widths + scan -> off[0..nch]
        hipLaunchKernelGGL(k_sell_width, dim3(1024), dim3(NT), 0, s, indptr, n, nch, tmp64);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        return hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, tmp64, off, (int)(nch + 1), s);
    }
    if (fp32) hipLaunchKernelGGL(k_sell_fill<float>, dim3(4096), dim3(NT), 0, s, indptr, indices, (const float *)data, n, nch, off, col, (float *)val);
    else hipLaunchKernelGGL(k_sell_fill<double>, dim3(4096), dim3(NT), 0, s, indptr, indices, (const double *)data, n, nch, off, col, (double *)val);
    return hipGetLastError();
}

// Dictionary coding of a SELL chunk's columns: one wavefront per chunk collects the distinct
// offsets (col - row) of its entries in first-seen order (entry-major, lane-minor) into a
// dictionary of at most PK_CODES, held by lanes 0..14; each entry becomes a 4-bit code, eight
// per 32-bit word.  A chunk with more offsets keeps its int32 columns (dict[16q+15] = 1).
// Stencil operators have a handful of offsets per chunk: the 2D Vlasov operator 5 (+2 at the
// periodic x wrap), 4D 9 (+ wraps) -- 4 B of columns per entry become 0.5 B + 1 B per row.
__global__ __launch_bounds__(NT) void k_pk_width(const int64_t *__restrict__ off, int64_t nch, int64_t *__restrict__ w64) {
    for (int64_t q = (int64_t)blockIdx.x * NT + threadIdx.x; q <= nch; q += (int64_t)gridDim.x * NT) {
        const int64_t w = q < nch ? (off[q + 1] - off[q]) >> 6 : 0;
        w64[q] = 64 * ((w + 7) / 8);
    }
}

__global__ __launch_bounds__(NT) void k_sell_pack(const int64_t *__restrict__ off, const int64_t *__restrict__ pkoff,
                                                  const int32_t *__restrict__ col, int64_t nch,
                                                  uint32_t *__restrict__ pk, int32_t *__restrict__ dict,
                                                  unsigned long long *wide_cnt) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = ((int64_t)gridDim.x * NT) >> 6;
    for (int64_t q = ((int64_t)blockIdx.x * NT + threadIdx.x) >> 6; q < nch; q += nw) {
        const int64_t o0 = off[q];
        const int w = (int)((off[q + 1] - o0) >> 6);
        const int64_t row = q * 64 + lane;
        uint32_t *pw = pk + pkoff[q] + lane;
        int dl = 0, nd = 0;   // lane d < nd holds dictionary entry d
        bool wide = false;    // wave-uniform
        uint32_t word = 0xFFFFFFFFu;
        for (int k = 0; k < w && !wide; ++k) {
            const int32_t c = col[o0 + 64 * (int64_t)k + lane];
            const bool valid = c >= 0;
            const int o = valid ? (int)(c - row) : 0;   // both in [0, 2^31): fits
            int code = PK_CODES;
            for (int d = 0; d < nd; ++d) {
                const int dv = __shfl(dl, d, 64);
                if (valid && code == PK_CODES && dv == o) code = d;
            }
            for (;;) {
                const unsigned long long pend = __ballot(valid && code == PK_CODES);
                if (pend == 0) break;
                if (nd == PK_CODES) { wide = true; break; }
                const int v = __shfl(o, __ffsll((long long)pend) - 1, 64);
                if (lane == nd) dl = v;
                if (valid && code == PK_CODES && o == v) code = nd;
                ++nd;
            }
            const int sh = 4 * (k & 7);
            word = (word & ~(15u << sh)) | ((uint32_t)code << sh);
            if ((k & 7) == 7 || k == w - 1) {
                pw[(int64_t)(k >> 3) * 64] = word;
                word = 0xFFFFFFFFu;
            }
        }
        if (lane < 16) dict[q * 16 + lane] = lane < nd ? dl : (lane == 15 && wide ? 1 : 0);
        if (lane == 0 && wide) {
            atomicAdd(wide_cnt, 1ull);
            atomicAdd(wide_cnt + 1, 64ull * (unsigned long long)w);
        }
    }
}

hipError_t launch_sell_pack(const int64_t *off, int64_t nch, int64_t *pkoff, int64_t *tmp64, void *scan_tmp,
                            size_t scan_bytes, const int32_t *col, uint32_t *pk, int32_t *dict,
                            unsigned long long *wide_cnt, int phase, hipStream_t s) {
    if (phase == 0) {
        hipLaunchKernelGGL(k_pk_width, dim3(1024), dim3(NT), 0, s, off, nch, tmp64);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        return hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, tmp64, pkoff, (int)(nch + 1), s);
    }
    hipLaunchKernelGGL(k_sell_pack, dim3(4096), dim3(NT), 0, s, off, pkoff, col, nch, pk, dict, wide_cnt);
    return hipGetLastError();
}

size_t sell_scan_bytes(int64_t n) {
    const int64_t nch = (n + 63) / 64;
    size_t bytes = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (int64_t *)nullptr, (int64_t *)nullptr, (int)(nch + 1));
    return bytes;
}

// BJ variants: bs 0 (identity), 1..32 inverse rows, 2/4/8 tridiagonal factors; MAXBS bounds
// the instantiations (the DCGS2-fused kernel stops at 8: larger blocks spill).  SELL: the
// SELL-64 kernel, else the CSR-stream tiles.
#define VTK_SPMV_LAUNCH(EPI_, BS_, TRI_)                                                        \
    do {                                                                                        \
        if (sell) hipLaunchKernelGGL((k_sell<VT, HALO, EPI_, BS_, TRI_>), g, blk, 0, s, a);     \
        else hipLaunchKernelGGL((k_spmv<VT, HALO, EPI_, BS_, TRI_>), g, blk, 0, s, a);          \
    } while (0)

// workgroups of the plain SELL SpMV (no partials: free of GMAX); vtk::Tuning::plain_grid
static inline int plain_grid(const SpmvIn &in) { return in.plain_grid > 0 ? in.plain_grid : 2 * GMAX; }
static inline int sell_wu(const SpmvIn &in) {
    if (!in.sell || !in.groups) return 0;
    const int w = in.sell->uniform_w;
    return (w == 5 || w == 9) ? w : 0;
}
// the plain SpMV takes the compile-time path only for rows wider than one code word (C4 plain
// 848 -> 698 us); at width 5 the runtime loop is faster (C3 220 vs 233 us)
static inline int sell_wu_plain(const SpmvIn &in) {
    const int w = sell_wu(in);
    return w > 8 ? w : 0;
}

template <typename VT, bool HALO, int EPI, int MAXBS>
static hipError_t launch_bj_variant(const SpmvK<VT, HALO> &a, int bs, bool tri, bool sell, dim3 g, hipStream_t s) {
    const dim3 blk(NT);
    if (tri) {
        // 9-wide uniform rows (C4): the compile-time-width path (the cycle-start residual
        // kernel, 1440 us with the runtime loop)
        if (EPI != EPI_PREC_DC && sell && bs == 8 && a.sell_uw == 9) {
            if (a.g4.tab) hipLaunchKernelGGL((k_sell<VT, HALO, EPI, 8, true, 0, 9, 2>), g, blk, 0, s, a);
            else hipLaunchKernelGGL((k_sell<VT, HALO, EPI, 8, true, 0, 9>), g, blk, 0, s, a);
            return hipGetLastError();
        }
        switch (bs) {
            case 2: VTK_SPMV_LAUNCH(EPI, 2, true); break;
            case 4: VTK_SPMV_LAUNCH(EPI, 4, true); break;
            case 8: VTK_SPMV_LAUNCH(EPI, 8, true); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    switch (bs) {
        case 0: VTK_SPMV_LAUNCH(EPI, 0, false); break;
        case 1: VTK_SPMV_LAUNCH(EPI, 1, false); break;
        case 2: VTK_SPMV_LAUNCH(EPI, 2, false); break;
        case 4: VTK_SPMV_LAUNCH(EPI, 4, false); break;
        case 8: VTK_SPMV_LAUNCH(EPI, 8, false); break;
        case 16:
            if constexpr (MAXBS >= 16) { VTK_SPMV_LAUNCH(EPI, 16, false); break; }
            return hipErrorInvalidValue;
        case 32:
            if constexpr (MAXBS >= 32) { VTK_SPMV_LAUNCH(EPI, 32, false); break; }
            return hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <typename VT, bool HALO>
static SpmvK<VT, HALO> spmv_args(const SpmvIn &in, double *y, const double *b, const BjOp &bj, const double *v0,
                                 double *part0, double *part1, const int *stop_col, int col) {
    const bool sell = in.sell && in.groups;
    SpmvK<VT, HALO> a{in.indptr, in.indices, static_cast<const VT *>(in.data),
                      in.tiles ? in.tiles->d_row : nullptr, in.tiles ? in.tiles->d_end : nullptr,
                      in.tiles ? in.tiles->ntiles : 0, in.n_local, in.x, in.halo,
                      y, b, bj.inv, v0, part0, part1, stop_col, col, bj.tri, bj.tri_ld, nullptr, 0, 0, nullptr,
                      sell ? in.sell->d_off : nullptr, sell ? in.sell->d_col : nullptr,
                      sell ? static_cast<const VT *>(in.sell->d_val) : nullptr,
                      sell ? in.groups->d_list : nullptr, sell ? in.groups->count : 0,
                      sell ? in.sell->d_pk : nullptr, sell ? in.sell->d_pkoff : nullptr,
                      sell ? in.sell->d_dict : nullptr, sell ? in.sell->uniform_w : 0,
                      sell && !std::is_same<VT, float>::value ? in.lsv : nullptr, in.lsv_L, in.lsv_lblk, in.lsv_xord,
                      sell && !std::is_same<VT, float>::value && in.lsv ? in.lsv_canon : 0, in.swz,
                      sell ? in.g4 : Grid4{}};
    return a;
}

template <typename VT, bool HALO>
static hipError_t spmv_dispatch(const SpmvIn &in, int epi, double *y, const double *b, const BjOp &bj,
                                const double *v0, double *part0, double *part1, const int *stop_col, int col,
                                hipStream_t s) {
    SpmvK<VT, HALO> a = spmv_args<VT, HALO>(in, y, b, bj, v0, part0, part1, stop_col, col);
    a.swz = (in.swz >> (epi == EPI_PLAIN ? 0 : 1)) & 1;   // Tuning::sell_swz
    const bool sell = in.sell && in.groups;
    const dim3 g(spmv_grid(in)), blk(NT);
    const int bs = (bj.inv || bj.tri) ? bj.bs : 0;
    const bool tri = bj.tri != nullptr;
    if (epi == EPI_PLAIN) {
        // no partials: SELL fills the chip at its 8 waves/SIMD (52 VGPRs) with 2048 workgroups
        // (tools/probe_sell.hip, C4: 965 us at 2048 vs 1362 us at 1024; C3 within 2 %)
        const dim3 gp(sell ? (unsigned)std::max(1, std::min(in.groups->count, plain_grid(in))) : g.x);
        const int wu = sell_wu_plain(in);
        if (sell && wu == 9) hipLaunchKernelGGL((k_sell<VT, HALO, EPI_PLAIN, 1, false, 0, 9>), gp, blk, 0, s, a);
        else if (sell && (in.plain_var & 1)) hipLaunchKernelGGL((k_sell<VT, HALO, EPI_PLAIN, 1, false, 0, 0, 1>), gp, blk, 0, s, a);
        else if (sell) hipLaunchKernelGGL((k_sell<VT, HALO, EPI_PLAIN, 1, false>), gp, blk, 0, s, a);
        else hipLaunchKernelGGL((k_spmv<VT, HALO, EPI_PLAIN, 1, false>), g, blk, 0, s, a);
        return hipGetLastError();
    }
    if (epi == EPI_RESID) {
        VTK_SPMV_LAUNCH(EPI_RESID, 1, false);
        return hipGetLastError();
    }
    if (epi == EPI_PREC) return launch_bj_variant<VT, HALO, EPI_PREC, 32>(a, bs, tri, sell, g, s);
    return launch_bj_variant<VT, HALO, EPI_RESID_PREC, 32>(a, bs, tri, sell, g, s);
}

template <typename VT, bool HALO>
static hipError_t spmv_dc_dispatch(const SpmvIn &in, double *w, const BjOp &bj, const double *V, int64_t ld,
                                   int j, double *part, const int *stop_col, int col, hipStream_t s) {
    SpmvK<VT, HALO> a = spmv_args<VT, HALO>(in, w, nullptr, bj, nullptr, nullptr, nullptr, stop_col, col);
    a.swz = (in.swz >> 1) & 1;   // Tuning::sell_swz bit 1 (the partials follow the group order)
    a.V = V;
    a.ld = ld;
    a.j = j;
    a.dcpart = part;
    // BJ-fused tiles only (bs 1..8); the host falls back to the unfused dots otherwise
    const int bs = (bj.inv || bj.tri) ? bj.bs : 0;
    if (bs == 0) return hipErrorInvalidValue;
    // SELL chunks of <= 5 entries per row on average (the 2D operators: 5-point rows): one load
    // batch of 5 covers a row (C3 fused step 621 -> 590 us); wider rows keep batches of 4 (C4:
    // 5 would cost +5 %)
    const bool sell = in.sell && in.groups;
    const int wu = sell_wu(in);
    if (sell && bj.tri && bs == 8 && wu == 5) {
        hipLaunchKernelGGL((k_sell<VT, HALO, EPI_PREC_DC, 8, true, 5, 5>), dim3(spmv_grid(in)), dim3(NT), 0, s, a);
        return hipGetLastError();
    }
    if (sell && bj.tri && bs == 8 && wu == 9) {
        if (a.g4.tab) hipLaunchKernelGGL((k_sell<VT, HALO, EPI_PREC_DC, 8, true, DC_PSW9, 9, 2>), dim3(spmv_grid(in)), dim3(NT), 0, s, a);
        else hipLaunchKernelGGL((k_sell<VT, HALO, EPI_PREC_DC, 8, true, DC_PSW9, 9>), dim3(spmv_grid(in)), dim3(NT), 0, s, a);
        return hipGetLastError();
    }
    if (sell && bj.tri && bs == 8 && in.sell->nch > 0 && in.sell->entries <= in.sell->nch * 64 * 5) {
        hipLaunchKernelGGL((k_sell<VT, HALO, EPI_PREC_DC, 8, true, 5>), dim3(spmv_grid(in)), dim3(NT), 0, s, a);
        return hipGetLastError();
    }
    return launch_bj_variant<VT, HALO, EPI_PREC_DC, 8>(a, bs, bj.tri != nullptr, sell, dim3(spmv_grid(in)), s);
}

hipError_t launch_spmv_dc(const SpmvIn &in, double *w, const BjOp &bj, const double *V,
                          int64_t ld, int j, double *part, const int *stop_col, int col, hipStream_t s) {
    if (j > DC_MAXJ || spmv_grid(in) > GMAX) return hipErrorInvalidValue;
    const bool halo = in.halo != nullptr;
    if (in.fp32) {
        return halo ? spmv_dc_dispatch<float, true>(in, w, bj, V, ld, j, part, stop_col, col, s)
                    : spmv_dc_dispatch<float, false>(in, w, bj, V, ld, j, part, stop_col, col, s);
    }
    return halo ? spmv_dc_dispatch<double, true>(in, w, bj, V, ld, j, part, stop_col, col, s)
                : spmv_dc_dispatch<double, false>(in, w, bj, V, ld, j, part, stop_col, col, s);
}

hipError_t launch_spmv(const SpmvIn &in, int epi, double *y, const double *b, const BjOp &bj,
                       const double *v0, double *part0, double *part1,
                       const int *stop_col, int col, hipStream_t s) {
    // ntiles == 0 still launches: reducing epilogues must write their (zero) partials
    const bool halo = in.halo != nullptr;
    if (in.fp32) {
        return halo ? spmv_dispatch<float, true>(in, epi, y, b, bj, v0, part0, part1, stop_col, col, s)
                    : spmv_dispatch<float, false>(in, epi, y, b, bj, v0, part0, part1, stop_col, col, s);
    }
    return halo ? spmv_dispatch<double, true>(in, epi, y, b, bj, v0, part0, part1, stop_col, col, s)
                : spmv_dispatch<double, false>(in, epi, y, b, bj, v0, part0, part1, stop_col, col, s);
}

// ------------------------------------------------------------------------------------------
// block-Jacobi apply (standalone): one lane per row, serial j order.  inv == null: identity.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void k_bj_apply(const double *__restrict__ inv, int bs, int64_t n,
                                                 const double *__restrict__ r, double *__restrict__ z,
                                                 const double *__restrict__ v0, double *part0,
                                                 double *part1, const int *stop_col, int col) {
    __shared__ double red[NT / 64];
    if (stopped(stop_col, col)) return;
    double acc0 = 0.0, acc1 = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
        double v;
        if (inv == nullptr) {
            v = r[i];
        } else {
            const int64_t blk = i / bs;
            const double *irow = inv + (size_t)i * bs;
            const int64_t c0 = blk * bs;
            v = 0.0;
            for (int j = 0; j < bs; ++j) {
                const double rv = (c0 + j) < n ? r[c0 + j] : 0.0;
                v += irow[j] * rv;
            }
        }
        z[i] = v;
        acc0 += v * v;
        if (v0) acc1 += v0[i] * v;
    }
    if (part0) {
        const double t0 = block_sum(acc0, red);
        if (threadIdx.x == 0) part0[blockIdx.x] = t0;
    }
    if (part1 && v0) {
        const double t1 = block_sum(acc1, red);
        if (threadIdx.x == 0) part1[blockIdx.x] = t1;
    }
}

// tridiagonal-factor variant: the loop bound is workgroup-uniform so every lane of a block's
// group takes part in the scans
template <int BS>
__global__ __launch_bounds__(NT) void k_bj_apply_tri(const double *__restrict__ tri, int64_t ld, int64_t n,
                                                     const double *__restrict__ r, double *__restrict__ z,
                                                     const double *__restrict__ v0, double *part0,
                                                     double *part1, const int *stop_col, int col) {
    __shared__ double red[NT / 64];
    if (stopped(stop_col, col)) return;
    const int lane = threadIdx.x & 63;
    double acc0 = 0.0, acc1 = 0.0;
    for (int64_t i0 = (int64_t)blockIdx.x * NT; i0 < n; i0 += (int64_t)gridDim.x * NT) {
        const int64_t i = i0 + threadIdx.x;
        const bool act = i < n;
        const double v = bj_tri_group<BS>(act ? r[i] : 0.0, act, i, lane, tri, ld);
        if (act) {
            z[i] = v;
            acc0 += v * v;
            if (v0) acc1 += v0[i] * v;
        }
    }
    if (part0) {
        const double t0 = block_sum(acc0, red);
        if (threadIdx.x == 0) part0[blockIdx.x] = t0;
    }
    if (part1 && v0) {
        const double t1 = block_sum(acc1, red);
        if (threadIdx.x == 0) part1[blockIdx.x] = t1;
    }
}

hipError_t launch_bj_apply(const BjOp &bj, int64_t n, const double *r, double *z,
                           const double *v0, double *part0, double *part1, int grid,
                           const int *stop_col, int col, hipStream_t s) {
    if (bj.line) return launch_line_apply(*bj.line, r, z, v0, part0, part1, grid, stop_col, col, s);
    if (n == 0 && part0 == nullptr) return hipSuccess;
    if (bj.tri) {
        switch (bj.bs) {
            case 2: hipLaunchKernelGGL(k_bj_apply_tri<2>, dim3(grid), dim3(NT), 0, s, bj.tri, bj.tri_ld, n, r, z, v0, part0, part1, stop_col, col); break;
            case 4: hipLaunchKernelGGL(k_bj_apply_tri<4>, dim3(grid), dim3(NT), 0, s, bj.tri, bj.tri_ld, n, r, z, v0, part0, part1, stop_col, col); break;
            case 8: hipLaunchKernelGGL(k_bj_apply_tri<8>, dim3(grid), dim3(NT), 0, s, bj.tri, bj.tri_ld, n, r, z, v0, part0, part1, stop_col, col); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_bj_apply, dim3(grid), dim3(NT), 0, s, bj.bs > 0 ? bj.inv : nullptr, bj.bs > 0 ? bj.bs : 1,
                       n, r, z, v0, part0, part1, stop_col, col);
    return hipGetLastError();
}

// Tridiagonal factors of the diagonal blocks, one thread per block (setup, once).  Duplicates
// add up (toarray semantics); columns outside [0, n) (halo) are not block entries.  Thomas
// without pivoting: u_0 = d_0, l_i = a_i / u_{i-1}, u_i = d_i - l_i c_{i-1}; the factors are
// then checked column by column against the Gauss-Jordan inverse of the same block.
template <typename VT>
__global__ __launch_bounds__(NT) void k_bj_tri_setup(const int32_t *__restrict__ indptr,
                                                     const int32_t *__restrict__ indices,
                                                     const VT *__restrict__ data, int64_t n, int64_t nb, int bs,
                                                     const double *__restrict__ inv, double *__restrict__ tri,
                                                     int64_t ld, int *flags) {
    constexpr int MB = 8;
    const int64_t blk = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (blk >= nb || bs > MB) return;
    double sub[MB], dia[MB], sup[MB], l[MB], m[MB], g[MB];
    int bad = 0;
    const int64_t c0 = blk * bs;
    for (int i = 0; i < bs; ++i) {
        const int64_t row = c0 + i;
        sub[i] = 0.0;
        sup[i] = 0.0;
        dia[i] = row >= n ? 1.0 : 0.0;
        if (row >= n) continue;
        for (int k = indptr[row]; k < indptr[row + 1]; ++k) {
            const int64_t col = indices[k];
            if (col >= n) continue;
            const int64_t c = col - c0;
            if (c < 0 || c >= bs) continue;
            const double v = (double)data[k];
            if (c == i) dia[i] = dia[i] + v;
            else if (c == i - 1) sub[i] = sub[i] + v;
            else if (c == i + 1) sup[i] = sup[i] + v;
            else bad |= 1;
        }
    }
    double u = dia[0];
    l[0] = 0.0;
    for (int i = 0; i < bs; ++i) {
        if (i > 0) {
            l[i] = sub[i] / u;
            u = dia[i] - l[i] * sup[i - 1];
        }
        const double scale = __builtin_fabs(sub[i]) + __builtin_fabs(dia[i]) + __builtin_fabs(sup[i]);
        if (!(__builtin_fabs(u) > 1e-12 * scale)) bad |= 2;
        m[i] = 1.0 / u;
        g[i] = sup[i] * m[i];
    }
    if (!bad && inv) {
        double err = 0.0, mag = 0.0;
        for (int k = 0; k < bs; ++k) {
            double d[MB];
            for (int i = 0; i < bs; ++i) d[i] = (i == k ? 1.0 : 0.0) - (i > 0 ? l[i] * d[i - 1] : 0.0);
            double zn = 0.0;
            for (int i = bs - 1; i >= 0; --i) {
                zn = m[i] * d[i] - (i + 1 < bs ? g[i] * zn : 0.0);
                const double ref = inv[(size_t)(c0 + i) * bs + k];
                err = fmax(err, __builtin_fabs(zn - ref));
                mag = fmax(mag, __builtin_fabs(ref));
            }
        }
        if (!(err <= 1e-10 * mag)) bad |= 4;
    }
    for (int i = 0; i < bs; ++i) {
        tri[c0 + i] = l[i];
        tri[ld + c0 + i] = m[i];
        tri[2 * ld + c0 + i] = g[i];
    }
    if (bad) atomicOr(flags, bad);
}

hipError_t launch_bj_tri_setup(const int32_t *indptr, const int32_t *indices, const void *data, int fp32,
                               int64_t n, int bs, const double *inv, double *tri, int64_t ld, int *flags,
                               hipStream_t s) {
    const int64_t nb = (n + bs - 1) / bs;
    if (nb == 0) return hipSuccess;
    const dim3 g((unsigned)((nb + NT - 1) / NT));
    if (fp32) hipLaunchKernelGGL(k_bj_tri_setup<float>, g, dim3(NT), 0, s, indptr, indices, (const float *)data, n, nb, bs, inv, tri, ld, flags);
    else hipLaunchKernelGGL(k_bj_tri_setup<double>, g, dim3(NT), 0, s, indptr, indices, (const double *)data, n, nb, bs, inv, tri, ld, flags);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// line Jacobi: tridiagonal systems along x-line segments.  One lane per
// (segment, j); the 64 lanes of a wavefront take consecutive j, so every sweep step over the
// line index i (row R = i*stride + j) is one coalesced 512-B access per array.  The IEEE
// operations per row are those of orc_line_setup / orc_line_apply (bit-identical).
// ------------------------------------------------------------------------------------------
LineOp line_plan(int64_t n, int64_t row0, int64_t stride, int64_t seg) {
    LineOp L;
    L.n = n;
    L.row0 = row0;
    L.stride = stride;
    L.seg = seg;
    if (n <= 0 || stride <= 0 || seg <= 0) return L;
    L.i_lo = row0 / stride;
    L.i_hi = (row0 + n - 1) / stride;
    L.nseg = L.i_hi / seg - L.i_lo / seg + 1;
    if (L.i_lo == L.i_hi) {
        L.j0 = row0 % stride;
        L.jn = n;
    } else {
        L.j0 = 0;
        L.jn = stride;
    }
    L.jb = (L.jn + 63) / 64;
    return L;
}

// wavefront item t -> the segment's line range [i_beg, i_end) and this lane's j (jv: in range)
struct LineLane {
    int64_t i_beg, i_end, j;
    bool jv;
};
__device__ __forceinline__ LineLane line_lane(const LineOp &L, int64_t t, int lane) {
    const int64_t k = t / L.jb, jw = t - k * L.jb;
    const int64_t s = L.i_lo / L.seg + k;
    LineLane o;
    o.i_beg = s * L.seg > L.i_lo ? s * L.seg : L.i_lo;
    o.i_end = (s + 1) * L.seg < L.i_hi + 1 ? (s + 1) * L.seg : L.i_hi + 1;
    const int64_t jj = jw * 64 + lane;
    o.jv = jj < L.jn;
    o.j = L.j0 + jj;
    return o;
}

// Thomas factors along the lane's line segment: u = b | l = a m_prev, u = b - l c_prev;
// m = 1 / u; g = c m.  A row's "previous" is the lane's previous valid row (rows of one (j,
// segment) inside the block are contiguous in i), exactly the oracle's line_has(R, -1).
// ext (4 jn words, lane j - j0): min / max bit pattern of the a's and of the c's the lane's
// segment holds; equal min and max for every line = the x-couplings are constant along every
// line (x-invariant advection, the Vlasov operators), and the apply can form l and g from
// them instead of reading them (LineOp::compact).
template <typename VT>
__global__ __launch_bounds__(NT) void k_line_setup(const int32_t *__restrict__ indptr,
                                                   const int32_t *__restrict__ indices,
                                                   const VT *__restrict__ data, LineOp L,
                                                   unsigned long long *bad_row, unsigned long long *ext) {
    const int lane = threadIdx.x & 63;
    const int64_t t = ((int64_t)blockIdx.x * NT + threadIdx.x) >> 6;
    if (t >= L.nseg * L.jb) return;
    const LineLane q = line_lane(L, t, lane);
    if (!q.jv) return;
    const int64_t S = L.stride, r_end = L.row0 + L.n;
    double *l = L.f, *m = L.f + L.n, *g = L.f + 2 * L.n;
    double mp = 0.0, cp = 0.0;
    bool have = false;
    unsigned long long amin = ~0ull, amax = 0, cmin = ~0ull, cmax = 0;
    for (int64_t i = q.i_beg; i < q.i_end; ++i) {
        const int64_t R = i * S + q.j;
        if (R < L.row0 || R >= r_end) continue;
        const int64_t r = R - L.row0;
        const bool hl = have, hr = i + 1 < q.i_end && R + S < r_end;
        double b = 0.0, a = 0.0, c = 0.0;
        for (int32_t k = indptr[r]; k < indptr[r + 1]; ++k) {
            const int64_t col = indices[k];
            const double v = (double)data[k];
            if (col == r) b += v;
            else if (hl && col == r - S) a += v;
            else if (hr && col == r + S) c += v;
        }
        double lv = 0.0, uv;
        if (hl) {
            lv = a * mp;
            uv = b - lv * cp;
        } else {
            uv = b;
        }
        const double mv = 1.0 / uv;
        if (uv == 0.0 || !isfinite(uv) || !isfinite(mv)) atomicMin(bad_row, (unsigned long long)R);
        l[r] = lv;
        m[r] = mv;
        g[r] = c * mv;
        mp = mv;
        cp = c;
        have = true;
        if (hl) {
            const unsigned long long ab = (unsigned long long)__double_as_longlong(a);
            amin = ab < amin ? ab : amin;
            amax = ab > amax ? ab : amax;
        }
        if (hr) {
            const unsigned long long cb = (unsigned long long)__double_as_longlong(c);
            cmin = cb < cmin ? cb : cmin;
            cmax = cb > cmax ? cb : cmax;
        }
    }
    const int64_t jl = q.j - L.j0;
    if (amin <= amax) {
        atomicMin(ext + jl, amin);
        atomicMax(ext + L.jn + jl, amax);
    }
    if (cmin <= cmax) {
        atomicMin(ext + 2 * L.jn + jl, cmin);
        atomicMax(ext + 3 * L.jn + jl, cmax);
    }
}

// z = M^-1 r: forward d = r - l d_prev, backward z = m d - g z_next.  LMAX > 0: the forward
// sweep keeps e = m d and g in registers and every load of the sweep is issued before its
// recurrence (addresses clamped to row 0 off the block, results discarded); the backward
// sweep only stores.  COMPACT: l = a m_prev and g = c m from the line's constant couplings
// (L.ac) - 16 B/row read instead of 32; the same IEEE operations as the stored factors.
// LMAX == 0 (segments longer than 32): d goes through z.  r and z may alias (each row is read
// before it is written, by its lane).
// DCD (DCGS2 step j, line path): the step's dots fused behind the sweep -- w = z stays in the
// lane's registers, p and the basis rows of the lane's segment rows are read once here:
// s = V_j^T p, z = V_j^T w, ||p||^2, p.w, ||w||^2 as per-workgroup partials in launch_dc_dots'
// layout (dc.part[q * GMAX + block]); no separate dots kernel re-reads w.
struct LineDc {
    const double *V;
    int64_t ld;
    int j;
    const double *p;
    double *part;
};
template <int LMAX, bool COMPACT, bool DCD = false>
__global__ __launch_bounds__(NT) void k_line_apply(LineOp L, const double *r, double *z,
                                                   const double *__restrict__ v0, double *part0,
                                                   double *part1, const int *stop_col, int col,
                                                   LineDc dc = LineDc{}) {
    __shared__ double red[NT / 64];
    constexpr int NQW = 2 * DC_MAXJ + 3;
    __shared__ double stage[DCD ? (NT / 64) * NQW : 1];
    if (stopped(stop_col, col)) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t nitems = L.nseg * L.jb, S = L.stride, r0 = L.row0, r_end = L.row0 + L.n;
    const double *l = L.f, *m = L.f + L.n, *g = L.f + 2 * L.n;
    double acc0 = 0.0, acc1 = 0.0;
    [[maybe_unused]] double dsl = 0.0, dzl = 0.0, daa = 0.0, dab = 0.0, dag = 0.0;   // DCD
    for (int64_t t = (int64_t)blockIdx.x * (NT / 64) + wv; t < nitems; t += (int64_t)gridDim.x * (NT / 64)) {
        const LineLane q = line_lane(L, t, lane);
        const int64_t len = q.i_end - q.i_beg;
        if constexpr (LMAX > 0) {
            // row offsets k_u = k0 + u*S fit 32 bits (n_local < 2^31): 32-bit address math
            const int64_t k0l = q.i_beg * S + q.j - r0;
            const int nn = (int)L.n;
            double aj = 0.0, cj = 0.0;
            if constexpr (COMPACT) {
                if (q.jv) {
                    aj = L.ac[q.j - L.j0];
                    cj = L.ac[L.jn + q.j - L.j0];
                }
            }
            double e[LMAX], gg[LMAX];
            double dp = 0.0, mp = 0.0;
            bool pok = false;
            unsigned okm = 0;
#pragma unroll
            for (int u = 0; u < LMAX; ++u) {
                const int64_t kl = k0l + (int64_t)u * S;
                const bool ok = q.jv && u < len && kl >= 0 && kl < nn;
                const int k = ok ? (int)kl : 0;
                const double mv = ld_nt<8>(m + k);
                double lv, gv;
                if constexpr (COMPACT) {
                    const bool hl = ok && pok;
                    const bool hr = ok && u + 1 < len && kl + S < nn;
                    lv = hl ? aj * mp : 0.0;
                    gv = (hr ? cj : 0.0) * mv;
                } else {
                    lv = l[k];
                    gv = g[k];
                }
                const double dv = ld_nt<8>(r + k) - lv * dp;
                e[u] = mv * dv;
                gg[u] = gv;
                if (ok) {
                    dp = dv;
                    mp = mv;
                }
                pok = ok;
                okm |= (unsigned)ok << u;
            }
            double zn = 0.0;
#pragma unroll
            for (int u = LMAX - 1; u >= 0; --u) {
                const double zv = e[u] - gg[u] * zn;
                if ((okm >> u) & 1u) {
                    const int k = (int)(k0l + (int64_t)u * S);
                    st_nt<4>(z + k, zv);
                    zn = zv;
                    if constexpr (!DCD) {
                        acc0 += zv * zv;
                        if (v0) acc1 += v0[k] * zv;
                    }
                }
                if constexpr (DCD) e[u] = ((okm >> u) & 1u) ? zv : 0.0;   // w, kept for the dots
            }
            if constexpr (DCD) {
                // p on the lane's rows (gg is free after the sweep), then the basis vector by
                // vector: all of the lane's rows of V_k in flight at once, summed in the lane and
                // across the wave by the butterfly; lane k keeps the running sums of vector k
#pragma unroll
                for (int u = 0; u < LMAX; ++u) {
                    const int k = (int)(k0l + (int64_t)u * S);
                    gg[u] = ((okm >> u) & 1u) ? ld_nt<4>(dc.p + k) : 0.0;
                }
#pragma unroll
                for (int u = 0; u < LMAX; ++u) {
                    daa += gg[u] * gg[u];
                    dab += gg[u] * e[u];
                    dag += e[u] * e[u];
                }
                for (int kk = 0; kk < dc.j; ++kk) {
                    const double *vk = dc.V + (size_t)kk * dc.ld;
                    double sl = 0.0, zl = 0.0;
#pragma unroll
                    for (int u = 0; u < LMAX; ++u) {
                        const int k = (int)(k0l + (int64_t)u * S);
                        const double v = ((okm >> u) & 1u) ? __builtin_nontemporal_load(vk + k) : 0.0;
                        sl += v * gg[u];
                        zl += v * e[u];
                    }
                    const double ts = wave_allsum(sl), tz = wave_allsum(zl);
                    if (lane == kk) {
                        dsl += ts;
                        dzl += tz;
                    }
                }
            }
        } else {
            double dp = 0.0;
            for (int64_t u = 0; u < len; ++u) {
                const int64_t R = (q.i_beg + u) * S + q.j;
                if (!q.jv || R < r0 || R >= r_end) continue;
                const int64_t k = R - r0;
                const double dv = r[k] - l[k] * dp;
                z[k] = dv;
                dp = dv;
            }
            double zn = 0.0;
            for (int64_t u = len - 1; u >= 0; --u) {
                const int64_t R = (q.i_beg + u) * S + q.j;
                if (!q.jv || R < r0 || R >= r_end) continue;
                const int64_t k = R - r0;
                const double zv = m[k] * z[k] - g[k] * zn;
                z[k] = zv;
                zn = zv;
                acc0 += zv * zv;
                if (v0) acc1 += v0[k] * zv;
            }
        }
    }
    if constexpr (DCD) {
        // per-workgroup partials: the 4 waves' records summed in wave order
        double *rec = stage + wv * NQW;
        if (lane < dc.j) {
            rec[lane] = dsl;
            rec[DC_MAXJ + lane] = dzl;
        }
        const double t0 = wave_sum(daa), t1 = wave_sum(dab), t2 = wave_sum(dag);
        if (lane == 0) {
            rec[2 * DC_MAXJ] = t0;
            rec[2 * DC_MAXJ + 1] = t1;
            rec[2 * DC_MAXJ + 2] = t2;
        }
        __syncthreads();
        for (int qq = threadIdx.x; qq < DC_NQ; qq += NT) {
            const bool used = qq < dc.j || (qq >= DC_MAXJ && qq < DC_MAXJ + dc.j) || qq >= 2 * DC_MAXJ;
            if (used) {
                double t = 0.0;
#pragma unroll
                for (int w2 = 0; w2 < NT / 64; ++w2) t += stage[w2 * NQW + qq];
                dc.part[(size_t)qq * GMAX + blockIdx.x] = t;
            }
        }
        return;
    }
    if (part0) {
        const double t0 = block_sum(acc0, red);
        if (threadIdx.x == 0) part0[blockIdx.x] = t0;
    }
    if (part1 && v0) {
        const double t1 = block_sum(acc1, red);
        if (threadIdx.x == 0) part1[blockIdx.x] = t1;
    }
}

// Line path, one rank, canonical line-separable rows: the table SpMV y = A p
// formed inside the sweep kernel -- the lane's column of p along its segment, one line either
// side, in registers; p at v -+ 1 from the neighbouring lanes (DPP wave shifts; a wave covers 64
// positions, 128-B aligned rows, and the two columns just outside them arrive in LDS by LDS-DMA:
// no VGPR holds them -- round 6; the 62-position waves with a halo lane either side read
// misaligned 512-B rows, five cache lines for four, PMC 1.15x) -- then k_line_apply's sweeps and
// dots on it (COMPACT, DCD).  y is neither written nor read back (two vectors less per step) and
// p is read once for the SpMV and the dots.  The SpMV's products and their order are
// k_lsv_ring's (canonical row order), the sweeps k_line_apply's: w is bit-identical to the
// two-kernel form; the dots' partials follow the 64-lane blocks (another fixed order: the DCGS2
// bars).
template <int LMAX>
__global__ __launch_bounds__(NT) void k_line_spmv_dc(LineOp L, const double *__restrict__ lsv,
                                                     const double *__restrict__ p, double *__restrict__ w, int nb,
                                                     const int *stop_col, int col, LineDc dc) {
    constexpr int NQW = 2 * DC_MAXJ + 3;
    constexpr int HW = 4 * LMAX <= 64 ? 1 : 2;   // LDS-DMA instructions for the halo columns
    __shared__ double stage[(NT / 64) * NQW];
    __shared__ double halo[NT / 64][32 * HW];    // per wave: [line u][left, right] of the 64 columns
    if (stopped(stop_col, col)) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int n = (int)L.n, Lb = (int)L.stride, X = n / Lb, seg = (int)L.seg;
    const int64_t nitems = L.nseg * nb;
    const double *m = L.f + L.n;
    double dsl = 0.0, dzl = 0.0, daa = 0.0, dab = 0.0, dag = 0.0;
    for (int64_t t = (int64_t)blockIdx.x * (NT / 64) + wv; t < nitems; t += (int64_t)gridDim.x * (NT / 64)) {
        const int sg = (int)(t / nb), jw = (int)(t - (int64_t)sg * nb);
        const int xb = sg * seg, len = min(seg, X - xb);
        const int v0 = jw * 64, vv = v0 + lane;
        const bool use = vv < Lb;
        const int v = use ? vv : 0;
        const double aj = use ? L.ac[v] : 0.0, cj = use ? L.ac[L.jn + v] : 0.0;
        const double tx0 = lsv[n + v], tx1 = lsv[n + Lb + v];
        // the columns v0 - 1 and v0 + 64 of lines xb .. xb + len - 1 (the v -+ 1 neighbours of the
        // wave's first and last lane), one dword per lane straight into LDS; a column off the line
        // (v0 = 0, or v0 + 64 >= Lb: its term is skipped) reads the wave's own column instead
#pragma unroll
        for (int i = 0; i < HW; ++i) {
            const int d = 64 * i + lane, u = d >> 2, side = (d >> 1) & 1, half = d & 1;
            const int x = xb + min(u, len - 1);
            int vc = side ? v0 + 64 : v0 - 1;
            vc = vc < 0 || vc >= Lb ? v0 : vc;
            const char *src = reinterpret_cast<const char *>(p + (x * Lb + vc)) + 4 * half;
            __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void *)&halo[wv][32 * i], 4, 0, 0);
        }
        // p on the column: lines xb - 1 .. xb + len (periodic in x)
        double pc[LMAX + 2];
#pragma unroll
        for (int u = 0; u < LMAX + 2; ++u) {
            int x = xb - 1 + min(u, len + 1);
            x = x < 0 ? x + X : (x >= X ? x - X : x);
            pc[u] = ld_nt<8>(p + (x * Lb + v));
        }
        // every column load is in flight before the first wait (unfenced, the scheduler hoists the
        // first line's DPP shifts above the later loads: one memory latency per item); the halo
        // columns have landed once at most the column loads are outstanding (in order)
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LMAX + 2) : "memory");
        double e[LMAX], gg[LMAX];
        double dp = 0.0, mp = 0.0;
        bool pok = false;
        unsigned okm = 0;
#pragma unroll
        for (int u = 0; u < LMAX; ++u) {
            const bool ok = use && u < len;
            const int x = xb + min(u, len - 1);
            const int k = ok ? x * Lb + v : 0;
            const double mv = ld_nt<8>(m + k);
            // y(x, v): the row's five terms in the canonical order of line x (k_lsv_ring)
            const double drow = ld_nt<8>(lsv + (x * Lb + v));
            const double tv0 = lsv[n + 2 * Lb + x], tv1 = lsv[n + 2 * Lb + X + x];
            const double c0 = pc[u + 1];
            // v -+ 1: the neighbouring lanes' values by DPP wave shifts (wave_shr:1 / wave_shl:1),
            // the first and last lane's from the halo columns in LDS
            const double hm = halo[wv][2 * u], hq = halo[wv][2 * u + 1];
            const double sm = dpp_mov<0x138>(c0), sq = dpp_mov<0x130>(c0);
            const double pm = lane == 0 ? hm : sm, pq = lane == 63 ? hq : sq;
            const double t0 = tx0 * pc[u], t4 = tx1 * pc[u + 2], t2 = drow * c0, t1 = tv0 * pm, t3 = tv1 * pq;
            const bool h1 = v > 0, h3 = v < Lb - 1;
            double sa = 0.0;
            if (x == 0) {   // x - 1 wraps to line X - 1: last
                sa = h1 ? sa + t1 : sa;
                sa = sa + t2;
                sa = h3 ? sa + t3 : sa;
                sa = sa + t4;
                sa = sa + t0;
            } else if (x == X - 1) {   // x + 1 wraps to line 0: first
                sa = sa + t4;
                sa = sa + t0;
                sa = h1 ? sa + t1 : sa;
                sa = sa + t2;
                sa = h3 ? sa + t3 : sa;
            } else {
                sa = sa + t0;
                sa = h1 ? sa + t1 : sa;
                sa = sa + t2;
                sa = h3 ? sa + t3 : sa;
                sa = sa + t4;
            }
            // k_line_apply<LMAX, COMPACT>'s forward sweep on r = y
            const bool hl = ok && pok;
            const bool hr = ok && u + 1 < len && k + Lb < n;
            const double lv = hl ? aj * mp : 0.0;
            const double gv = (hr ? cj : 0.0) * mv;
            const double dv = sa - lv * dp;
            e[u] = mv * dv;
            gg[u] = gv;
            if (ok) {
                dp = dv;
                mp = mv;
            }
            pok = ok;
            okm |= (unsigned)ok << u;
        }
        double zn = 0.0;
#pragma unroll
        for (int u = LMAX - 1; u >= 0; --u) {
            const double zv = e[u] - gg[u] * zn;
            if ((okm >> u) & 1u) {
                st_nt<4>(w + ((xb + u) * Lb + v), zv);
                zn = zv;
            }
            e[u] = ((okm >> u) & 1u) ? zv : 0.0;   // w, kept for the dots
        }
        // the dots (k_line_apply's DCD), p from the column
#pragma unroll
        for (int u = 0; u < LMAX; ++u) gg[u] = ((okm >> u) & 1u) ? pc[u + 1] : 0.0;
#pragma unroll
        for (int u = 0; u < LMAX; ++u) {
            daa += gg[u] * gg[u];
            dab += gg[u] * e[u];
            dag += e[u] * e[u];
        }
        for (int kk = 0; kk < dc.j; ++kk) {
            const double *vk = dc.V + (size_t)kk * dc.ld;
            double sl = 0.0, zl = 0.0;
#pragma unroll
            for (int u = 0; u < LMAX; ++u) {
                const double vvk = ((okm >> u) & 1u) ? __builtin_nontemporal_load(vk + ((xb + u) * Lb + v)) : 0.0;
                sl += vvk * gg[u];
                zl += vvk * e[u];
            }
            const double ts = wave_allsum(sl), tz = wave_allsum(zl);
            if (lane == kk) {
                dsl += ts;
                dzl += tz;
            }
        }
    }
    double *rec = stage + wv * NQW;
    if (lane < dc.j) {
        rec[lane] = dsl;
        rec[DC_MAXJ + lane] = dzl;
    }
    const double t0 = wave_sum(daa), t1 = wave_sum(dab), t2 = wave_sum(dag);
    if (lane == 0) {
        rec[2 * DC_MAXJ] = t0;
        rec[2 * DC_MAXJ + 1] = t1;
        rec[2 * DC_MAXJ + 2] = t2;
    }
    __syncthreads();
    for (int qq = threadIdx.x; qq < DC_NQ; qq += NT) {
        const bool used = qq < dc.j || (qq >= DC_MAXJ && qq < DC_MAXJ + dc.j) || qq >= 2 * DC_MAXJ;
        if (used) {
            double t = 0.0;
#pragma unroll
            for (int w2 = 0; w2 < NT / 64; ++w2) t += stage[w2 * NQW + qq];
            dc.part[(size_t)qq * GMAX + blockIdx.x] = t;
        }
    }
}

hipError_t launch_line_spmv_dc(const LineOp &L, const double *lsv, const double *p, double *w, const double *V,
                               int64_t ld, int j, double *part, int grid, const int *stop_col, int col, hipStream_t s) {
    const int64_t Lb = L.stride, X = Lb > 0 ? L.n / Lb : 0;
    // one rank's whole slab, lines of Lb rows, the lanes over every position, compact factors
    if (!L.compact || !L.ac || L.row0 != 0 || Lb <= 0 || L.n % Lb != 0 || X < 3 || L.j0 != 0 || L.jn != Lb ||
        L.i_lo != 0 || L.i_hi != X - 1 || L.seg <= 0 || L.seg > 32 || j < 0 || j > DC_MAXJ || grid < 1 ||
        grid > GMAX || L.n > INT32_MAX / 2 || !lsv || !p || !part)
        return hipErrorInvalidValue;
    const int nb = (int)((Lb + 63) / 64);
    const dim3 g(grid), b(NT);
    const LineDc dc{V, ld, j, p, part};
    if (L.seg <= 8) hipLaunchKernelGGL(k_line_spmv_dc<8>, g, b, 0, s, L, lsv, p, w, nb, stop_col, col, dc);
    else if (L.seg <= 16) hipLaunchKernelGGL(k_line_spmv_dc<16>, g, b, 0, s, L, lsv, p, w, nb, stop_col, col, dc);
    else if (L.seg <= 25) hipLaunchKernelGGL(k_line_spmv_dc<25>, g, b, 0, s, L, lsv, p, w, nb, stop_col, col, dc);
    else hipLaunchKernelGGL(k_line_spmv_dc<32>, g, b, 0, s, L, lsv, p, w, nb, stop_col, col, dc);
    return hipGetLastError();
}

hipError_t launch_line_setup(const int32_t *indptr, const int32_t *indices, const void *data, int fp32,
                             const LineOp &L, unsigned long long *bad_row, unsigned long long *ext, hipStream_t s) {
    const int64_t threads = L.nseg * L.jb * 64;
    if (threads == 0) return hipSuccess;
    const dim3 g((unsigned)((threads + NT - 1) / NT));
    if (fp32) hipLaunchKernelGGL(k_line_setup<float>, g, dim3(NT), 0, s, indptr, indices, (const float *)data, L, bad_row, ext);
    else hipLaunchKernelGGL(k_line_setup<double>, g, dim3(NT), 0, s, indptr, indices, (const double *)data, L, bad_row, ext);
    return hipGetLastError();
}

// line apply + DCGS2 dots of step j (segments <= 32; else hipErrorInvalidValue: the caller
// runs the unfused dots)
hipError_t launch_line_dc(const LineOp &L, const double *r, double *w, const double *V, int64_t ld, int j,
                          const double *p, double *part, int grid, const int *stop_col, int col, hipStream_t s) {
    if (j > DC_MAXJ || grid > GMAX || L.seg > 32 || L.seg <= 0) return hipErrorInvalidValue;
    const dim3 g(grid), b(NT);
    const LineDc dc{V, ld, j, p, part};
#define VTK_LINE_DC_LAUNCH(LM)                                                                               \
    do {                                                                                                     \
        if (L.compact) hipLaunchKernelGGL((k_line_apply<LM, true, true>), g, b, 0, s, L, r, w, nullptr, nullptr, nullptr, stop_col, col, dc); \
        else hipLaunchKernelGGL((k_line_apply<LM, false, true>), g, b, 0, s, L, r, w, nullptr, nullptr, nullptr, stop_col, col, dc);        \
    } while (0)
    if (L.seg <= 8) VTK_LINE_DC_LAUNCH(8);
    else if (L.seg <= 16) VTK_LINE_DC_LAUNCH(16);
    else if (L.seg <= 25) VTK_LINE_DC_LAUNCH(25);
    else VTK_LINE_DC_LAUNCH(32);
#undef VTK_LINE_DC_LAUNCH
    return hipGetLastError();
}

hipError_t launch_line_apply(const LineOp &L, const double *r, double *z, const double *v0, double *part0,
                             double *part1, int grid, const int *stop_col, int col, hipStream_t s) {
    if (L.n == 0 && part0 == nullptr) return hipSuccess;
    const dim3 g(grid), b(NT);
#define VTK_LINE_LAUNCH(LM)                                                                                  \
    do {                                                                                                     \
        if (L.compact) hipLaunchKernelGGL((k_line_apply<LM, true>), g, b, 0, s, L, r, z, v0, part0, part1, stop_col, col); \
        else hipLaunchKernelGGL((k_line_apply<LM, false>), g, b, 0, s, L, r, z, v0, part0, part1, stop_col, col);        \
    } while (0)
    if (L.seg <= 8) VTK_LINE_LAUNCH(8);
    else if (L.seg <= 16) VTK_LINE_LAUNCH(16);
    else if (L.seg <= 25) VTK_LINE_LAUNCH(25);
    else if (L.seg <= 32) VTK_LINE_LAUNCH(32);
    else hipLaunchKernelGGL((k_line_apply<0, false>), g, b, 0, s, L, r, z, v0, part0, part1, stop_col, col);
#undef VTK_LINE_LAUNCH
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// block-Jacobi setup: dense diagonal block, Gauss-Jordan with partial pivoting.
// BS a power of two <= 64: one lane per block row (BS lanes per block), rows swapped and the
// pivot row broadcast with cross-lane shuffles, everything in registers.  Same op sequence as
// orc_bj_setup.  Other bs: one lane per block, block in a global workspace.
// ------------------------------------------------------------------------------------------
template <typename VT, int BS>
__global__ __launch_bounds__(NT) void k_bj_setup(const int32_t *__restrict__ indptr,
                                                 const int32_t *__restrict__ indices,
                                                 const VT *__restrict__ data, int64_t n,
                                                 int64_t nb, double *__restrict__ inv, int *singular) {
    const int64_t gt = (int64_t)blockIdx.x * NT + threadIdx.x;
    const int64_t blk = gt / BS;
    const int ii = (int)(gt % BS);
    const int lane = threadIdx.x & 63;
    const int gb = lane & ~(BS - 1);
    const bool live = blk < nb;
    const int64_t row = blk * BS + ii;
    double A[BS], I[BS];
#pragma unroll
    for (int j = 0; j < BS; ++j) {
        A[j] = 0.0;
        I[j] = (j == ii) ? 1.0 : 0.0;
    }
    if (live) {
        if (row >= n) {
#pragma unroll
            for (int j = 0; j < BS; ++j) if (j == ii) A[j] = 1.0;
        } else {
            const int64_t c0 = blk * BS;
            for (int k = indptr[row]; k < indptr[row + 1]; ++k) {
                if (indices[k] >= n) continue;   // halo column (local numbering >= n_local)
                const int64_t c = indices[k] - c0;
                const double v = (double)data[k];
#pragma unroll
                for (int j = 0; j < BS; ++j) if (c == j) A[j] = A[j] + v;   // duplicates add (toarray)
            }
        }
    }
    bool sing = false;
#pragma unroll
    for (int c = 0; c < BS; ++c) {
        // pivot: first row r >= c with the largest |A[r][c]|
        double best = (ii >= c) ? __builtin_fabs(A[c]) : -1.0;
        int bidx = ii;
#pragma unroll
        for (int off = 1; off < BS; off <<= 1) {
            const double ob = __shfl_xor(best, off, 64);
            const int oi = __shfl_xor(bidx, off, 64);
            if (ob > best || (ob == best && oi < bidx)) { best = ob; bidx = oi; }
        }
        if (best == 0.0) sing = true;
        const int piv = bidx;
        // swap rows c and piv
#pragma unroll
        for (int j = 0; j < BS; ++j) {
            const double ac = __shfl(A[j], gb + c, 64), ap = __shfl(A[j], gb + piv, 64);
            const double ic = __shfl(I[j], gb + c, 64), ip = __shfl(I[j], gb + piv, 64);
            if (ii == c) { A[j] = ap; I[j] = ip; }
            else if (ii == piv) { A[j] = ac; I[j] = ic; }
        }
        const double d = __shfl(A[c], gb + c, 64);
        if (ii == c) {
#pragma unroll
            for (int j = 0; j < BS; ++j) { A[j] = A[j] / d; I[j] = I[j] / d; }
        }
        const double f = A[c];
#pragma unroll
        for (int j = 0; j < BS; ++j) {
            const double pa = __shfl(A[j], gb + c, 64), pi = __shfl(I[j], gb + c, 64);
            if (ii != c) { A[j] = A[j] - f * pa; I[j] = I[j] - f * pi; }
        }
    }
    if (live) {
        if (sing && ii == 0) atomicMin(singular, (int)blk);
        double *o = inv + (size_t)(blk * BS + ii) * BS;
#pragma unroll
        for (int j = 0; j < BS; ++j) o[j] = I[j];
    }
}

template <typename VT>
__global__ __launch_bounds__(NT) void k_bj_setup_generic(const int32_t *__restrict__ indptr,
                                                         const int32_t *__restrict__ indices,
                                                         const VT *__restrict__ data, int64_t n,
                                                         int64_t nb, int bs, double *__restrict__ inv,
                                                         double *__restrict__ work, int *singular) {
    const int64_t blk = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (blk >= nb) return;
    double *A = work + (size_t)blk * bs * bs;
    double *I = inv + (size_t)blk * bs * bs;
    for (int k = 0; k < bs * bs; ++k) { A[k] = 0.0; I[k] = 0.0; }
    for (int i = 0; i < bs; ++i) {
        const int64_t row = blk * bs + i;
        I[i * bs + i] = 1.0;
        if (row >= n) { A[i * bs + i] = 1.0; continue; }
        for (int k = indptr[row]; k < indptr[row + 1]; ++k) {
            if (indices[k] >= n) continue;   // halo column
            const int64_t c = indices[k] - blk * bs;
            if (c >= 0 && c < bs) A[i * bs + c] = A[i * bs + c] + (double)data[k];
        }
    }
    for (int c = 0; c < bs; ++c) {
        int piv = c;
        double best = __builtin_fabs(A[c * bs + c]);
        for (int r = c + 1; r < bs; ++r) {
            const double v = __builtin_fabs(A[r * bs + c]);
            if (v > best) { best = v; piv = r; }
        }
        if (best == 0.0) { atomicMin(singular, (int)blk); return; }
        if (piv != c) {
            for (int j = 0; j < bs; ++j) {
                double t = A[c * bs + j]; A[c * bs + j] = A[piv * bs + j]; A[piv * bs + j] = t;
                t = I[c * bs + j]; I[c * bs + j] = I[piv * bs + j]; I[piv * bs + j] = t;
            }
        }
        const double d = A[c * bs + c];
        for (int j = 0; j < bs; ++j) { A[c * bs + j] = A[c * bs + j] / d; I[c * bs + j] = I[c * bs + j] / d; }
        for (int r = 0; r < bs; ++r) {
            if (r == c) continue;
            const double f = A[r * bs + c];
            for (int j = 0; j < bs; ++j) {
                A[r * bs + j] = A[r * bs + j] - f * A[c * bs + j];
                I[r * bs + j] = I[r * bs + j] - f * I[c * bs + j];
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// Block-Jacobi setup on the matrix cores (bs 16, 32): blocked Gauss-Jordan with
// partial pivoting, one wave per diagonal block, [A | I] (BS x 2BS) staged in LDS.  Per panel of
// 4 columns the lanes (one per row) run the 4 pivot steps on the panel and on W (the transformed
// unit vectors e_c, inserted at their step), which gives the panel's transform as I + U C^T
// after the recorded row swaps; the rest of [A | I] is updated by  Q += U Q[C, :]  -- a rank-4
// update: one v_mfma_f64_16x16x4f64 per 16x16 tile (operand maps checked by
// tools/probe_mfma_f64.hip).  Pivots: the first row of largest |a| among the unpivoted rows, as
// the scalar kernel; the rank-4 sums round differently from its rank-1 sequence, so the inverse
// agrees to ~1e-15 relative, not bit for bit (a tolerance mode, VTK_BJ_SETUP_MFMA).
// ------------------------------------------------------------------------------------------
typedef double d4v __attribute__((ext_vector_type(4)));
// NB blocks per wave: lane group g = lane / BS holds the rows of block g during the load and the
// panel pivoting (bs 16: four blocks per wave, every lane busy); the MFMA tiles of the NB blocks
// are issued back to back by the whole wave.
template <typename VT, int BS, int NB>
__global__ __launch_bounds__(256) void k_bj_setup_mfma(const int32_t *__restrict__ indptr,
                                                        const int32_t *__restrict__ indices,
                                                        const VT *__restrict__ data, int64_t n, int64_t nb,
                                                        double *__restrict__ inv, int *singular) {
    constexpr int S = 2 * BS + 1;          // LDS row stride (odd: conflict-free column reads)
    constexpr int RT = BS / 16, CT = 2 * BS / 16;
    static_assert(NB * BS <= 64, "one lane per block row");
    __shared__ double Ts[4][NB][BS * S];
    __shared__ double Ws[4][NB][BS * 4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int grp = lane / BS, r = lane % BS;
    const bool gl = grp < NB;              // a lane of a block group
    const int64_t blk0 = ((int64_t)blockIdx.x * 4 + wv) * NB;
    if (blk0 >= nb) return;                // wave-uniform; no workgroup barrier below
    const int64_t blk = blk0 + (gl ? grp : 0);
    const bool live = gl && blk < nb;      // blocks past nb: identity, not stored
    // [A | I]: the block's rows (duplicates add, halo columns skipped), padding rows = identity
    for (int g = 0; g < NB; ++g)
        for (int e = lane; e < BS * 2 * BS; e += 64) {
            const int rr = e / (2 * BS), cc = e % (2 * BS);
            Ts[wv][g][rr * S + cc] = (cc == BS + rr || (blk0 + g >= nb && cc == rr)) ? 1.0 : 0.0;
        }
    __builtin_amdgcn_wave_barrier();
    if (live) {
        double *T = Ts[wv][grp];
        const int64_t row = blk * BS + r;
        if (row >= n) {
            T[r * S + r] = 1.0;
        } else {
            const int64_t c0 = blk * BS;
            for (int k = indptr[row]; k < indptr[row + 1]; ++k) {
                if (indices[k] >= n) continue;
                const int64_t cc = indices[k] - c0;
                if (cc >= 0 && cc < BS) T[r * S + cc] = T[r * S + cc] + (double)data[k];
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    double *Tg = Ts[wv][gl ? grp : 0];
    double *Wg = Ws[wv][gl ? grp : 0];
    const int gb = (gl ? grp : 0) * BS;    // first lane of the group
    bool sing = false;
    for (int c0 = 0; c0 < BS; c0 += 4) {
        // panel: lane r of group g holds row r of block g's 4 panel columns and of W
        double pr[4], wr[4];
        int pv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            pr[k] = gl ? Tg[r * S + c0 + k] : 0.0;
            wr[k] = 0.0;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int c = c0 + k;
            double best = (gl && r >= c) ? __builtin_fabs(pr[k]) : -1.0;
            int bidx = r;
#pragma unroll
            for (int off = 1; off < BS; off <<= 1) {
                const double ob = __shfl_xor(best, off, 64);
                const int oi = __shfl_xor(bidx, off, 64);
                if (ob > best || (ob == best && oi < bidx)) { best = ob; bidx = oi; }
            }
            if (best == 0.0 && live) sing = true;
            const int piv = bidx;
            pv[k] = piv;
            // swap rows c and piv of the panel and W (within the group)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const double pc = __shfl(pr[q], gb + c, 64), pp = __shfl(pr[q], gb + piv, 64);
                const double wc = __shfl(wr[q], gb + c, 64), wp = __shfl(wr[q], gb + piv, 64);
                if (r == c) { pr[q] = pp; wr[q] = wp; }
                else if (r == piv) { pr[q] = pc; wr[q] = wc; }
            }
            wr[k] = r == c ? 1.0 : 0.0;   // e_c enters W at its step
            const double d = __shfl(pr[k], gb + c, 64);
            if (r == c) {
#pragma unroll
                for (int q = 0; q < 4; ++q) { pr[q] = pr[q] / d; wr[q] = wr[q] / d; }
            }
            const double f = pr[k];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const double pcq = __shfl(pr[q], gb + c, 64), wcq = __shfl(wr[q], gb + c, 64);
                if (r != c) { pr[q] = pr[q] - f * pcq; wr[q] = wr[q] - f * wcq; }
            }
        }
        // U = W - [e_c0 .. e_c0+3]
        if (gl) {
#pragma unroll
            for (int k = 0; k < 4; ++k) Wg[r * 4 + k] = wr[k] - (r == c0 + k ? 1.0 : 0.0);
        }
        // the panel's row swaps on the whole of [A | I] (Q = P [A | I]), per group
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int c = c0 + k;
            __builtin_amdgcn_wave_barrier();
            if (gl && pv[k] != c) {
                for (int cc = r; cc < 2 * BS; cc += BS) {
                    const double x0 = Tg[c * S + cc], x1 = Tg[pv[k] * S + cc];
                    Tg[c * S + cc] = x1;
                    Tg[pv[k] * S + cc] = x0;
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        // Q += U Q[C, :] for every block: the pivot rows (B operands) read before any tile is written
        double bq[NB][CT], ua[NB][RT];
#pragma unroll
        for (int g = 0; g < NB; ++g) {
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) bq[g][ct] = Ts[wv][g][(c0 + (lane >> 4)) * S + ct * 16 + (lane & 15)];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) ua[g][rt] = Ws[wv][g][(rt * 16 + (lane & 15)) * 4 + (lane >> 4)];
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int g = 0; g < NB; ++g) {
            double *T = Ts[wv][g];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
                for (int ct = 0; ct < CT; ++ct) {
                    d4v acc;
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[i] = T[(rt * 16 + (lane >> 4) + 4 * i) * S + ct * 16 + (lane & 15)];
                    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(ua[g][rt], bq[g][ct], acc, 0, 0, 0);
                    const int col = ct * 16 + (lane & 15);
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int rr = rt * 16 + (lane >> 4) + 4 * i;
                        // the panel columns are exactly e_C after their eliminations
                        T[rr * S + col] = (col >= c0 && col < c0 + 4) ? (rr == col ? 1.0 : 0.0) : acc[i];
                    }
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (sing && r == 0) atomicMin(singular, (int)blk);
    if (live) {
        double *o = inv + (size_t)blk * BS * BS;
        for (int e = r; e < BS * BS; e += BS) o[e] = Tg[(e / BS) * S + BS + e % BS];
    }
}

template <typename VT>
static hipError_t bj_setup_mfma_t(const int32_t *indptr, const int32_t *indices, const VT *data, int64_t n, int bs,
                                  double *inv, int *sing, hipStream_t s) {
    const int64_t nb = (n + bs - 1) / bs;
    if (nb == 0) return hipSuccess;
    if (bs == 16) {   // 4 blocks per wave, 16 per workgroup
        const dim3 g((unsigned)((nb + 15) / 16));
        hipLaunchKernelGGL((k_bj_setup_mfma<VT, 16, 4>), g, dim3(256), 0, s, indptr, indices, data, n, nb, inv, sing);
    } else if (bs == 32) {
        const dim3 g((unsigned)((nb + 3) / 4));
        hipLaunchKernelGGL((k_bj_setup_mfma<VT, 32, 1>), g, dim3(256), 0, s, indptr, indices, data, n, nb, inv, sing);
    }
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_bj_setup_mfma(const int32_t *indptr, const int32_t *indices, const void *data, int fp32, int64_t n,
                                int bs, double *inv, int *d_singular, hipStream_t s) {
    if (fp32) return bj_setup_mfma_t<float>(indptr, indices, static_cast<const float *>(data), n, bs, inv, d_singular, s);
    return bj_setup_mfma_t<double>(indptr, indices, static_cast<const double *>(data), n, bs, inv, d_singular, s);
}

template <typename VT>
static hipError_t bj_setup_t(const int32_t *indptr, const int32_t *indices, const VT *data, int64_t n,
                             int bs, double *inv, int *sing, double *work, hipStream_t s) {
    const int64_t nb = (n + bs - 1) / bs;
    if (nb == 0) return hipSuccess;
    const int64_t threads = nb * bs;
    const dim3 g((unsigned)((threads + NT - 1) / NT));
    switch (bs) {
        case 1: hipLaunchKernelGGL((k_bj_setup<VT, 1>), g, dim3(NT), 0, s, indptr, indices, data, n, nb, inv, sing); break;
        case 2: hipLaunchKernelGGL((k_bj_setup<VT, 2>), g, dim3(NT), 0, s, indptr, indices, data, n, nb, inv, sing); break;
        case 4: hipLaunchKernelGGL((k_bj_setup<VT, 4>), g, dim3(NT), 0, s, indptr, indices, data, n, nb, inv, sing); break;
        case 8: hipLaunchKernelGGL((k_bj_setup<VT, 8>), g, dim3(NT), 0, s, indptr, indices, data, n, nb, inv, sing); break;
        case 16: hipLaunchKernelGGL((k_bj_setup<VT, 16>), g, dim3(NT), 0, s, indptr, indices, data, n, nb, inv, sing); break;
        case 32: hipLaunchKernelGGL((k_bj_setup<VT, 32>), g, dim3(NT), 0, s, indptr, indices, data, n, nb, inv, sing); break;
        default: {
            const dim3 gg((unsigned)((nb + NT - 1) / NT));
            hipLaunchKernelGGL(k_bj_setup_generic<VT>, gg, dim3(NT), 0, s, indptr, indices, data, n, nb,
                               bs, inv, work, sing);
        }
    }
    return hipGetLastError();
}

hipError_t launch_bj_setup(const int32_t *indptr, const int32_t *indices, const void *data, int fp32,
                           int64_t n, int bs, double *inv, int *d_singular, double *work, hipStream_t s) {
    if (fp32) return bj_setup_t<float>(indptr, indices, static_cast<const float *>(data), n, bs, inv, d_singular, work, s);
    return bj_setup_t<double>(indptr, indices, static_cast<const double *>(data), n, bs, inv, d_singular, work, s);
}

// ------------------------------------------------------------------------------------------
// Modified Gram-Schmidt step (iterative.py:756-759): h = <v_k, w> (reduced); w -= h*v_k;
// fused with the partial <v_{k+1}, w> of the next step (or ||w||^2 after the last one).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void k_mgs(Red hin, double *hout, double *__restrict__ w,
                                            const double *__restrict__ vk,
                                            const double *__restrict__ vn, int64_t n,
                                            double *part_out, const int *stop_col, int col) {
    __shared__ double red[NT / 64];
    if (stopped(stop_col, col)) return;
    const double h = reduce_red(hin, red);
    if (blockIdx.x == 0 && threadIdx.x == 0 && hout) *hout = h;
    double acc = 0.0;
    const int64_t stride = 2 * (int64_t)gridDim.x * NT;
    for (int64_t i = 2 * ((int64_t)blockIdx.x * NT + threadIdx.x); i < n; i += stride) {
        if (i + 1 < n) {
            double2 wv = *reinterpret_cast<const double2 *>(w + i);
            const d2v kv = ldnt2(vk + i);
            wv.x = wv.x - h * kv.x;
            wv.y = wv.y - h * kv.y;
            *reinterpret_cast<double2 *>(w + i) = wv;
            if (vn) {
                const double2 nv = *reinterpret_cast<const double2 *>(vn + i);
                acc += nv.x * wv.x;
                acc += nv.y * wv.y;
            } else {
                acc += wv.x * wv.x;
                acc += wv.y * wv.y;
            }
        } else {
            const double wv = w[i] - h * vk[i];
            w[i] = wv;
            acc += (vn ? vn[i] : wv) * wv;
        }
    }
    const double t = block_sum(acc, red);
    if (threadIdx.x == 0) part_out[blockIdx.x] = t;
}

hipError_t launch_mgs(Red hin, double *hout, double *w, const double *vk, const double *vnext,
                      int64_t n, double *part_out, int grid, const int *stop_col, int col,
                      hipStream_t s) {
    hipLaunchKernelGGL(k_mgs, dim3(grid), dim3(NT), 0, s, hin, hout, w, vk, vnext, n, part_out,
                       stop_col, col);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Arnoldi tail (iterative.py:761-794): h1 = ||w||, breakdown test, v_{col+1} = w * (1/h1);
// workgroup 0 / lane 0 rotates column col of H and decides whether the cycle stops.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void k_tail(Red h0r, Red w2r, const double *__restrict__ w,
                                             double *__restrict__ vn, int64_t n, int col, int m,
                                             double *H, double *S, double *giv, GmresState *st,
                                             int *stop_map) {
    __shared__ double red[NT / 64];
    if (st->stop_col < col) return;
    const double h0 = __builtin_sqrt(reduce_red(h0r, red));
    const double h1 = __builtin_sqrt(reduce_red(w2r, red));
    const bool brk = h1 <= DBL_EPSILON * h0;
    const double sc = brk ? 1.0 : 1.0 / h1;
    const int64_t stride = 2 * (int64_t)gridDim.x * NT;
    for (int64_t i = 2 * ((int64_t)blockIdx.x * NT + threadIdx.x); i < n; i += stride) {
        if (i + 1 < n) {
            double2 v = *reinterpret_cast<const double2 *>(w + i);
            v.x = v.x * sc;
            v.y = v.y * sc;
            *reinterpret_cast<double2 *>(vn + i) = v;
        } else {
            vn[i] = w[i] * sc;
        }
    }
    __shared__ double hcs[MAX_RESTART + 1];
    if (blockIdx.x == 0) {   // LDS copy of column col: the rotation chain never touches global memory
        for (int k = threadIdx.x; k <= col; k += NT) hcs[k] = H[(size_t)col * (m + 1) + k];
        __syncthreads();
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        double *hc = hcs;
        hc[col + 1] = brk ? 0.0 : h1;
        for (int k = 0; k < col; ++k) {
            const double c = giv[2 * k], s = giv[2 * k + 1];
            const double n0 = hc[k], n1 = hc[k + 1];
            hc[k] = c * n0 + s * n1;
            hc[k + 1] = -s * n0 + c * n1;
        }
        double c, s, mag;
        d_lartg(hc[col], hc[col + 1], c, s, mag);
        giv[2 * col] = c;
        giv[2 * col + 1] = s;
        hc[col] = mag;
        hc[col + 1] = 0.0;
        double *hg = H + (size_t)col * (m + 1);
        for (int k = 0; k <= col + 1; ++k) hg[k] = hc[k];
        const double t = -s * S[col];
        S[col] = c * S[col];
        S[col + 1] = t;
        const double presid = __builtin_fabs(t);
        st->presid = presid;
        st->inner += 1;
        if (presid <= st->ptol || brk) {
            st->breakdown = brk ? 1 : 0;
            st->stop_col = col;
            if (stop_map) __hip_atomic_store(stop_map, col, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

hipError_t launch_tail(Red h0, Red w2, const double *w, double *vnext, int64_t n, int col, int m,
                       double *H, double *S, double *giv, GmresState *st, int *stop_map, int grid,
                       hipStream_t s) {
    hipLaunchKernelGGL(k_tail, dim3(grid), dim3(NT), 0, s, h0, w2, w, vnext, n, col, m, H, S, giv, st,
                       stop_map);
    return hipGetLastError();
}

// v0 *= 1/t (iterative.py:742-747)
__global__ __launch_bounds__(NT) void k_scale0(Red p, double *__restrict__ v0, int64_t n, double *S,
                                               int m, GmresState *st) {
    __shared__ double red[NT / 64];
    const double t = __builtin_sqrt(reduce_red(p, red));
    const double sc = 1.0 / t;
    const int64_t stride = 2 * (int64_t)gridDim.x * NT;
    for (int64_t i = 2 * ((int64_t)blockIdx.x * NT + threadIdx.x); i < n; i += stride) {
        if (i + 1 < n) {
            double2 v = *reinterpret_cast<const double2 *>(v0 + i);
            v.x = v.x * sc;
            v.y = v.y * sc;
            st_nt2<1>(v0 + i, v.x, v.y);
        } else {
            v0[i] = v0[i] * sc;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        for (int k = 0; k <= m; ++k) S[k] = 0.0;
        S[0] = t;
        st->stop_col = BIG_COL;
        st->breakdown = 0;
        st->xup_tag = -1;
    }
}

hipError_t launch_scale0(Red p, double *v0, int64_t n, double *S, int m, GmresState *st, int grid,
                         hipStream_t s) {
    hipLaunchKernelGGL(k_scale0, dim3(grid), dim3(NT), 0, s, p, v0, n, S, m, st);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// x += y @ V[0..col] with y from the (m+1) x m Hessenberg least squares
// (iterative.py:799-814).  Workgroup-redundant triangular solve on lane 0, into LDS.
// ------------------------------------------------------------------------------------------

__global__ __launch_bounds__(NT) void k_xupdate(const double *__restrict__ H, const double *__restrict__ S,
                                                const double *__restrict__ V, int64_t ld,
                                                double *__restrict__ x, int64_t n, int m,
                                                const GmresState *st) {
    extern __shared__ __attribute__((aligned(16))) double ys[];
    if (st->xup_tag >= 0) return;   // a DCGS2 update pass did it
    const int col = st->stop_col < m ? st->stop_col : m - 1;
    if (threadIdx.x == 0) hess_solve(H, S, m, col, ys);
    __syncthreads();
    const int64_t stride = 2 * (int64_t)gridDim.x * NT;
    for (int64_t i = 2 * ((int64_t)blockIdx.x * NT + threadIdx.x); i < n; i += stride) {
        if (i + 1 < n) {
            double ax = 0.0, ay = 0.0;
            for (int k = 0; k <= col; ++k) {
                const d2v v = ldnt2(V + (size_t)k * ld + i);
                ax += ys[k] * v.x;
                ay += ys[k] * v.y;
            }
            double2 xv = *reinterpret_cast<const double2 *>(x + i);
            xv.x = xv.x + ax;
            xv.y = xv.y + ay;
            st_nt2<1>(x + i, xv.x, xv.y);
        } else {
            double a = 0.0;
            for (int k = 0; k <= col; ++k) a += ys[k] * V[(size_t)k * ld + i];
            x[i] = x[i] + a;
        }
    }
}

hipError_t launch_xupdate(const double *H, const double *S, const double *V, int64_t ld, double *x,
                          int64_t n, int m, const GmresState *st, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_xupdate, dim3(grid), dim3(NT), (m + 1) * sizeof(double), s, H, S, V, ld, x, n, m, st);
    return hipGetLastError();
}

__global__ __launch_bounds__(NT) void k_finalize(Red p, double *dst, int do_sqrt) {
    __shared__ double red[NT / 64];
    const double t = reduce_red(p, red);
    if (threadIdx.x == 0) *dst = do_sqrt ? __builtin_sqrt(t) : t;
}

hipError_t launch_finalize(Red p, double *dst, int do_sqrt, hipStream_t s) {
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(NT), 0, s, p, dst, do_sqrt);
    return hipGetLastError();
}

__global__ __launch_bounds__(NT) void k_dot(const double *__restrict__ x, const double *__restrict__ y,
                                            int64_t n, double *part) {
    __shared__ double red[NT / 64];
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT)
        acc += x[i] * (y ? y[i] : x[i]);
    const double t = block_sum(acc, red);
    if (threadIdx.x == 0) part[blockIdx.x] = t;
}

// *flag = 1.0 if any x[i] != 0 (NaN counts as nonzero, as numpy's any); the caller zeroes it
__global__ __launch_bounds__(NT) void k_any_nonzero(const double *__restrict__ x, int64_t n, double *flag) {
    bool nz = false;
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) nz |= x[i] != 0.0;
    if (__any(nz) && (threadIdx.x & 63) == 0) *flag = 1.0;   // every writer stores the same value
}

hipError_t launch_any_nonzero(const double *x, int64_t n, double *flag, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_any_nonzero, dim3(vector_grid(n)), dim3(NT), 0, s, x, n, flag);
    return hipGetLastError();
}

hipError_t launch_dot(const double *x, const double *y, int64_t n, double *part, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_dot, dim3(grid), dim3(NT), 0, s, x, y, n, part);
    return hipGetLastError();
}

__global__ void k_gather(const double *__restrict__ x, const int32_t *__restrict__ idx, int64_t cnt,
                         double *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = x[idx[i]];
}

hipError_t launch_gather(const double *x, const int32_t *idx, int64_t cnt, double *out, hipStream_t s) {
    if (cnt == 0) return hipSuccess;
    const int g = (int)((cnt + NT - 1) / NT < 1024 ? (cnt + NT - 1) / NT : 1024);
    hipLaunchKernelGGL(k_gather, dim3(g), dim3(NT), 0, s, x, idx, cnt, out);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// device-side operator assembly: counts -> exclusive scan -> fill
// ------------------------------------------------------------------------------------------
// min / max of device column indices (vtk_csr_create with device arrays validates them before
// any SpMV gathers through them); integer atomics: exact in any order
__global__ __launch_bounds__(NT) void k_index_range(const int32_t *__restrict__ idx, int64_t n, int *mm) {
    int lo = INT_MAX, hi = INT_MIN;
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
        const int v = idx[i];
        lo = v < lo ? v : lo;
        hi = v > hi ? v : hi;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const int ol = __shfl_xor(lo, off, 64), oh = __shfl_xor(hi, off, 64);
        lo = ol < lo ? ol : lo;
        hi = oh > hi ? oh : hi;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMin(mm, lo);
        atomicMax(mm + 1, hi);
    }
}

hipError_t launch_index_range(const int32_t *idx, int64_t n, int *mm, hipStream_t s) {
    hipLaunchKernelGGL(k_index_range, dim3(1024), dim3(NT), 0, s, idx, n, mm);
    return hipGetLastError();
}

__global__ void k_vlasov_counts(vtk_vlasov_params p, int64_t r0, int64_t nrows, int32_t *counts) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nrows; i += (int64_t)gridDim.x * blockDim.x)
        counts[i] = vlasov_row_count(p, r0 + i);
    if (blockIdx.x == 0 && threadIdx.x == 0) counts[nrows] = 0;
}

template <typename VT>
__global__ void k_vlasov_fill(vtk_vlasov_params p, int64_t r0, int64_t nrows, const int32_t *indptr,
                              int32_t *indices, VT *data) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nrows; i += (int64_t)gridDim.x * blockDim.x) {
        VlasovRow row;
        vlasov_row(p, r0 + i, row);
        const int32_t o = indptr[i];
        for (int k = 0; k < row.count; ++k) {
            indices[o + k] = (int32_t)row.col[k];
            data[o + k] = (VT)row.val[k];
        }
    }
}

hipError_t launch_vlasov_counts(const vtk_vlasov_params &p, int64_t r0, int64_t nrows, int32_t *counts,
                                hipStream_t s) {
    hipLaunchKernelGGL(k_vlasov_counts, dim3(2048), dim3(NT), 0, s, p, r0, nrows, counts);
    return hipGetLastError();
}

hipError_t launch_vlasov_fill(const vtk_vlasov_params &p, int64_t r0, int64_t nrows, const int32_t *indptr,
                              int32_t *indices, void *data, hipStream_t s) {
    if (p.fp32)
        hipLaunchKernelGGL(k_vlasov_fill<float>, dim3(2048), dim3(NT), 0, s, p, r0, nrows, indptr, indices,
                           static_cast<float *>(data));
    else
        hipLaunchKernelGGL(k_vlasov_fill<double>, dim3(2048), dim3(NT), 0, s, p, r0, nrows, indptr, indices,
                           static_cast<double *>(data));
    return hipGetLastError();
}

hipError_t launch_exclusive_scan(const int32_t *in, int32_t *out, int64_t n, void *tmp, size_t *tmp_bytes,
                                 hipStream_t s) {
    return hipcub::DeviceScan::ExclusiveSum(tmp, *tmp_bytes, in, out, (int)n, s);
}

// global column -> local (owned: c - row_begin; halo: n_local + rank in halo_cols)
__global__ void k_remap(int32_t *indices, int64_t nnz, int64_t row_begin, int64_t n_local,
                        const int64_t *halo_cols, int64_t n_halo) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nnz; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t c = indices[k];
        const int64_t lc = c - row_begin;
        if (lc >= 0 && lc < n_local) {
            indices[k] = (int32_t)lc;
        } else {
            int64_t lo = 0, hi = n_halo;   // lower_bound
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (halo_cols[mid] < c) lo = mid + 1; else hi = mid;
            }
            indices[k] = (int32_t)(n_local + lo);
        }
    }
}

hipError_t launch_remap_cols(int32_t *indices, int64_t nnz, int64_t row_begin, int64_t n_local,
                             const int64_t *halo_cols, int64_t n_halo, hipStream_t s) {
    if (nnz == 0) return hipSuccess;
    hipLaunchKernelGGL(k_remap, dim3(2048), dim3(NT), 0, s, indices, nnz, row_begin, n_local, halo_cols, n_halo);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// DCGS2 Arnoldi (one global reduction per step).  State entering step j: V_j = [v_0..v_{j-1}]
// orthonormal, candidate p_j = V[j] (orthogonalised once, normalised by an estimate), raw
// Hessenberg column j-1 tentative.  Step j: w = M^-1 A p_j (SpMV); ONE pass of dots
// s = V_j^T p_j, z = V_j^T w, alpha = |p|^2, beta = p.w, gamma = |w|^2; the scalar step
// re-orthogonalises p_j (v_j = (p_j - V_j s)/r, r = sqrt(alpha - s.s)), finalises column j-1
// (h += nu s, h_{j,j-1} = nu r), runs SciPy's Givens/stop logic on it, and forms the tentative
// column j (c' = (e - H_j s)/r, e = [z; (beta - s.z)/r]) and nu_{j+1} = sqrt(gamma - e.e)/r;
// ONE update pass writes v_j and p_{j+1} = (w - [V_j v_j] e) / (r nu).  Derivation: DESIGN.md.
// ------------------------------------------------------------------------------------------
// The same dots with every thread owning row pairs (as k_dc_update): p and w are read once per
// row instead of once per wave, every basis vector streams through 16-B non-temporal loads and
// the thread keeps JM >= j accumulators per quantity.  Same partial layout.
template <int JM>
__global__ __launch_bounds__(NT) void k_dc_dots_rows(const double *__restrict__ V, int64_t ld, int j,
                                                     const double *__restrict__ w, int64_t n, double *part,
                                                     const int *stop_col, int col) {
    __shared__ double red[NT / 64][DC_NQ];
    if (stopped(stop_col, col)) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const double *p = V + (size_t)j * ld;
    double as[JM], az[JM];
#pragma unroll
    for (int k = 0; k < JM; ++k) { as[k] = 0.0; az[k] = 0.0; }
    double aa = 0.0, ab = 0.0, ag = 0.0;
    const int64_t stride = 2 * (int64_t)gridDim.x * NT;
    for (int64_t i = 2 * ((int64_t)blockIdx.x * NT + threadIdx.x); i < n; i += stride) {
        const bool two = i + 1 < n;
        double2 pv, wv2 = make_double2(0.0, 0.0);
        if (two) {
            pv = ld_nt2<4>(p + i);
            if (w) wv2 = ld_nt2<4>(w + i);
        } else {
            pv = make_double2(p[i], 0.0);
            if (w) wv2 = make_double2(w[i], 0.0);
        }
#pragma unroll
        for (int k = 0; k < JM; ++k) {
            if (k < j) {
                const double *vk = V + (size_t)k * ld + i;
                d2v v;
                if (two) v = ldnt2(vk);
                else { v.x = vk[0]; v.y = 0.0; }
                as[k] += v.x * pv.x;
                as[k] += v.y * pv.y;
                if (w) {
                    az[k] += v.x * wv2.x;
                    az[k] += v.y * wv2.y;
                }
            }
        }
        aa += pv.x * pv.x;
        aa += pv.y * pv.y;
        if (w) {
            ab += pv.x * wv2.x;
            ab += pv.y * wv2.y;
            ag += wv2.x * wv2.x;
            ag += wv2.y * wv2.y;
        }
    }
#pragma unroll
    for (int k = 0; k < JM; ++k) {
        if (k < j) {   // wave-uniform
            const double ts = wave_sum(as[k]);
            const double tz = w ? wave_sum(az[k]) : 0.0;
            if (lane == 0) { red[wv][k] = ts; red[wv][DC_MAXJ + k] = tz; }
        }
    }
    {
        const double t0 = wave_sum(aa), t1 = wave_sum(ab), t2 = wave_sum(ag);
        if (lane == 0) { red[wv][2 * DC_MAXJ] = t0; red[wv][2 * DC_MAXJ + 1] = t1; red[wv][2 * DC_MAXJ + 2] = t2; }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < DC_NQ; q += NT) {
        const bool used = q < j || (q >= DC_MAXJ && q < DC_MAXJ + j && w) || q == 2 * DC_MAXJ ||
                          (w && q > 2 * DC_MAXJ);
        if (used) {
            double t = 0.0;
#pragma unroll
            for (int w2 = 0; w2 < NT / 64; ++w2) t += red[w2][q];
            part[(size_t)q * GMAX + blockIdx.x] = t;
        }
    }
}

hipError_t launch_dc_dots(const double *V, int64_t ld, int j, const double *w, int64_t n, double *part,
                          int grid, const int *stop_col, int col, hipStream_t s) {
    if (j > DC_MAXJ) return hipErrorInvalidValue;
    const dim3 g(grid), b(NT);
    if (j <= 8) hipLaunchKernelGGL(k_dc_dots_rows<8>, g, b, 0, s, V, ld, j, w, n, part, stop_col, col);
    else if (j <= 16) hipLaunchKernelGGL(k_dc_dots_rows<16>, g, b, 0, s, V, ld, j, w, n, part, stop_col, col);
    else if (j <= 24) hipLaunchKernelGGL(k_dc_dots_rows<24>, g, b, 0, s, V, ld, j, w, n, part, stop_col, col);
    else hipLaunchKernelGGL(k_dc_dots_rows<DC_MAXJ>, g, b, 0, s, V, ld, j, w, n, part, stop_col, col);
    return hipGetLastError();
}

// one workgroup per used quantity: scal[q] = sum of its partials (fixed order)
__global__ __launch_bounds__(NT) void k_dc_finalize(const double *part, int cnt, int j, int with_w,
                                                    double *scal, const int *stop_col, int col) {
    __shared__ double red[NT / 64];
    if (stopped(stop_col, col)) return;
    const int b = blockIdx.x;
    int q;
    if (b < j) q = b;
    else if (with_w && b < 2 * j) q = DC_MAXJ + (b - j);
    else q = 2 * DC_MAXJ + (b - (with_w ? 2 * j : j));
    const double t = block_sum(strided_sum<GMAX / NT, NT>(part + (size_t)q * GMAX, cnt, threadIdx.x), red);
    if (threadIdx.x == 0) scal[q] = t;
    // the rank's failure vote (DC_VOTE, set by the host when one of its launches failed) rides
    // in the step's all-reduce: a nonzero sum stops every rank at this step (dc_scalar_body)
    if (b == 0 && threadIdx.x == 0) scal[DC_VOTE] = scal[DC_VOTE + 1];
}

hipError_t launch_dc_finalize(const double *part, int cnt, int j, int with_w, double *scal,
                              const int *stop_col, int col, hipStream_t s) {
    const int nblk = with_w ? 2 * j + 3 : j + 1;
    hipLaunchKernelGGL(k_dc_finalize, dim3(nblk), dim3(NT), 0, s, part, cnt, j, with_w, scal, stop_col, col);
    return hipGetLastError();
}

// Scalar step of DCGS2 step j: one 1024-thread workgroup runs dc_scalar_body (vtk_scalar.hpp)
__global__ __launch_bounds__(1024) void k_dc_scalar(const double *part, int cnt, const double *scal, int j,
                                                    int m, int closing, double *Hraw, double *H,
                                                    double *S, double *giv, DcCoef *cf,
                                                    GmresState *st, int *stop_map) {
    __shared__ DcScalarLds sl;
    dc_scalar_body<false, 3>(sl, part, cnt, scal, j, m, closing, Hraw, H, S, giv, cf, st, stop_map);
}

hipError_t launch_dc_scalar(const double *part, int cnt, const double *scal, int j, int m, int closing,
                            double *Hraw, double *H, double *S, double *giv, DcCoef *cf, GmresState *st,
                            int *stop_map, hipStream_t s) {
    hipLaunchKernelGGL(k_dc_scalar, dim3(1), dim3(1024), 0, s, part, cnt, scal, j, m, closing, Hraw, H, S, giv,
                       cf, st, stop_map);
    return hipGetLastError();
}


// NTPW: p_j and w loaded non-temporal (A/B: +2 % on the unfused (line) path, -1 % after the
// fused BJ step, whose w the update re-reads warm)
template <bool NTPW>
__global__ __launch_bounds__(NT) void k_dc_update(double *__restrict__ V, int64_t ld, int j,
                                                  const double *__restrict__ w, int64_t n,
                                                  const DcCoef *cf, const GmresState *st, double *x,
                                                  const double *H, const double *S, int m) {
    __shared__ double cs[DC_MAXJ], ce[DC_MAXJ + 1];
    __shared__ double rinv_s, q_s;
    if (__builtin_nontemporal_load(&st->xup_tag) == j) {   // the cycle's x update (one basis read less)
        dc_xupdate_body<0>(V, ld, j, __builtin_nontemporal_load(&st->stop_col), n, cf, x, H, S, m, nullptr);
        return;
    }
    if (stopped(&st->stop_col, j)) return;
    for (int k = threadIdx.x; k <= j; k += NT) {
        if (k < j) cs[k] = cf->s[k];
        ce[k] = cf->e[k];
    }
    if (threadIdx.x == 0) { rinv_s = cf->rinv; q_s = cf->q; }
    __syncthreads();
    const double rinv = rinv_s, q = q_s, ej = ce[j];
    double *pj = V + (size_t)j * ld;
    double *pn = V + (size_t)(j + 1) * ld;
    const int64_t stride = 2 * (int64_t)gridDim.x * NT;
    for (int64_t i = 2 * ((int64_t)blockIdx.x * NT + threadIdx.x); i < n; i += stride) {
        if (i + 1 < n) {
            double2 p, t;
            if constexpr (NTPW) {
                const d2v pp = ldnt2(pj + i), tt = ldnt2(w + i);
                p = make_double2(pp.x, pp.y);
                t = make_double2(tt.x, tt.y);
            } else {
                p = *reinterpret_cast<const double2 *>(pj + i);
                t = *reinterpret_cast<const double2 *>(w + i);
            }
            double2 a = p;
            auto acc1 = [&](int k, const d2v &v) {
                const double sk = cs[k], ek = ce[k];
                a.x = a.x - sk * v.x;
                a.y = a.y - sk * v.y;
                t.x = t.x - ek * v.x;
                t.y = t.y - ek * v.y;
            };
            for (int k = 0; k < j; ++k) acc1(k, ldnt2(V + (size_t)k * ld + i));
            double2 vj = p;
            if (j >= 1) {
                vj.x = a.x * rinv;
                vj.y = a.y * rinv;
                st_nt2<2>(pj + i, vj.x, vj.y);
            }
            t.x = t.x - ej * vj.x;
            t.y = t.y - ej * vj.y;
            t.x = t.x * q;
            t.y = t.y * q;
            st_nt2<2>(pn + i, t.x, t.y);
        } else {
            const double p = pj[i];
            double a = p, t = w[i];
            for (int k = 0; k < j; ++k) {
                const double v = V[(size_t)k * ld + i];
                a = a - cs[k] * v;
                t = t - ce[k] * v;
            }
            double vj = p;
            if (j >= 1) { vj = a * rinv; pj[i] = vj; }
            t = t - ej * vj;
            pn[i] = t * q;
        }
    }
}

hipError_t launch_dc_update(double *V, int64_t ld, int j, const double *w, int64_t n, const DcCoef *cf,
                            int grid, const GmresState *st, double *x, const double *H, const double *S, int m,
                            int nt_pw, hipStream_t s) {
    if (nt_pw) hipLaunchKernelGGL((k_dc_update<true>), dim3(grid), dim3(NT), 0, s, V, ld, j, w, n, cf, st, x, H, S, m);
    else hipLaunchKernelGGL((k_dc_update<false>), dim3(grid), dim3(NT), 0, s, V, ld, j, w, n, cf, st, x, H, S, m);
    return hipGetLastError();
}

int vector_grid(int64_t n) {
    int64_t g = (n + 2 * NT - 1) / (2 * NT);
    if (g < 1) g = 1;
    if (g > GMAX) g = GMAX;
    return (int)g;
}



}  // namespace vtk
