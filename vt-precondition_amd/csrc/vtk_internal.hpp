// vtk_internal.hpp — types shared by the C-ABI/driver (vtk_api.cpp, vtk_host.cpp) and the
// gfx950 kernels (vtk_kernels.hip).  Not part of the public ABI.
#pragma once
#include <cmath>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/vtkrylov.h"

namespace vtk {

// ---- kernel geometry -------------------------------------------------------
constexpr int NT = 256;            // threads per workgroup, every vector kernel
constexpr int TILE_ROWS = 512;     // max rows of one SpMV tile (CSR-stream)
constexpr int TILE_NNZ = 4096;     // max nnz of one stream tile: products staged in LDS (32 KB)
constexpr int GMAX = 1024;         // max workgroups of a reducing kernel = partial-sum slots
constexpr int MAX_RESTART = 1024;  // restart length bound (LDS for y in the x update)
constexpr int BIG_COL = 1 << 30;   // "not stopped" marker of GmresState::stop_col

// ---- device-resident solver scalars ---------------------------------------------------------
struct GmresState {
    double ptol;          // inner tolerance of this cycle (host writes before each cycle)
    double presid;        // |S[col+1]| after the last Givens step
    double rnorm;         // ||b - A x|| (finalise)
    double scal[8];       // misc finalised scalars (bnorm, Mb norm, ...)
    int stop_col;         // column at which the cycle stopped (BIG_COL while running)
    int breakdown;        // h1 <= eps*h0 at stop_col
    long long inner;      // inner iterations, cumulative
    int xup_tag;          // DCGS2: the update pass (step tag) that does the cycle's x update
                          // (-1: none, the host-enqueued k_xupdate does it)
    int pad_;
};

// DCGS2 (delayed classical Gram-Schmidt with re-orthogonalisation, one reduction per Arnoldi
// step): per-step coefficients produced by the scalar kernel for the update pass
constexpr int DC_MAXJ = 32;          // restart <= 32 in this mode (4 waves x 8 vectors per lane)
constexpr int DC_NQ = 2 * DC_MAXJ + 3;   // reduction slots: s[32] | z[32] | alpha beta gamma
// across ranks the all-reduced payload carries one more slot, the failure vote (vtk_ctx::d_scal
// [DC_VOTE]; [DC_VOTE + 1] holds this rank's own vote, nonzero once a launch of it failed)
constexpr int DC_VOTE = DC_NQ;
constexpr int DC_NQV = DC_NQ + 1;
constexpr int PEER_FAILED = 2;           // GmresState::breakdown: the vote stopped the cycle
struct DcCoef {
    double s[DC_MAXJ];        // re-orthogonalisation coefficients of the candidate p_j
    double e[DC_MAXJ + 1];    // projection of w on [V_j, v_j]
    double rinv;              // 1 / r_j  (r_j = ||p_j - V_j s||, Pythagorean)
    double q;                 // 1 / (r_j * nu_{j+1})
    double nu;                // tentative h_{j+1,j}
    double h0[DC_MAXJ + 1];   // ||B v_c|| per column (breakdown test, iterative.py:766)
    int committed[DC_MAXJ + 1];   // column already rotated into H (early or exact commit)
    // the previous step's e and q (k_dc_scalar saves them before overwriting): the line-band
    // step recomputes p_j = (w_{j-1} - sum_k e_prev[k] V_k) q_prev instead of storing it
    double e_prev[DC_MAXJ + 1];
    double q_prev;
};

// a reduced scalar as seen by a consumer kernel: G partials (single GPU) or 1 value (after
// the RCCL all-reduce).  Every consumer workgroup sums the partials in the same fixed order.
struct Red {
    const double *p;
    int cnt;
};

// ---- CSR tiles (CSR-stream row blocks) -----------------------------------------------------
struct Tiles {
    int32_t *d_row = nullptr;   // tile t = rows [row[t], row[t+1])
    int32_t *d_end = nullptr;   // optional (split lists): tile t = rows [row[t], end[t])
    int ntiles = 0;
    int align = 1;              // every boundary is a multiple of align (except n_local)
    bool has_long = false;      // some tile is a single row with nnz > TILE_NNZ
    bool aligned = true;        // no align-group had to be split into single-row tiles
    int grid = 0;               // workgroups of the tile kernels = min(ntiles, GMAX)
    int64_t nrows = 0;          // rows covered (split lists: byte accounting)
};

// SELL-64 copy of a CSR (vtk_kernels.hip k_sell): chunk q = local rows 64q..64q+63
struct Sell {
    int64_t *d_off = nullptr;   // [nch+1] entry offsets (multiples of 64)
    int32_t *d_col = nullptr;   // [entries], -1 = padding
    void *d_val = nullptr;      // [entries] f64 (C4: f32)
    int64_t nch = 0, entries = 0;
    // dictionary-coded columns (k_sell_pack): entry k of row 64q+l is the 4-bit code
    // (pk[pk_off[q] + 64*(k/8) + l] >> 4*(k%8)) & 15; code 15 = padding, else
    // col = row + dict[16q + code].  dict[16q + 15] != 0: the chunk has more than
    // PK_CODES distinct (col - row) offsets and reads d_col instead ("wide")
    uint32_t *d_pk = nullptr;
    int64_t *d_pkoff = nullptr;  // [nch+1] word offsets (multiples of 64)
    int32_t *d_dict = nullptr;   // [nch][16]
    int64_t n_wide = 0;          // chunks that kept int32 columns
    int64_t wide_entries = 0;    // their entries (64 per row slot)
    int64_t pk_words = 0;
    int uniform_w = 0;           // every chunk has this width (offsets are 64 W q): no offset loads
};
constexpr int PK_CODES = 15;     // offsets per chunk dictionary (codes 0..14; 15 = padding)

// groups of 4 SELL chunks (256 rows) a SELL launch covers: all (d_list null) or a list
struct Groups {
    int32_t *d_list = nullptr;
    int count = 0;
    int grid = 0;               // workgroups = min(count, GMAX), >= 1
};

// line-Jacobi operator: the tridiagonal systems along x-lines, cut into
// segments of `seg` consecutive line indices i = R / stride (R global) and at the rank's row
// block [row0, row0 + n).  f = [l | m | g] (n doubles each), Thomas factors (vtk_kernels.hip
// k_line_setup; the oracle's orc_line_setup).  Work items: one wavefront per (segment, 64
// consecutive j = R mod stride starting at j0).
struct LineOp {
    double *f = nullptr;
    int64_t n = 0, row0 = 0, stride = 1, seg = 1;
    int64_t i_lo = 0, i_hi = -1;   // line indices of the block's first / last row
    int64_t nseg = 0;              // segments touching the block
    int64_t j0 = 0, jn = 0;        // lanes cover j = j0 .. j0 + jn - 1
    int64_t jb = 0;                // wavefronts per segment = ceil(jn / 64)
    // compact (x-invariant couplings): a_j = ac[j - j0], c_j = ac[jn + j - j0]; the apply forms
    // l = a m_prev and g = c m and reads only m of f (k_line_setup's ext check)
    double *ac = nullptr;
    int compact = 0;
};

// 4D phase-space grid of the Vlasov operators (row = ((ix Ny + iy) Nvx + jvx) Nvy + jvy, x and y
// periodic, vx and vy Dirichlet): every row couples to x +- 1 (value by jvx),
// y +- 1 (by jvy), vx +- 1 (by ix), vy +- 1 (by iy) and itself, in ascending column order.  When
// vtk_csr_set_grid4 / the Vlasov assembly / the drop-in detection verified that (bit for bit),
// the solver's SELL launches take each row's columns from its coordinates and its values from
// D[n] (the stored value type) and the per-coordinate tables: 4 B of matrix per row (C4) instead
// of 9 values and 9 codes.  X = local x planes; lblk: across ranks the halo block holding the
// left x neighbour plane (-1: one rank, x periodic inside the slab).
struct Grid4 {
    int Ny = 0, Nvx = 0, Nvy = 0, X = 0;
    int lblk = -1;
    // across ranks, where the halo planes' columns sit in a row's stored (global column) order:
    // bit 0: the left plane's after the row (the slab starts at plane 0: its left is the last
    // plane), bit 1: the right plane's before it (the slab ends at the last plane)
    int xord = 0;
    const double *tab = nullptr;   // TX[2][Nvx] | TY[2][Nvy] | TVX[2][X] | TVY[2][Ny] (-, + each)
    const void *D = nullptr;       // diagonal per row, the operator's value type
};
inline size_t grid4_tab_len(const Grid4 &g) { return 2 * ((size_t)g.Nvx + g.Nvy + g.X + g.Ny); }
// k_g4_ring's limits (vtk_band.hip): the LDS table TX | TY | TVX | TVY of <= G4TAB doubles and a
// ring of <= 8192 doubles holding the y-line window 2 S3 plus two groups of rows (512 per group for
// gr >= 512 outside the fused-dots mode 1, else 256).  The solver takes the ring step only for grids
// that fit (else the SELL grid-row kernels); launch_g4_ring refuses the others
constexpr int G4TAB = 1024;
constexpr int G4RM = 64;   // k_g4_ring: mirrored slots at each end of the x ring (> Nvy)
inline int g4_ring_group(int gr) { return gr >= 512 ? 512 : 256; }
// groups per workgroup of a k_g4_ring launch over ng groups of G rows for ~wgs workgroups,
// XCD-aligned: a workgroup's x -+ 1 plane rows belong to the workgroups q = S4 / (per G) indices
// away; per is rounded so that q is a multiple of 8, which puts them on the same XCD (workgroups
// are dealt round-robin over the eight XCDs) -- those reads hit its L2 (C4: per 48 -> 31, ring
// 384 -> 369 us)
// (only where a plane spans >= 8 groups and q would stay <= 32: with a few groups per
// workgroup the rounding cannot hold q near a multiple of 8)
inline int64_t g4_ring_per(int64_t ng, int64_t S4, int G, int wgs) {
    const int64_t per0 = std::max<int64_t>(1, (ng + std::max(1, wgs) - 1) / std::max(1, wgs));
    const double gpp = (double)S4 / G;   // groups per x-plane
    if (gpp < 8.0 || gpp / (double)per0 > 32.0) return per0;
    const int64_t q = std::max<int64_t>(8, (int64_t)std::ceil(gpp / (double)per0 / 8.0) * 8);
    return std::max<int64_t>(1, std::llround(gpp / (double)q));
}
inline bool g4_ring_fits(const Grid4 &g, int64_t n, int gr) {
    const int64_t S3 = (int64_t)g.Nvx * g.Nvy;
    return n > 0 && n <= INT32_MAX / 2 && 2 * S3 + 2 * g4_ring_group(gr) <= 8192 && grid4_tab_len(g) <= (size_t)G4TAB &&
           g.Nvy < G4RM;
}

// Tuning switches of a context (vtk_ctx_set_tuning): the defaults are the
// production path, the others exist for in-process A/B measurements and the bit-identity tests
// (the same sums with and without a byte-saving form).  Initialised from VTK_<KEY> (upper case)
// once, at vtk_ctx_create -- never read per launch.
struct Tuning {
    int band = 1;             // line-band DCGS2 step allowed (vtk_gmres_set_band)
    int band_lsv = 1;         // solver launches read the line-separable values (else SELL values)
    int sell_canon = 1;       // ... and canonical rows' columns from the line index (no codes)
    int band_canon = 1;       // the band step reads no codes on canonical rows
    int band_opt = 31;        // band step variant bits (vtk_band.hip k_band_step OPT; in-process A/B
                              // C3: SpMV operands prefetched j00 254 -> 217 us, + three workgroups per
                              // CU for j <= BAND_J3: j00 190, j01 283 -> 246 us; solve 42.66 -> 42.31 ms;
                              // round 6: bit 2, a line range's two parts on one XCD: 40.56 -> 40.30 ms;
                              // bit 3, LDS-DMA L2 prefetch for J > BAND_PF: j13-j18 -21..-50 us each;
                              // bit 4, odd line ranges walk backwards: 39.98 -> 39.81 ms, C3/8 slab
                              // 6.652 vs 6.676 ms (neutral).  Since round 6 also across ranks)
    int band_long_rows = 16000000;   // band_opt bits 3 and 4 only on basis vectors of >= this many rows
                              // (in-process A/B, round 6: bit 3 on vs off, C3 20M rows 39.30 vs 39.78 ms,
                              // C3/2 slab 10M 20.20 vs 20.09, C2 5M 10.98 vs 10.86, C3/8 slab 2.5M 6.53
                              // vs 6.51; bit 4 on vs off, C3 39.24 vs 39.34, C3/2 20.13 vs 20.00, C3/4
                              // 11.02 vs 10.95, C2 10.92 vs 10.87)
    int lsv_ring = 2048;      // > 0: the line path's table SpMV with x staged through LDS, ~that many
                              // workgroups (in-process A/B, C3 line solve: 8.64 -> 8.26 ms; 167 -> 105 us)
    int prof_perj = 0;        // profile class per band step index (band_step_jNN)
    int comm_solo = 0;        // vtk_comm_init with world 1 builds a one-rank RCCL communicator
    int auto_band = 1;        // vtk_csr_create detects the line band and the 4D grid (drop-in path)
    int grid4 = 1;            // solver launches read 4D grid rows from their coordinates (Grid4)
    int c4_fused = 1;         // with grid4 and no ring: the DCGS2 dots fused into the 9-wide SELL step
    int g4_ring = 2048;       // > 0: the split step's SpMV + BJ of grid rows with x staged through LDS
                              // (k_g4_ring, ~that many workgroups), step 0's dots and the cycle-start
                              // residual in it too; takes precedence over c4_fused
    int g4_gr = 512;          // k_g4_ring: rows per group = lanes per workgroup (256 | 512)
    int g4_fast = 1;          // (A/B) k_g4_ring's straight-line sum for waves of inner rows
    int line_fuse = 1;        // line path (one rank, canonical rows): the SpMV inside the sweep kernel
    int cyc_ring = 512;       // > 0: cycle-start residual and DCGS2 step 0 through the x-line ring
                              // (k_lsv_ring_epi, ~that many workgroups; 2D line-separable rows)
    int fail_step = -1;       // (test hook) >= 0: this rank's DCGS2 step of that index fails in the
                              // first cycle as a refused launch would (the peer-failure vote, vtk_gmres)
};
}  // namespace vtk

struct vtk_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t comm_stream = nullptr;    // halo exchange overlapped with interior tiles
    hipEvent_t ev_pack = nullptr, ev_halo = nullptr;
    std::string err;
    int rank = 0, world = 1;
    bool dist = false;                    // distributed code paths: world > 1, or a one-rank
                                          // RCCL communicator (VTK_COMM_SOLO=1, testing)
    ncclComm_t comm = nullptr;            // RCCL (production transport)
    bool host_comm = false;               // host-staged hooks (vtk_comm_init_host)
    bool comm_broken = false;             // an RCCL call failed: vtk_ctx_destroy aborts the communicator
    vtk_host_comm hops{};
    int orth = VTK_ORTH_AUTO;
    vtk::Tuning tune;                     // A/B switches (vtk_ctx_set_tuning), env at creation
    int n_cu = 0;                         // compute units (band step grid)
    // scratch shared by calls on this context
    double *d_part = nullptr;        // [8][GMAX] partial sums
    double *d_scal = nullptr;        // [256] reduced scalars (all-reduce slots)
    vtk::GmresState *d_state = nullptr;
    vtk::GmresState *h_state = nullptr;   // pinned mirror
    int *h_stop = nullptr;                // pinned, device-mapped: k_tail writes the stop column
    int *d_stop = nullptr;                // device alias of h_stop
    void *ws = nullptr;                   // solver workspace (grow-only, reused across solves)
    size_t ws_bytes = 0;
    // kernel profile (vtk_profile_enable)
    struct ProfPending { int cls; int col; double bytes; hipEvent_t e0, e1; };
    struct ProfAcc { std::string name; int64_t launches = 0; double seconds = 0, bytes = 0; };
    bool prof_on = false;
    std::vector<ProfPending> prof_pending;
    std::vector<ProfAcc> prof_acc;
    std::vector<hipEvent_t> prof_pool;
};

struct vtk_csr {
    vtk_ctx *ctx = nullptr;
    int device = 0;   // the context's device: destroy never dereferences ctx (it may be gone)
    int64_t n_global = 0, row_begin = 0, row_end = 0, n_local = 0, nnz = 0;
    int fp32 = 0;
    int32_t *d_indptr = nullptr, *d_indices = nullptr;  // local column indices
    void *d_data = nullptr;
    std::vector<int32_t> h_indptr;                      // host copy (tile planning)
    std::vector<uint8_t> row_halo;                      // world > 1: row reads a halo column
    // SELL-64 layout (vtk_csr_set_layout): built when its padding is small (AUTO) or asked for
    vtk::Sell sell;
    bool use_sell = false;
    int layout = VTK_LAYOUT_AUTO;
    vtk::Groups g_all, g_in, g_bd;                      // g_in/g_bd: world > 1 (halo overlap)
    std::vector<int64_t> offsets;                       // partition, world+1
    vtk::Tiles tiles;                                   // align 1
    // halo (world > 1)
    int64_t n_halo = 0;
    std::vector<int64_t> halo_cols;                     // global ids, ascending
    std::vector<int64_t> recv_cnt, recv_off;            // per rank, into d_halo
    std::vector<int64_t> send_cnt, send_off;            // per rank, into d_send_buf
    double *d_halo = nullptr;
    int32_t *d_send_idx = nullptr;                      // local rows to pack
    double *d_send_buf = nullptr;
    int64_t n_send = 0;
    int64_t band_L = 0;                                 // line-band structure (vtk_csr_set_line_band)
    bool band_vloc = false;                             // ... with every column within v-1..v+1 of its row
    // line-separable values (k_lsv_build): every coupling to line x+-1 depends
    // only on the position v (table TX[2][L]), every coupling to v+-1 in the same line only on
    // the line x (TV[2][X]), the diagonal per row (D[n]) -- verified bit-exactly against the CSR
    // when the band is set; the band step then reads 8 B of values per row instead of 40.
    // d_lsv = D | TX | TV; null: not separable (the band step reads the SELL values)
    double *d_lsv = nullptr;
    bool lsv_canon = false;   // ... and every row canonical (canon_order): the band step reads no codes
    // 4D grid structure (vtk::Grid4; tables owned here); g4_dims = 0: not set
    vtk::Grid4 g4;
    double *d_g4tab = nullptr;
    void *d_g4D = nullptr;
    // distributed band step: the halo is two neighbour lines; peers and the alltoallv layout of
    // the per-step ghost exchange (BAND_GHOST_VECS L doubles per side), -1 offsets: no such side
    bool band_ghost = false;                            // band across ranks: per-step ghost exchange
    int band_lblk = 0;
    int band_xord = 0;                                  // bit 0: slab starts at global line 0, bit 1: ends at the last line
    int band_peer[2] = {-1, -1};                        // left, right neighbour rank
    std::vector<int64_t> band_scnt, band_soff, band_rcnt, band_roff;
    int64_t band_off_first = -1, band_off_last = -1;    // send offsets of the first / last line
    int64_t band_off_left = -1, band_off_right = -1;    // recv offsets of the left / right ghost
};

struct vtk_prec {
    vtk_csr *A = nullptr;
    int device = 0;   // destroy never dereferences A (a finaliser may have freed it first)
    int bs = 8;
    int64_t nb = 0;
    double *d_inv = nullptr;     // [nb][bs][bs]
    vtk::Tiles tiles;            // aligned to bs (fused SpMV + BJ)
    bool fused = false;          // fused SpMV+BJ kernel usable
    // world > 1, fused: the same tiles split into interior (no halo column: run while the halo
    // exchange is in flight) and boundary tiles (after it lands)
    vtk::Tiles tiles_in, tiles_bd;
    bool split = false;
    // tridiagonal blocks: LU factors l | m | g (SoA, stride tri_ld = nb * bs), vtk_bj_mode
    double *d_tri = nullptr;
    int64_t tri_ld = 0;
    bool tri_ok = false;
    int mode = VTK_BJ_AUTO;
    // line Jacobi (vtk_linejacobi_create): kind VTK_PREC_LINE, factors in line.f
    int kind = VTK_PREC_BJACOBI;
    vtk::LineOp line;
    bool line_compact_ok = false;   // x-invariant couplings found at setup (line.ac valid)
};

namespace vtk {

// ---- kernel launchers (vtk_kernels.hip) ------------------------------------------------------
struct SpmvIn {
    const int32_t *indptr, *indices;
    const void *data;
    int fp32;
    const Tiles *tiles;       // CSR-stream tiles (used when sell/groups are null)
    int n_local;
    const double *x, *halo;   // halo may be null (world == 1)
    const Sell *sell = nullptr;
    const Groups *groups = nullptr;
    // line-separable values (SELL, f64; solver launches only -- vtk_spmv keeps the SELL values)
    const double *lsv = nullptr;
    int lsv_L = 0, lsv_lblk = -1;
    int lsv_xord = 0;    // across ranks: the halo lines' place in the stored order (vtk_csr::band_xord)
    int lsv_canon = 0;   // ... and every row canonical: k_sell computes the columns (canon_row)
    int plain_grid = 0;  // workgroups of the plain SELL SpMV (0: 2 GMAX)
    Grid4 g4{};          // 4D grid rows (solver launches; g4.tab null: not used)
    int swz = 0;         // XCD-aware SELL group order: bit 0 the plain SpMV, bit 1 the other epilogues
    int plain_var = 0;   // plain SELL SpMV variant bits (k_sell VAR)
};

LineOp line_plan(int64_t n, int64_t row0, int64_t stride, int64_t seg);

// block-Jacobi operator as the kernels see it: inverse rows f64[nb][bs][bs], or (tri != null)
// the LU factors of tridiagonal blocks, SoA l | m | g with stride tri_ld (vtk_api.cpp, BJ
// modes).  bs == 0: identity.
struct BjOp {
    const double *inv = nullptr;
    const double *tri = nullptr;
    int64_t tri_ld = 0;
    int bs = 0;
    const LineOp *line = nullptr;   // line Jacobi instead (inv/tri unused)
};

// mm[0] = min, mm[1] = max of idx[0..n) (mm preset to INT_MAX, INT_MIN)
hipError_t launch_index_range(const int32_t *idx, int64_t n, int *mm, hipStream_t s);

// workgroups (= partials) of a launch on this input
inline int spmv_grid(const SpmvIn &in) { return (in.sell && in.groups) ? in.groups->grid : in.tiles->grid; }

// EPI_PREC_DC: w = M^-1 A p_j plus the DCGS2 step's dot products (launch_spmv_dc)
enum Epi { EPI_PLAIN = 0, EPI_RESID = 1, EPI_PREC = 2, EPI_RESID_PREC = 3, EPI_PREC_DC = 4 };

// y = A x (PLAIN); y = b - A x, part0 = sum y^2 (RESID); y = M^-1 A x with M = BJ(inv, bs)
// or identity (inv == null), part0 = sum y^2, part1 = sum v0*y (PREC, v0 may be null);
// RESID_PREC: r = b - A x, y = M^-1 r, part0 = sum r^2, part1 = sum y^2.
hipError_t launch_spmv(const SpmvIn &in, int epi, double *y, const double *b, const BjOp &bj,
                       const double *v0, double *part0, double *part1,
                       const int *stop_col, int col, hipStream_t s);
// z = M^-1 r (BJ or identity when inv == null); part0 = sum z^2, part1 = sum v0*z (optional)
hipError_t launch_bj_apply(const BjOp &bj, int64_t n, const double *r, double *z,
                           const double *v0, double *part0, double *part1, int grid,
                           const int *stop_col, int col, hipStream_t s);
// factors of tridiagonal diagonal blocks (bs in {2, 4, 8}): tri[i] = l_i, tri[ld + i] = m_i = 1/u_i,
// tri[2 ld + i] = g_i = sup_i m_i (Thomas, no pivoting); *flags |= 1 a block is not tridiagonal,
// 2 a pivot is tiny, 4 the factors disagree with the Gauss-Jordan inverse beyond 1e-10
// SELL-64 build: phase 0 = chunk widths + scan into off (scan_tmp of sell_scan_bytes(n),
// tmp64 of nch+1 int64), phase 1 = fill col/val
hipError_t launch_sell_build(const int32_t *indptr, const int32_t *indices, const void *data, int fp32, int64_t n,
                             int64_t *off, int64_t *tmp64, void *scan_tmp, size_t scan_bytes, int32_t *col,
                             void *val, int phase, hipStream_t s);
size_t sell_scan_bytes(int64_t n);
// dictionary-coded columns of a built SELL: phase 0 = word offsets + scan into pkoff (tmp64
// [nch+1], scan_tmp as above), phase 1 = codes + dictionaries, n_wide counted into *wide_cnt
hipError_t launch_sell_pack(const int64_t *off, int64_t nch, int64_t *pkoff, int64_t *tmp64, void *scan_tmp,
                            size_t scan_bytes, const int32_t *col, uint32_t *pk, int32_t *dict,
                            unsigned long long *wide_cnt, int phase, hipStream_t s);
// line Jacobi: factors (flags: *bad_row = min global row with a zero / non-finite pivot; ext:
// 4 jn words, per line min/max bit patterns of the a's and c's, init ~0 / 0 / ~0 / 0) and
// z = M^-1 r with part0 = sum z^2, part1 = sum v0*z (optional) over `grid` workgroups
hipError_t launch_line_setup(const int32_t *indptr, const int32_t *indices, const void *data, int fp32,
                             const LineOp &L, unsigned long long *bad_row, unsigned long long *ext, hipStream_t s);
// z = M_line^-1 r fused with DCGS2 step j's dots (p = the SpMV input, partials in the
// launch_dc_dots layout); hipErrorInvalidValue when the segments are too long (> 32)
hipError_t launch_line_dc(const LineOp &L, const double *r, double *w, const double *V, int64_t ld, int j,
                          const double *p, double *part, int grid, const int *stop_col, int col, hipStream_t s);
// the same with y = A p formed inside (k_line_spmv_dc): one rank, canonical line-separable rows
// (lsv: vtk_csr::d_lsv), lines of L.stride rows, compact factors; hipErrorInvalidValue otherwise
hipError_t launch_line_spmv_dc(const LineOp &L, const double *lsv, const double *p, double *w, const double *V,
                               int64_t ld, int j, double *part, int grid, const int *stop_col, int col, hipStream_t s);
hipError_t launch_line_apply(const LineOp &L, const double *r, double *z, const double *v0, double *part0,
                             double *part1, int grid, const int *stop_col, int col, hipStream_t s);
hipError_t launch_bj_tri_setup(const int32_t *indptr, const int32_t *indices, const void *data, int fp32,
                               int64_t n, int bs, const double *inv, double *tri, int64_t ld, int *flags,
                               hipStream_t s);
hipError_t launch_bj_setup(const int32_t *indptr, const int32_t *indices, const void *data,
                           int fp32, int64_t n, int bs, double *inv, int *d_singular,
                           double *work, hipStream_t s);
// the same inverses for bs 16 / 32 by blocked Gauss-Jordan on the matrix cores (k_bj_setup_mfma;
// agrees with launch_bj_setup to rounding, not bit for bit)
hipError_t launch_bj_setup_mfma(const int32_t *indptr, const int32_t *indices, const void *data, int fp32, int64_t n,
                                int bs, double *inv, int *d_singular, hipStream_t s);
// w -= h v_k with h = reduce(hin); part_out = sum v_next*w (or sum w^2 if v_next == null)
hipError_t launch_mgs(Red hin, double *hout, double *w, const double *vk, const double *vnext,
                      int64_t n, double *part_out, int grid, const int *stop_col, int col,
                      hipStream_t s);
// h0 = sqrt(reduce(h0)), h1 = sqrt(reduce(w2)); v_next = w * (1/h1) (w if breakdown);
// workgroup 0 applies the Givens rotations to column col of H and sets the stop flag.
hipError_t launch_tail(Red h0, Red w2, const double *w, double *vnext, int64_t n, int col,
                       int m, double *H, double *S, double *giv, GmresState *st, int *stop_map,
                       int grid, hipStream_t s);
// v0 = v0 * (1/t), t = sqrt(reduce(p)); S[0] = t, S[1..m] = 0, stop_col = BIG_COL
hipError_t launch_scale0(Red p, double *v0, int64_t n, double *S, int m, GmresState *st,
                         int grid, hipStream_t s);
// y = triangular solve (H, S) at stop column; x += y @ V
// (returns at entry when a DCGS2 update pass already did it: st->xup_tag >= 0)
hipError_t launch_xupdate(const double *H, const double *S, const double *V, int64_t ld,
                          double *x, int64_t n, int m, const GmresState *st, int grid, hipStream_t s);
// dst = sqrt(reduce(p)) if do_sqrt else reduce(p)   (single workgroup)
hipError_t launch_finalize(Red p, double *dst, int do_sqrt, hipStream_t s);
// part = sum x^2 (or x*y)
hipError_t launch_dot(const double *x, const double *y, int64_t n, double *part, int grid,
                      hipStream_t s);
// *flag = 1.0 when some x[i] != 0 (zeroed by the caller)
hipError_t launch_any_nonzero(const double *x, int64_t n, double *flag, hipStream_t s);
hipError_t launch_gather(const double *x, const int32_t *idx, int64_t cnt, double *out,
                         hipStream_t s);
// device operator assembly
hipError_t launch_vlasov_counts(const vtk_vlasov_params &p, int64_t r0, int64_t nrows,
                                int32_t *counts, hipStream_t s);
hipError_t launch_vlasov_fill(const vtk_vlasov_params &p, int64_t r0, int64_t nrows,
                              const int32_t *indptr, int32_t *indices, void *data,
                              hipStream_t s);
hipError_t launch_exclusive_scan(const int32_t *in, int32_t *out, int64_t n, void *tmp,
                                 size_t *tmp_bytes, hipStream_t s);
hipError_t launch_remap_cols(int32_t *indices, int64_t nnz, int64_t row_begin, int64_t n_local,
                             const int64_t *halo_cols, int64_t n_halo, hipStream_t s);

// DCGS2: dots pass (s = V_j^T p_j, z = V_j^T w, alpha, beta, gamma; w == null: s, alpha only),
// per-quantity finalize (one workgroup per quantity), single-lane scalar step, update pass.
hipError_t launch_dc_dots(const double *V, int64_t ld, int j, const double *w, int64_t n,
                          double *part, int grid, const int *stop_col, int col, hipStream_t s);
// DCGS2 step j fused into the SpMV: w = M^-1 A p_j with p_j = V[j] (in.x), and per workgroup
// the partials of s = V_j^T p_j, z = V_j^T w, |p|^2, p.w, |w|^2 (layout of launch_dc_dots);
// grid = tiles->grid partials.  BJ-fused tiles with bs in {1, 2, 4, 8} only.
hipError_t launch_spmv_dc(const SpmvIn &in, double *w, const BjOp &bj, const double *V,
                          int64_t ld, int j, double *part, const int *stop_col, int col, hipStream_t s);
hipError_t launch_dc_finalize(const double *part, int cnt, int j, int with_w, double *scal,
                              const int *stop_col, int col, hipStream_t s);
// part != null: reduce the G partials in-kernel (one GPU); else read the all-reduced scal
hipError_t launch_dc_scalar(const double *part, int cnt, const double *scal, int j, int m,
                            int closing, double *Hraw, double *H, double *S, double *giv,
                            DcCoef *cf, GmresState *st, int *stop_map, hipStream_t s);
// update pass of step j; when the step's scalar kernel stopped the cycle (st->xup_tag == j) it
// does the cycle's x update instead: x += V[0..c] y, y = H^-1 S at c = stop_col (j-1 or j; for
// c = j the v_j of the pass is formed in registers), reading the basis once
hipError_t launch_dc_update(double *V, int64_t ld, int j, const double *w, int64_t n,
                            const DcCoef *cf, int grid, const GmresState *st, double *x,
                            const double *H, const double *S, int m, int nt_pw, hipStream_t s);

// Line-band DCGS2 step (k_band_step): update pass of step j + SpMV, tridiagonal
// BJ(8) and dots of step j+1 in one sweep over x-lines of L rows (SELL-64 uniform width 5, coded
// columns, fp64 values; across ranks through the ghost lines).  grid workgroups (<= X lines, <= GMAX), partials of step j+1 in
// the launch_dc_dots layout.  p_j is recomputed from w_{j-1} (w_prev) and stored only for
// j + 1 = m - 1 (k_dc_update's operand); w rotates over three buffers.
struct BandK {
    const uint32_t *pk;
    const int32_t *dict;
    const double *val;
    const double *mtri;
    double *V;
    int64_t ld;
    int j, m;
    const double *w_in;          // w_j
    const double *w_prev;        // w_{j-1} (unused at j = 0)
    double *w_out;               // w_{j+1}
    const DcCoef *cf;
    const GmresState *st;
    double *x;
    const double *H, *S;
    double *part;
    int64_t n;
    int L, X, H_parts;           // line length, lines, parts per line (grid = ranges x H_parts)
    const double *ghost;         // distributed: [2][m+2][L] the left / right neighbour lines'
                                 // v_k (k < j) and w_j, w_{j-1} by parity in slots m, m+1
                                 // (k_ghost_unpack); null on one rank
    int left_blk;                // halo block (0 / 1) holding the left neighbour line
    int xord = 0;                // bit 0: the slab starts at global line 0, bit 1: ends at the last line
    const double *lsv;           // line-separable values (vtk_csr::d_lsv) or null: SELL values
    int canon;                   // with lsv: canonical rows (vtk_csr::lsv_canon), no codes read;
                                 // 2: the SpMV as straight-line code per line order
    int opt = 0;                 // kernel variant bits (vtk::Tuning::band_opt; vtk_band.hip OPT)
};
hipError_t launch_band_step(const BandK &a, int grid, int wu, hipStream_t s);
// geometry (k_band_step): a workgroup of BAND_T threads owns <= BAND_LP rows of a
// line (one part; parts per line = band_parts), BAND_WPC workgroups per CU (LDS-bound)
constexpr int BAND_LP = 400, BAND_T = 448, BAND_WPC = 2;
constexpr int BAND_JV = 19;    // basis vectors staged per line (j + 1 <= 19: restart <= 20)
// band steps j <= BAND_J3 run three workgroups per CU (Tuning::band_opt bit 1): their LDS (ring +
// (j + 1) staged basis rows of BAND_LP doubles) fits three times into 160 KB, and their registers
// the 80-VGPR cap (j = 3 / 4 fit too since the x update is inline, but measured within noise)
constexpr int BAND_J3 = 2;
// vectors per ghost line and step of the distributed band step: v_{j-1} (v_0 at j = 0), w_j
constexpr int BAND_GHOST_VECS = 2;
hipError_t launch_band_check_dist(const int32_t *indptr, const int32_t *indices, int64_t n, int L, int lblk, int *bad,
                                  hipStream_t s);
hipError_t launch_ghost_pack(const double *V, int64_t ld, int j, const double *w, int64_t n, int L, double *sbuf,
                             int64_t off_first, int64_t off_last, hipStream_t s);
hipError_t launch_ghost_unpack(const double *rbuf, int64_t off_left, int64_t off_right, int j, int m, int L,
                               double *ghost, hipStream_t s);
int band_parts(int64_t L, int lp = BAND_LP);   // parts per line (rows per part <= lp, multiple of 8); 0: none (vtk_host.cpp)
// *bad |= 1 when some column is outside the lines x-1..x+1 (mod X) of its row, |= 2 when one is
// more than one row off its row's position in the line (bad zeroed by the caller)
// line-separable values (vtk_csr::d_lsv): build D | TX | TV from the CSR, then *bad |= 1 when
// some entry is not reproduced bit-exactly (or is no diagonal / v+-1 / same-position x+-1
// coupling).  lblk < 0: one rank (x couplings periodic); else the halo block of the left line
hipError_t launch_lsv_build(const int32_t *indptr, const int32_t *indices, const double *data, int64_t n, int L,
                            int lblk, int xord, double *lsv, int *bad, hipStream_t s);
// y = A x from the line-separable tables and the SELL codes (uniform width 5, coded columns):
// k_sell's plain SpMV, the same bits.  halo != null: the distributed layout (lblk the left block)
// the x-line ring SpMV with the solver's epilogues (one rank, canonical rows; k_lsv_ring_epi):
// EPI_RESID (y = b - A x, p0 = |r|^2 partials), EPI_RESID_PREC (y = M^-1 (b - A x), p0, p1 =
// |r|^2, |z|^2), EPI_PREC_DC (y = M^-1 A x, DCGS2 step-0 dots |x|^2, x.y, |y|^2 into dcpart);
// *grid_out partials (<= GMAX)
hipError_t launch_lsv_ring_epi(int epi, const double *lsv, const double *x, const double *b, const double *mtri,
                               double *y, double *p0, double *p1, double *dcpart, int64_t n, int L, int ring_wgs,
                               const int *stop_col, int col, int *grid_out, hipStream_t s, const double *halo = nullptr,
                               int lblk = -1, int xord = 0);   // halo: across ranks, the two neighbour lines
hipError_t launch_lsv_spmv(const uint32_t *pk, const int32_t *dict, const double *lsv, const double *x,
                           const double *halo, double *y, int64_t n, int L, int lblk, const int *stop_col, int col,
                           hipStream_t s, int canon, int grid_cap,
                           int ring_wgs = 0, int xord = 0);   // canon: rows canonical, no codes read; ring_wgs > 0: LDS-staged x
                                                // (k_lsv_ring, about that many workgroups; one rank, canon)
// 4D grid tables (vtk::Grid4) from the CSR (pass 0) and the check (pass 1): *bad |= 1 when an entry
// is no grid coupling or differs from its table value, |= 2 when a row is not in ascending
// canonical order; D and tab written here
hipError_t launch_grid4_build(const int32_t *indptr, const int32_t *indices, const void *data, int fp32, int64_t n,
                              const Grid4 &g, double *tab, void *D, int *bad, hipStream_t s);
// w = M^-1 A x for 4D grid rows with x staged through LDS (k_g4_ring): the tridiagonal BJ(8) of
// m = mtri; about wgs workgroups, each a contiguous range of 256-row groups; halo != null: across
// ranks (g.lblk the left plane's halo block).  Bit-identical to the SELL launch.  dots != null:
// DCGS2 step 0's dots (mode 2: |p|^2, p.w, |w|^2) or the cycle-start residual (mode 3, w = M^-1
// (b - A x)); partials per workgroup (at most GMAX workgroups, the count in *grid_out).
struct G4Dots {
    int mode = 2;                  // 2: step 0's dots; 3: cycle-start residual
    double *part = nullptr;        // mode 2: the dots partials (launch_dc_dots' layout)
    const double *b = nullptr;     // mode 3: the right-hand side; |r|^2, |w|^2 partials
    double *p0 = nullptr, *p1 = nullptr;
    int part_off = 0;              // the launch's first partial slot (split launches side by side)
};
// g_lo, g_hi: the group range (GR-row groups; -1: all), per: groups per workgroup (0: from wgs)
hipError_t launch_g4_ring(const Grid4 &g, const double *x, const double *halo, const double *mtri, double *w, int64_t n,
                          int fp32, int wgs, int gr, const G4Dots *dots, int *grid_out, const int *stop_col,
                          int col, hipStream_t s, int g_lo = 0, int g_hi = -1, int per = 0, int fast = 1);
hipError_t launch_band_check(const int32_t *indptr, const int32_t *indices, int64_t n, int L, int X, int *bad,
                             hipStream_t s);

int vector_grid(int64_t n);

// ---- host helpers (vtk_host.cpp) -------------------------------------------------------------
void build_tiles(const std::vector<int32_t> &indptr, int align, std::vector<int32_t> &rows,
                 bool &has_long, bool &aligned);
void set_context_free_error(const std::string &msg);

}  // namespace vtk
