/* vtkrylov.h — C-ABI of libvtkrylov.so, the MI355X-native preconditioned-Krylov path.
 *
 * Boundary.  jwang1x/VT-precondition has no solver, no FFI and no plugin
 * interface (the reference is Python provisioning scripts only).  The
 * entry points below replace the calls the north_star's "reference scipy.sparse path"
 * makes — the reference-side binding a maintainer adds is the ctypes stub in
 * INTEGRATION.md (vtkrylov/_abi.py in this repo) — and each declaration names the SciPy
 * interface it stands in for:
 *   vtk_csr_create      <- scipy.sparse.csr_matrix((data, indices, indptr), shape)
 *                          (scipy/sparse/_compressed.py _cs_matrix.__init__)
 *   vtk_spmv            <- csr_matrix @ x -> _matmul_vector (scipy/sparse/_compressed.py:518-530)
 *   vtk_bjacobi_create  <- numpy.linalg.inv on the bs x bs diagonal blocks
 *   vtk_bjacobi_apply   <- LinearOperator(matvec=einsum('bij,bj->bi'))
 *   vtk_linejacobi_*    <- LinearOperator(matvec=splu(M).solve), M = diagonal + x-line
 *                          couplings (line-implicit x-direction solve)
 *   vtk_gmres           <- scipy.sparse.linalg.gmres(A, b, x0, rtol=, atol=, restart=,
 *                          maxiter=, M=) (scipy/sparse/linalg/_isolve/iterative.py:582-841)
 * The config/entry layer the reference does have (XML node lookups, ini_info.py:72-118;
 * step objects with main(), hypervisor.py:589-594) is mirrored in Python by
 * vt-precondition_amd/vtconfig + vtsetup, which call this ABI through ctypes.
 *
 * Conventions: every int-returning function returns VTK_OK (0) or a negative vtk_status;
 * nothing throws or aborts across the boundary; vtk_last_error() explains the last failure
 * of a context (vtk_last_error(NULL, ...) the last failure of a context-free call).
 * Handles are opaque, owned by the caller, freed by the matching *_destroy.  Host arrays
 * passed in stay owned by the caller (they are copied).  A handle is not thread-safe:
 * one context per thread and device, one rank per process.
 */
#ifndef VTKRYLOV_H
#define VTKRYLOV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VTK_ABI_VERSION 6   /* 6: VTK_ERR_PEER, vtk_precond_matvec */

typedef struct vtk_ctx vtk_ctx;
typedef struct vtk_csr vtk_csr;
typedef struct vtk_prec vtk_prec;

typedef enum {
    VTK_OK = 0,
    VTK_ERR_ARG = -1,       /* bad argument / shape / index                        */
    VTK_ERR_HIP = -2,       /* HIP runtime error                                   */
    VTK_ERR_RCCL = -3,      /* RCCL error                                          */
    VTK_ERR_SINGULAR = -4,  /* singular diagonal block (numpy.linalg.LinAlgError)  */
    VTK_ERR_NOMEM = -5,     /* host or device allocation failed                    */
    VTK_ERR_STATE = -6,     /* call not valid in this state (e.g. comm not set)    */
    VTK_ERR_NODEVICE = -7,  /* no HIP device: the product has no CPU fallback      */
    VTK_ERR_PEER = -8       /* another rank failed mid-solve; this rank left the   */
                            /* solve at the same Arnoldi step (vtk_gmres)          */
} vtk_status;

typedef enum { VTK_PTR_HOST = 0, VTK_PTR_DEVICE = 1 } vtk_ptr_kind;

typedef enum {
    VTK_ORTH_MGS = 0,   /* modified Gram-Schmidt, SciPy's sequence (iterative.py:755-759):
                           j+2 dependent reductions per Arnoldi step                        */
    VTK_ORTH_DCGS2 = 1, /* delayed classical GS with re-orthogonalisation: ONE reduction and
                           two passes over the basis per step; restart <= 32                */
    VTK_ORTH_AUTO = 2   /* default: DCGS2 when restart <= 32, else MGS (stats.orth reports) */
} vtk_orth;

/* How the block-Jacobi preconditioner is applied (same M^-1 either way):                   */
typedef enum {
    VTK_BJ_AUTO = 0,    /* default: TRIDIAG when available, else INVERSE                      */
    VTK_BJ_INVERSE = 1, /* z_b = inv_b r_b, serial row dots: bit-identical to the oracle      */
    VTK_BJ_TRIDIAG = 2  /* every diagonal block tridiagonal (bs 2/4/8): LU factors, 24 B/row
                           instead of 8 bs B/row; equal to INVERSE to rounding (factors are
                           checked against the inverse to 1e-10 at setup)                    */
} vtk_bj_mode;

/* Device layout of a CSR operator's SpMV (results are bit-identical in both: every row is
 * summed serially in stored order, as csr_matvec does):                                     */
typedef enum {
    VTK_LAYOUT_AUTO = 0, /* default: SELL when its padding is <= 25 % of nnz, else CSR        */
    VTK_LAYOUT_CSR = 1,  /* CSR-stream tiles (products staged in LDS, one lane per row)       */
    VTK_LAYOUT_SELL = 2, /* SELL-64 copy: one wavefront per 64 rows, entries column-major;
                          * columns dictionary-coded per 64-row chunk (4-bit codes into the
                          * chunk's <= 15 distinct col-row offsets; chunks with more keep int32) */
    VTK_LAYOUT_SELL32 = 3 /* SELL-64 with int32 columns everywhere                              */
} vtk_layout;

/* what vtk_csr_layout_info reports: the layout in use and the bytes one SpMV reads of the
 * operator in it (values, columns or codes + dictionaries, offsets)                          */
typedef struct {
    int layout;              /* vtk_layout in use (never AUTO)                                */
    double matrix_bytes;
    int64_t sell_chunks, sell_entries, wide_chunks;
} vtk_layout_info;

/* Synthetic Vlasov operator parameters. */
typedef struct {
    int dim;            /* 1, 2 or 4                                   */
    int fp32;           /* 1: values stored as float32 (C4)            */
    int64_t shape[4];   /* (n) | (Nx, Nv) | (Nx, Ny, Nvx, Nvy)          */
    double vmax, E0, nu, alpha, cfl;
} vtk_vlasov_params;

typedef struct {
    int64_t inner_iters;   /* Arnoldi steps over all restart cycles (SciPy's inner_iter)  */
    int64_t restarts;      /* restart cycles run                                          */
    double presid;         /* last preconditioned residual estimate                       */
    double rnorm;          /* last true residual ||b - A x||                              */
    double bnorm;          /* ||b||                                                       */
    double atol_eff;       /* max(atol, rtol*||b||)  (_get_atol_rtol, iterative.py:19)    */
    double t_solve;        /* seconds, device work of the solve (host wall, synced)       */
    double bytes_moved;    /* algorithmic HBM bytes of the solve           */
    int breakdown;         /* 1 if the last cycle hit h1 <= eps*h0                        */
    int orth;              /* vtk_orth used                                               */
    int band;              /* 1: the line-band DCGS2 step ran (vtk_csr_set_line_band)      */
} vtk_stats;

/* ---- library ------------------------------------------------------------------------ */
int vtk_abi_version(void);
/* 16 hex digits: SHA-256 of the library's sources (the .hip, .hpp and .cpp files of csrc, this
 * header, the Makefile and its EXTRA flags) at build time.  Callers that ship a prebuilt binary next to the
 * sources (the GPU box) compare it with the checked-out tree (vtkrylov._abi.check_build_id).
 * (ABI 5) */
const char *vtk_build_id(void);
const char *vtk_status_string(int status);
/* last error message of ctx (or of the last context-free call when ctx == NULL) */
int vtk_last_error(vtk_ctx *ctx, char *buf, size_t len);

/* ---- host-only helpers (no GPU required) -------------------------------------------- */
/* operator assembly (Appendix A) */
int vtk_vlasov_size(const vtk_vlasov_params *p, int64_t *n, int64_t *nnz);
/* rows [r0, r1): indptr has r1-r0+1 entries starting at 0; indices are global columns;
 * data is double[] or float[] per p->fp32; buffers sized for the row block's nnz */
int vtk_vlasov_generate(const vtk_vlasov_params *p, int64_t r0, int64_t r1, int32_t *indptr,
                        int32_t *indices, void *data);
/* b[i - r0] = 2 * ((splitmix64(seed + i) >> 11) * 2^-53) - 1   */
int vtk_rhs_splitmix(uint64_t seed, int64_t r0, int64_t r1, double *b);
/* contiguous row partition: offsets[world+1], boundaries multiples of align, balanced by
 * nnz when indptr (global, n+1 entries) is given, else by rows */
int vtk_partition_rows(int64_t n, const int32_t *indptr, int world, int align, int64_t *offsets);
/* Halo plan of one rank's row block.  In: local CSR with GLOBAL column
 * indices, the partition offsets.  Out: local_indices (nnz entries; owned column c ->
 * c - row_begin, halo column -> n_local + position in halo_cols), halo_cols (global ids,
 * sorted ascending, so grouped by owner rank) and halo_count_per_rank[world].  Pass
 * halo_cols == NULL to query *n_halo first. */
int vtk_halo_plan(int64_t n_global, const int64_t *offsets, int world, int rank,
                  int64_t nnz, const int32_t *indices, int32_t *local_indices,
                  int64_t *n_halo, int64_t *halo_cols, int64_t *halo_count_per_rank);

/* Geometry of the line-band DCGS2 step (vtk_csr_set_line_band) for a slab of
 * n_local rows in lines of line_len rows on a device with n_cu compute units (n_cu <= 0: 256).
 * VTK_ERR_ARG when the step cannot run on such a slab: line_len not a multiple of 8, n_local
 * not whole lines, fewer than 2 lines, or a slab (with its two halo lines) beyond the kernels'
 * 32-bit row / column indices.  (ABI 3) */
typedef struct {
    int parts;          /* wavefronts per line, <= 56 rows each (> 1 needs couplings within v-1..v+1) */
    int wg_per_range;   /* workgroups per line range */
    int waves_per_wg;   /* wavefronts per workgroup (<= 8: two per SIMD) */
    int ranges;         /* line ranges of one launch; every range walks its lines in order */
    int64_t lines;      /* lines of the slab */
} vtk_band_geometry;
int vtk_line_band_plan(int64_t n_local, int64_t line_len, int n_cu, vtk_band_geometry *out);

/* ---- device context / communicator ---------------------------------------------------- */
int vtk_device_count(int *count);
int vtk_ctx_create(int hip_device, vtk_ctx **out);      /* owns one hipStream_t */
void vtk_ctx_destroy(vtk_ctx *ctx);
int vtk_ctx_stream(vtk_ctx *ctx, void **hip_stream);    /* the stream all work runs on */
int vtk_ctx_synchronize(vtk_ctx *ctx);
/* Tuning switches of a context.  Defaults are the production path; the other
 * settings exist for in-process A/B measurements and for the bit-identity tests (the same sums
 * with and without a byte-saving form).  Each key is seeded from the environment variable
 * VTK_<KEY in upper case> once, when the context is created; the library reads its environment
 * nowhere else (fail_step is a test hook: this rank fails its DCGS2 step of that index in the
 * first cycle, vtk_gmres).  Keys: band, band_lsv, sell_canon, band_canon, band_opt, band_long_rows, lsv_ring,
 * prof_perj, comm_solo, auto_band, grid4, c4_fused, g4_ring, g4_gr, g4_fast, line_fuse, cyc_ring,
 * fail_step.
 * VTK_ERR_ARG for an unknown key; a VTK_<KEY> variable of a key removed in round 5 draws a
 * warning on stderr at context creation and is otherwise ignored.  (ABI 5; fail_step ABI 6;
 * band_long_rows round 6: band_opt bits 3 and 4 only on ranks of at least that many rows) */
int vtk_ctx_set_tuning(vtk_ctx *ctx, const char *key, int value);
int vtk_ctx_get_tuning(vtk_ctx *ctx, const char *key, int *value);
/* rank 0 creates the 128-byte RCCL unique id; the caller broadcasts it (any transport) */
int vtk_comm_unique_id(void *out128);
int vtk_comm_init(vtk_ctx *ctx, int rank, int world, const void *rccl_unique_id);
/* Host-staged communicator (test/debug transport, e.g. several ranks sharing one GPU, which
 * RCCL refuses): the library synchronises its stream, copies the payload to host memory, calls
 * these hooks and copies the result back.  Counts and offsets are in elements.  Each hook
 * returns 0 on success.  The production path is RCCL (vtk_comm_init). */
typedef struct {
    void *user;
    int (*allreduce_sum_f64)(void *user, double *buf, int64_t count);
    int (*alltoallv)(void *user, const void *sendbuf, const int64_t *send_counts,
                     const int64_t *send_offsets, void *recvbuf, const int64_t *recv_counts,
                     const int64_t *recv_offsets, int64_t elem_bytes);
    int (*allgather)(void *user, const void *sendbuf, void *recvbuf, int64_t bytes_per_rank);
} vtk_host_comm;
int vtk_comm_init_host(vtk_ctx *ctx, int rank, int world, const vtk_host_comm *ops);
int vtk_comm_info(vtk_ctx *ctx, int *rank, int *world);
/* ranks of the context's RCCL communicator (ncclCommCount); 0 when the context has none
 * (world 1, or the host-staged transport) */
int vtk_comm_rccl_count(vtk_ctx *ctx, int *count);

/* ---- operator ------------------------------------------------------------------------ */
/* Row block [offsets[rank], offsets[rank+1]) of an n_global x n_global CSR matrix with
 * GLOBAL column indices.  offsets has world+1 entries (NULL when world == 1).  Arrays are
 * host or device memory per ptr_kind and are copied. */
int vtk_csr_create(vtk_ctx *ctx, int64_t n_global, const int64_t *offsets, int64_t nnz_local,
                   const int32_t *indptr, const int32_t *indices, const void *data,
                   int data_is_fp32, int ptr_kind, vtk_csr **out);
/* generate this rank's rows of the Vlasov operator directly into device memory */
int vtk_csr_create_vlasov(vtk_ctx *ctx, const vtk_vlasov_params *p, const int64_t *offsets,
                          vtk_csr **out);
int vtk_csr_info(vtk_csr *A, int64_t *n_global, int64_t *row_begin, int64_t *row_end,
                 int64_t *nnz_local, int64_t *n_halo);
/* copy this rank's CSR back (indices GLOBAL), host memory */
int vtk_csr_download(vtk_csr *A, int32_t *indptr, int32_t *indices, void *data);
void vtk_csr_destroy(vtk_csr *A);
/* choose the SpMV layout (vtk_layout); SELL builds the copy on first use (device memory:
 * 12 B per padded entry, 8 B with f32 values) */
int vtk_csr_set_layout(vtk_csr *A, int layout);
int vtk_csr_get_layout(vtk_csr *A, int *layout_in_use);
int vtk_csr_layout_info(vtk_csr *A, vtk_layout_info *out);
/* Line-band structure: rows form x-lines of `line_len` consecutive rows and
 * every column lies in the lines x-1, x, x+1 (mod n / line_len) of its row's line x -- the 2D
 * Vlasov operators with line_len = Nv (set automatically by vtk_csr_create_vlasov, on one rank
 * or across ranks).  Checked on the device (VTK_ERR_ARG when the structure does not hold;
 * line_len 0 clears it; the local row count and its halo must fit 32-bit indices).  Across
 * ranks (world > 1) the call is collective: each rank's slab must hold whole lines with the two
 * neighbour lines as its halo, and the band is set on every rank or on none.  With it,
 * vtk_gmres runs each DCGS2 update pass together with the next step's SpMV + BJ + dots in one
 * sweep (SELL layout, tridiagonal BJ(8), restart <= 20; across ranks the neighbours' edge lines
 * of v_{j-1} and w_j travel as ghost lines each step): the basis is read once per Arnoldi step
 * instead of twice, and the candidate p_j is recomputed in registers instead of stored.
 * Same operator, same update arithmetic. */
int vtk_csr_set_line_band(vtk_csr *A, int64_t line_len);
int vtk_csr_get_line_band(vtk_csr *A, int64_t *line_len);
/* *separable = 1 when the line band is set and the operator's values are line-separable: every
 * coupling to line x+-1 depends only on the position v in the line, every coupling to v+-1 in
 * the same line only on the line x (the 2D Vlasov operators: advection in x with speed v, force
 * along v with field E(x)).  Checked bit for bit against the CSR when the band is set; the band
 * step then reads the diagonal per row and those couplings from per-position / per-line tables
 * (8 B of values per row instead of 40; the same values, summed in the same order).  2: also
 * every row canonical (the couplings to x-1, v-1, the diagonal, v+1, x+1 in ascending column
 * order): the band step derives the entries' kinds and order from the row's line and reads no
 * column codes either.  ABI 4. */
int vtk_csr_get_line_values(vtk_csr *A, int *separable);
/* 4D phase-space grid: rows ((ix Ny + iy) Nvx + jvx) Nvy + jvy, x and y periodic,
 * vx and vy Dirichlet, every row coupled to x+-1, y+-1, vx+-1, vy+-1 in ascending column order,
 * each coupling's value depending on one coordinate (x: jvx, y: jvy, vx: ix, vy: iy) -- the 4D
 * Vlasov operators.  Checked on the device bit for bit (VTK_ERR_ARG when it does not hold; Ny 0
 * clears it); set automatically by vtk_csr_create_vlasov (dim 4) and by vtk_csr_create when the
 * first row's column distances are 1, Nvy, Nvx Nvy, Ny Nvx Nvy.  With it the solver's SpMV
 * launches take each row's columns from its coordinates and its values from the diagonal per row
 * and per-coordinate tables (one value per row read instead of nine values and nine codes; the
 * same sums).  Rank-local, not collective; across ranks the slabs must be whole x planes with the
 * two neighbour planes as the halo.  dims = {Ny, Nvx, Nvy} (zeros: not set).  (ABI 5) */
int vtk_csr_set_grid4(vtk_csr *A, int64_t Ny, int64_t Nvx, int64_t Nvy);
int vtk_csr_get_grid4(vtk_csr *A, int64_t *dims);

/* y = A x on this rank's rows; x holds this rank's rows of the vector (halo exchanged
 * internally over RCCL when world > 1).  Bit-identical to csr_matvec (serial row sums). */
int vtk_spmv(vtk_csr *A, const double *x, double *y, int ptr_kind);

/* ---- block-Jacobi preconditioner ------------------------------------------------------- */
int vtk_bjacobi_create(vtk_csr *A, int block_size, vtk_prec **out);
/* how the block inverses are computed: EXACT = Gauss-Jordan with partial pivoting, one lane per
 * block row, bit-identical to numpy.linalg.inv's oracle restatement; MFMA (bs 16 / 32 only) =
 * blocked Gauss-Jordan whose rank-4 panel updates run on v_mfma_f64_16x16x4f64 -- the same pivot
 * rule, rounding-level differences; AUTO = MFMA for bs 16 and 32 (2.3x / 4.7x
 * faster at C3), EXACT otherwise.  vtk_bjacobi_create uses EXACT. */
typedef enum { VTK_BJ_SETUP_EXACT = 0, VTK_BJ_SETUP_MFMA = 1, VTK_BJ_SETUP_AUTO = 2 } vtk_bj_setup;
int vtk_bjacobi_create_ex(vtk_csr *A, int block_size, int setup, vtk_prec **out);
/* export the block inverses: (n_local + bs - 1) / bs blocks of bs*bs doubles, row-major */
int vtk_bjacobi_inverse(vtk_prec *M, double *inv, int ptr_kind);
int vtk_bjacobi_apply(vtk_prec *M, const double *r, double *z, int ptr_kind);
/* select the apply (vtk_bj_mode) for vtk_bjacobi_apply and vtk_gmres; VTK_ERR_ARG if TRIDIAG
 * is asked for blocks that are not tridiagonal (or whose factors failed the check) */
int vtk_bjacobi_set_mode(vtk_prec *M, int mode);
/* *mode_in_use = VTK_BJ_INVERSE or VTK_BJ_TRIDIAG; *tridiag_available = 0/1 (either may be NULL) */
int vtk_bjacobi_get_mode(vtk_prec *M, int *mode_in_use, int *tridiag_available);
void vtk_prec_destroy(vtk_prec *M);

/* ---- line-Jacobi preconditioner --------------------------------------
 * Line-implicit x-direction preconditioner.  M keeps A's diagonal and the couplings between
 * global rows R and R +- stride whose line index R / stride lies in the same segment of `seg`
 * consecutive line indices (segments also end at the rank's row block): every (segment,
 * R mod stride) is a tridiagonal system along an x-line, factored by Thomas (no pivoting) and
 * applied by a forward and a backward sweep (24 B of factors per row).  SciPy statement:
 * splu(M).solve as a LinearOperator.  Vlasov operators: stride 1 (1D), Nv (2D), Ny*Nvx*Nvy
 * (4D); seg dividing Nx / world makes M independent of the rank count.  VTK_ERR_SINGULAR
 * when a pivot is zero or not finite.  Apply with vtk_prec_apply (or vtk_bjacobi_apply); use
 * as vtk_gmres's M. */
typedef enum { VTK_PREC_BJACOBI = 0, VTK_PREC_LINE = 1 } vtk_prec_kind;
int vtk_linejacobi_create(vtk_csr *A, int64_t stride, int64_t seg, vtk_prec **out);
/* export the factors l | m | g (3 * n_local doubles; the oracle's orc_line_setup layout) */
int vtk_linejacobi_factors(vtk_prec *M, double *f, int ptr_kind);
/* COMPACT apply (default when available): when every line's x-couplings are bit-equal along
 * the line (x-invariant advection, as in the Vlasov operators, checked at setup) the apply
 * forms l and g from them and reads only m: 16 B/row instead of 32, same result bits.
 * set_compact(0) forces the stored-factor apply; set_compact(1) fails when unavailable. */
int vtk_linejacobi_set_compact(vtk_prec *M, int on);
int vtk_linejacobi_get_compact(vtk_prec *M, int *in_use, int *available);
/* z = M^-1 r for any preconditioner; *kind = vtk_prec_kind */
int vtk_prec_apply(vtk_prec *M, const double *r, double *z, int ptr_kind);
int vtk_prec_kind_of(vtk_prec *M, int *kind);
/* w = M^-1 (A x): the preconditioned operator GMRES applies at every Arnoldi step (SciPy:
 * M.matvec(A @ x), iterative.py:752), computed by the launch the solver's split DCGS2 step uses
 * for this operator and preconditioner (the 4D grid-row ring kernel -- across ranks in the
 * solver's interior / boundary form --, else the SpMV with the BJ epilogue, else SpMV then
 * apply); M may be NULL (w = A x).  Bit-identical across those forms: the kernel-level pin. */
int vtk_precond_matvec(vtk_csr *A, vtk_prec *M, const double *x, double *w, int ptr_kind);

/* ---- solver --------------------------------------------------------------------------- */
/* scipy.sparse.linalg.gmres semantics (iterative.py:582-841, callback=None): restarted,
 * left-preconditioned GMRES(restart); maxiter counts restart cycles (<= 0: 10 n); x holds
 * x0 on entry and the solution on exit; info = 0 on convergence else maxiter.
 * Across ranks (DCGS2): a rank whose launch fails mid-solve returns its error, and every
 * rank -- the failing one included -- leaves the solve after the same Arnoldi step: the
 * failure travels as a vote in the step's all-reduce, so no rank is left blocked in a
 * collective; the peers return VTK_ERR_PEER and the communicator stays usable.  A failed
 * collective itself (VTK_ERR_RCCL) marks the communicator broken: vtk_ctx_destroy then
 * aborts it (ncclCommAbort) instead of destroying it.  (The modelled failure is a launch the
 * rank could not issue; a device fault that kills the HIP context cannot join any collective
 * and is left to the launcher's watchdog.) */
int vtk_gmres(vtk_csr *A, vtk_prec *M, const double *b, double *x, double rtol, double atol,
              int restart, int64_t maxiter, int ptr_kind, int *info, vtk_stats *stats);
int vtk_gmres_set_orth(vtk_ctx *ctx, int orth);
/* on (default) / off: the line-band DCGS2 step when the operator and preconditioner allow it
 * (vtk_csr_set_line_band); off keeps the separate update pass and fused SpMV step */
int vtk_gmres_set_band(vtk_ctx *ctx, int on);

/* ---- kernel profile (measurement) ------------------------------------------
 * When enabled, every kernel the library launches is bracketed by HIP events on the
 * context's stream; per kernel class the driver accumulates launches, device seconds and the
 * ALGORITHMIC bytes of each launch (the per-unit figures of SURVEY.md §8d).  No-op launches
 * after a cycle's stop column are not counted.  Costs ~a few us per launch: not for timing
 * whole solves. */
typedef struct {
    char name[32];       /* kernel class, e.g. "spmv_bj", "mgs", "tail", "spmv"        */
    int64_t launches;
    double seconds;      /* sum of event-measured durations                            */
    double bytes;        /* sum of algorithmic bytes                                   */
} vtk_kernel_profile;
int vtk_profile_enable(vtk_ctx *ctx, int on);   /* on: also clears the counters */
int vtk_profile_read(vtk_ctx *ctx, vtk_kernel_profile *out, int max_entries, int *n_entries);

#ifdef __cplusplus
}
#endif
#endif /* VTKRYLOV_H */
