/* vtk_oracle.h — CPU restatement of the vtkrylov hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library; the product (vt-precondition_amd/) never links or calls it.
 *
 * The reference (jwang1x/VT-precondition) has no numerical code, so this
 * file restates the path the north_star names — SciPy 1.15.3's scipy.sparse.linalg.gmres
 * with a block-Jacobi LinearOperator on the Appendix-A Vlasov operator — in plain C.
 * It is pinned against SciPy-generated golden vectors in tests/golden (make_golden.py).
 * Built with -ffp-contract=off so every + - * / is a single IEEE-rounded op.
 */
#ifndef VTK_ORACLE_H
#define VTK_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int dim;            /* 1, 2, 4 */
    int fp32;           /* store values as float32 */
    int64_t shape[4];   /* (n) | (Nx,Nv) | (Nx,Ny,Nvx,Nvy) */
    double vmax, E0, nu, alpha, cfl;
} orc_vlasov;

int64_t orc_n(const orc_vlasov *p);
int64_t orc_nnz(const orc_vlasov *p);
/* rows [r0,r1): indptr local (r1-r0+1, starts at 0), global column indices */
int orc_generate(const orc_vlasov *p, int64_t r0, int64_t r1, int32_t *indptr,
                 int32_t *indices, void *data);
double orc_rhs_value(uint64_t seed, int64_t i);
void orc_rhs(uint64_t seed, int64_t r0, int64_t r1, double *b);

void orc_spmv(int64_t nrows, const int32_t *indptr, const int32_t *indices, const void *data,
              int fp32, const double *x, double *y);
/* Gauss-Jordan with partial pivoting per diagonal block; returns 0 or -(block+1) if singular */
int64_t orc_bj_setup(int64_t n, const int32_t *indptr, const int32_t *indices, const void *data,
                     int fp32, int bs, double *inv);
void orc_bj_apply(int64_t n, int bs, const double *inv, const double *r, double *z);
void orc_lartg(double f, double g, double *c, double *s, double *r);

/* line Jacobi (x-direction line segments): factors f = [l | m | g] (3n
 * doubles) of the rows [row0, row0+n) with GLOBAL column indices; returns 0 or -(row+1) when a
 * pivot is zero or not finite.  apply: z = M^-1 r. */
int64_t orc_line_setup(int64_t n, const int32_t *indptr, const int32_t *indices, const void *data,
                       int fp32, int64_t row0, int64_t stride, int64_t seg, double *f);
void orc_line_apply(int64_t n, int64_t row0, int64_t stride, int64_t seg, const double *f,
                    const double *r, double *z);

typedef struct {
    int64_t inner_iters;
    int64_t restarts;
    double presid;
    double rnorm;
} orc_stats;

/* SciPy iterative.py:582-841 (callback_type=None), left-preconditioned GMRES(restart) + MGS */
int orc_gmres(int64_t n, const int32_t *indptr, const int32_t *indices, const void *data,
              int fp32, const double *bj_inv, int bs, const double *b, double *x, double rtol,
              double atol, int restart, int64_t maxiter, int *info, orc_stats *st);

/* the same GMRES with the line-Jacobi preconditioner (factors of orc_line_setup, row0 = 0) */
int orc_gmres_line(int64_t n, const int32_t *indptr, const int32_t *indices, const void *data,
                   int fp32, const double *line_f, int64_t stride, int64_t seg, const double *b,
                   double *x, double rtol, double atol, int restart, int64_t maxiter, int *info,
                   orc_stats *st);

#ifdef __cplusplus
}
#endif
#endif
