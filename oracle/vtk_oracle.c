/* vtk_oracle.c — CPU restatement of the vtkrylov hot path.  TEST INFRASTRUCTURE ONLY
 * (see vtk_oracle.h).  Every function cites what it restates:
 *   - operator / RHS: SURVEY.md Appendix A and §8(d); the NumPy twin oracle/twin.py
 *     (_rows_entries, rhs) uses the identical operation order.
 *   - SpMV: scipy sparsetools csr_matvec, reached from scipy/sparse/_compressed.py:518-530
 *     (serial per-row sum, ascending column order, sum starts at 0).
 *   - BJ: SURVEY.md §8a rows a3/a4 (dense diagonal blocks, inverse, batched matvec).
 *   - GMRES: scipy/sparse/linalg/_isolve/iterative.py:692-841 and _get_atol_rtol :10-21.
 *   - lartg: LAPACK 3.10+ dlartg.f90 (the version bundled with SciPy 1.15's OpenBLAS).
 * Compile with -ffp-contract=off (oracle/Makefile).
 */
#include "vtk_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

int64_t orc_n(const orc_vlasov *p) {
    if (p->dim == 1) return p->shape[0];
    if (p->dim == 2) return p->shape[0] * p->shape[1];
    return p->shape[0] * p->shape[1] * p->shape[2] * p->shape[3];
}

int64_t orc_nnz(const orc_vlasov *p) {
    int64_t n = orc_n(p);
    if (p->dim == 1) return 3 * n;
    if (p->dim == 2) return 5 * n - 2 * p->shape[0];
    return 9 * n - 2 * (n / p->shape[2]) - 2 * (n / p->shape[3]);
}

static int64_t pmod(int64_t a, int64_t m) { int64_t r = a % m; return r < 0 ? r + m : r; }

/* candidate entries of one row, in twin.py _rows_entries order; returns count K (cols<0 = absent) */
static int row_entries(const orc_vlasov *p, int64_t r, int64_t *cols, double *vals) {
    const double vmax = p->vmax, E0 = p->E0, nu = p->nu, alpha = p->alpha, cfl = p->cfl;
    if (p->dim == 1) {
        int64_t n = p->shape[0];
        double dx = 1.0 / (double)n;
        double dt = cfl * dx / 1.0;
        double cx = dt / dx;
        double v = 1.0, av = 1.0;
        cols[0] = pmod(r - 1, n); vals[0] = cx * (-0.5 * v - alpha * av);
        cols[1] = r;              vals[1] = 1.0 + 2.0 * alpha * cx * av;
        cols[2] = pmod(r + 1, n); vals[2] = cx * (0.5 * v - alpha * av);
        return 3;
    }
    if (p->dim == 2) {
        int64_t Nx = p->shape[0], Nv = p->shape[1];
        int64_t i = r / Nv, j = r % Nv;
        double dx = 1.0 / (double)Nx;
        double dv = 2.0 * vmax / (double)Nv;
        double dt = cfl * dx / vmax;
        double cx = dt / dx, cv = dt / dv, d2 = nu * dt / (dv * dv);
        double v = -vmax + ((double)j + 0.5) * dv;
        double s = ((double)i + 0.5) / (double)Nx;
        double E = E0 * (1.0 - 4.0 * fabs(s - 0.5));
        double av = fabs(v), aE = fabs(E);
        cols[0] = pmod(i - 1, Nx) * Nv + j;   vals[0] = cx * (-0.5 * v - alpha * av);
        cols[1] = j > 0 ? r - 1 : -1;         vals[1] = cv * (-0.5 * E - alpha * aE) - d2;
        cols[2] = r;                          vals[2] = 1.0 + 2.0 * alpha * cx * av + 2.0 * alpha * cv * aE + 2.0 * d2;
        cols[3] = j < Nv - 1 ? r + 1 : -1;    vals[3] = cv * (0.5 * E - alpha * aE) - d2;
        cols[4] = pmod(i + 1, Nx) * Nv + j;   vals[4] = cx * (0.5 * v - alpha * av);
        return 5;
    }
    int64_t Nx = p->shape[0], Ny = p->shape[1], Nvx = p->shape[2], Nvy = p->shape[3];
    int64_t jy = r % Nvy, t = r / Nvy;
    int64_t jx = t % Nvx; t = t / Nvx;
    int64_t iy = t % Ny, ix = t / Ny;
    double dx = 1.0 / (double)Nx, dy = 1.0 / (double)Ny;
    double dvx = 2.0 * vmax / (double)Nvx, dvy = 2.0 * vmax / (double)Nvy;
    double dt = cfl * (dx < dy ? dx : dy) / vmax;
    double cx = dt / dx, cy = dt / dy, cvx = dt / dvx, cvy = dt / dvy;
    double d2x = nu * dt / (dvx * dvx), d2y = nu * dt / (dvy * dvy);
    double vx = -vmax + ((double)jx + 0.5) * dvx;
    double vy = -vmax + ((double)jy + 0.5) * dvy;
    double sx = ((double)ix + 0.5) / (double)Nx, sy = ((double)iy + 0.5) / (double)Ny;
    double Ex = E0 * (1.0 - 4.0 * fabs(sx - 0.5)), Ey = E0 * (1.0 - 4.0 * fabs(sy - 0.5));
    double avx = fabs(vx), avy = fabs(vy), aEx = fabs(Ex), aEy = fabs(Ey);
    int64_t sxs = Ny * Nvx * Nvy, sys = Nvx * Nvy;
    int64_t base = r - ix * sxs - iy * sys;
    cols[0] = pmod(ix - 1, Nx) * sxs + iy * sys + base;  vals[0] = cx * (-0.5 * vx - alpha * avx);
    cols[1] = pmod(ix + 1, Nx) * sxs + iy * sys + base;  vals[1] = cx * (0.5 * vx - alpha * avx);
    cols[2] = ix * sxs + pmod(iy - 1, Ny) * sys + base;  vals[2] = cy * (-0.5 * vy - alpha * avy);
    cols[3] = ix * sxs + pmod(iy + 1, Ny) * sys + base;  vals[3] = cy * (0.5 * vy - alpha * avy);
    cols[4] = jx > 0 ? r - Nvy : -1;        vals[4] = cvx * (-0.5 * Ex - alpha * aEx) - d2x;
    cols[5] = jx < Nvx - 1 ? r + Nvy : -1;  vals[5] = cvx * (0.5 * Ex - alpha * aEx) - d2x;
    cols[6] = jy > 0 ? r - 1 : -1;          vals[6] = cvy * (-0.5 * Ey - alpha * aEy) - d2y;
    cols[7] = jy < Nvy - 1 ? r + 1 : -1;    vals[7] = cvy * (0.5 * Ey - alpha * aEy) - d2y;
    cols[8] = r;
    vals[8] = 1.0 + 2.0 * alpha * cx * avx + 2.0 * alpha * cy * avy + 2.0 * alpha * cvx * aEx
              + 2.0 * alpha * cvy * aEy + 2.0 * d2x + 2.0 * d2y;
    return 9;
}

int orc_generate(const orc_vlasov *p, int64_t r0, int64_t r1, int32_t *indptr,
                 int32_t *indices, void *data) {
    int64_t cols[9];
    double vals[9];
    int64_t nz = 0;
    indptr[0] = 0;
    for (int64_t r = r0; r < r1; ++r) {
        int K = row_entries(p, r, cols, vals);
        /* stable insertion sort of the valid entries by column */
        int64_t c[9];
        double v[9];
        int m = 0;
        for (int k = 0; k < K; ++k) {
            if (cols[k] < 0) continue;
            int q = m++;
            while (q > 0 && c[q - 1] > cols[k]) { c[q] = c[q - 1]; v[q] = v[q - 1]; --q; }
            c[q] = cols[k];
            v[q] = vals[k];
        }
        for (int k = 0; k < m; ++k) {
            indices[nz] = (int32_t)c[k];
            if (p->fp32) ((float *)data)[nz] = (float)v[k];
            else ((double *)data)[nz] = v[k];
            ++nz;
        }
        indptr[r - r0 + 1] = (int32_t)nz;
    }
    return 0;
}

static uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

double orc_rhs_value(uint64_t seed, int64_t i) {
    double u = (double)(splitmix64(seed + (uint64_t)i) >> 11) * 0x1p-53;
    return 2.0 * u - 1.0;
}

void orc_rhs(uint64_t seed, int64_t r0, int64_t r1, double *b) {
    for (int64_t i = r0; i < r1; ++i) b[i - r0] = orc_rhs_value(seed, i);
}

static inline double val_at(const void *data, int fp32, int64_t k) {
    return fp32 ? (double)((const float *)data)[k] : ((const double *)data)[k];
}

/* sparsetools csr_matvec: sum = 0; sum += Ax[jj] * Xx[Aj[jj]] (ascending jj) */
void orc_spmv(int64_t nrows, const int32_t *indptr, const int32_t *indices, const void *data,
              int fp32, const double *x, double *y) {
    for (int64_t i = 0; i < nrows; ++i) {
        double sum = 0.0;
        for (int32_t k = indptr[i]; k < indptr[i + 1]; ++k) sum += val_at(data, fp32, k) * x[indices[k]];
        y[i] = sum;
    }
}

/* Dense diagonal block k of rows [k*bs, k*bs+bs) (short last block padded with identity),
 * inverted by Gauss-Jordan with partial pivoting (first max |a|).  The HIP setup kernel
 * (vtk_bjacobi.hip) performs the identical sequence of IEEE operations. */
int64_t orc_bj_setup(int64_t n, const int32_t *indptr, const int32_t *indices, const void *data,
                     int fp32, int bs, double *inv) {
    int64_t nb = (n + bs - 1) / bs;
    double *A = (double *)malloc(sizeof(double) * bs * bs);
    double *I = (double *)malloc(sizeof(double) * bs * bs);
    for (int64_t b = 0; b < nb; ++b) {
        memset(A, 0, sizeof(double) * bs * bs);
        memset(I, 0, sizeof(double) * bs * bs);
        for (int i = 0; i < bs; ++i) {
            int64_t r = b * bs + i;
            I[i * bs + i] = 1.0;
            if (r >= n) { A[i * bs + i] = 1.0; continue; }
            for (int32_t k = indptr[r]; k < indptr[r + 1]; ++k) {
                int64_t c = indices[k];
                /* duplicates add up in stored order (csr_matrix.toarray()) */
                if (c >= b * bs && c < b * bs + bs) A[i * bs + (c - b * bs)] += val_at(data, fp32, k);
            }
        }
        for (int c = 0; c < bs; ++c) {
            int piv = c;
            double best = fabs(A[c * bs + c]);
            for (int r = c + 1; r < bs; ++r) {
                double a = fabs(A[r * bs + c]);
                if (a > best) { best = a; piv = r; }
            }
            if (best == 0.0) { free(A); free(I); return -(b + 1); }
            if (piv != c) {
                for (int j = 0; j < bs; ++j) {
                    double t = A[c * bs + j]; A[c * bs + j] = A[piv * bs + j]; A[piv * bs + j] = t;
                    t = I[c * bs + j]; I[c * bs + j] = I[piv * bs + j]; I[piv * bs + j] = t;
                }
            }
            double d = A[c * bs + c];
            for (int j = 0; j < bs; ++j) { A[c * bs + j] = A[c * bs + j] / d; I[c * bs + j] = I[c * bs + j] / d; }
            for (int r = 0; r < bs; ++r) {
                if (r == c) continue;
                double f = A[r * bs + c];
                for (int j = 0; j < bs; ++j) {
                    A[r * bs + j] = A[r * bs + j] - f * A[c * bs + j];
                    I[r * bs + j] = I[r * bs + j] - f * I[c * bs + j];
                }
            }
        }
        memcpy(inv + b * bs * bs, I, sizeof(double) * bs * bs);
    }
    free(A);
    free(I);
    return 0;
}

/* z_b = inv_b * r_b, serial j order per row */
void orc_bj_apply(int64_t n, int bs, const double *inv, const double *r, double *z) {
    int64_t nb = (n + bs - 1) / bs;
    for (int64_t b = 0; b < nb; ++b) {
        for (int i = 0; i < bs; ++i) {
            int64_t row = b * bs + i;
            if (row >= n) break;
            double s = 0.0;
            for (int j = 0; j < bs; ++j) {
                int64_t col = b * bs + j;
                double rv = col < n ? r[col] : 0.0;
                s += inv[(b * bs + i) * bs + j] * rv;
            }
            z[row] = s;
        }
    }
}

/* LAPACK 3.10+ dlartg.f90 */
void orc_lartg(double f, double g, double *c, double *s, double *r) {
    const double safmin = DBL_MIN;            /* 2^-1022 */
    const double safmax = 1.0 / DBL_MIN;      /* 2^1022  */
    const double rtmin = sqrt(safmin);
    const double rtmax = sqrt(safmax / 2.0);
    double f1 = fabs(f), g1 = fabs(g);
    if (g == 0.0) {
        *c = 1.0; *s = 0.0; *r = f;
    } else if (f == 0.0) {
        *c = 0.0; *s = copysign(1.0, g); *r = g1;
    } else if (f1 > rtmin && f1 < rtmax && g1 > rtmin && g1 < rtmax) {
        double d = sqrt(f * f + g * g);
        *c = f1 / d;
        *r = copysign(d, f);
        *s = g / *r;
    } else {
        double u = f1 > g1 ? f1 : g1;
        if (u < safmin) u = safmin;
        if (u > safmax) u = safmax;
        double fs = f / u, gs = g / u;
        double d = sqrt(fs * fs + gs * gs);
        *c = fabs(fs) / d;
        double rr = copysign(d, f);
        *s = gs / rr;
        *r = rr * u;
    }
}

/* ---- line Jacobi (line-implicit x-direction preconditioner) -------------
 * M keeps A's diagonal and the couplings between global rows R and R +- stride whose line
 * index i = R / stride falls in the same segment i / seg, both rows inside [row0, row0 + n).
 * Each (segment, j = R mod stride) is a tridiagonal system along its line; Thomas without
 * pivoting over the line in ascending i:
 *   u = b (first row) | l = a * m_prev, u = b - l * c_prev;   m = 1 / u;   g = c * m
 * with b, a, c the sums (stored order, from 0.0: toarray() semantics) of the row's entries in
 * columns R, R - stride, R + stride.  f = [l | m | g], n doubles each (l = 0 on first rows).
 * (l = a * m_prev rather than a / u_prev: the fused SpMV + line kernel forms l from the row's own
 * entry a and the previous row's m, so only m is stored for it.)  The HIP setup
 * (vtk_kernels.hip k_line_setup) runs the same IEEE operations per line. */
static int line_has(int64_t R, int64_t d, int64_t row0, int64_t n, int64_t stride, int64_t seg) {
    const int64_t Q = R + d * stride;
    return Q >= row0 && Q < row0 + n && (Q / stride) / seg == (R / stride) / seg;
}

int64_t orc_line_setup(int64_t n, const int32_t *indptr, const int32_t *indices, const void *data,
                       int fp32, int64_t row0, int64_t stride, int64_t seg, double *f) {
    double *cs = (double *)malloc(sizeof(double) * (n ? n : 1));   /* c of each row */
    double *l = f, *mm = f + n, *g = f + 2 * n;
    for (int64_t r = 0; r < n; ++r) {
        const int64_t R = row0 + r;
        const int hl = line_has(R, -1, row0, n, stride, seg), hr = line_has(R, 1, row0, n, stride, seg);
        double b = 0.0, a = 0.0, c = 0.0;
        for (int32_t k = indptr[r]; k < indptr[r + 1]; ++k) {
            const int64_t col = indices[k];
            const double v = val_at(data, fp32, k);
            if (col == R) b += v;
            else if (hl && col == R - stride) a += v;
            else if (hr && col == R + stride) c += v;
        }
        double lv = 0.0, uv;
        if (hl) {
            lv = a * mm[r - stride];
            uv = b - lv * cs[r - stride];
        } else {
            uv = b;
        }
        const double mv = 1.0 / uv;
        if (uv == 0.0 || !isfinite(uv) || !isfinite(mv)) { free(cs); return -(r + 1); }
        cs[r] = c;
        l[r] = lv;
        mm[r] = mv;
        g[r] = c * mv;
    }
    free(cs);
    return 0;
}

/* z = M^-1 r: forward d = r - l d_prev (d_prev = 0 on a first row), backward
 * z = m d - g z_next (z_next = 0 on a last row) */
void orc_line_apply(int64_t n, int64_t row0, int64_t stride, int64_t seg, const double *f,
                    const double *r, double *z) {
    const double *l = f, *mm = f + n, *g = f + 2 * n;
    double *d = (double *)malloc(sizeof(double) * (n ? n : 1));
    for (int64_t i = 0; i < n; ++i) {
        const double dp = line_has(row0 + i, -1, row0, n, stride, seg) ? d[i - stride] : 0.0;
        d[i] = r[i] - l[i] * dp;
    }
    for (int64_t i = n - 1; i >= 0; --i) {
        const double zn = line_has(row0 + i, 1, row0, n, stride, seg) ? z[i + stride] : 0.0;
        z[i] = mm[i] * d[i] - g[i] * zn;
    }
    free(d);
}

static double dot(int64_t n, const double *a, const double *b) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i) s += a[i] * b[i];
    return s;
}
static double nrm2(int64_t n, const double *a) { return sqrt(dot(n, a, a)); }

typedef struct {
    int64_t n;
    const int32_t *indptr, *indices;
    const void *data;
    int fp32;
    const double *inv;
    int bs;
    const double *line;   /* line-Jacobi factors (orc_line_setup), row0 = 0 */
    int64_t stride, seg;
} op_t;

static void matvec(const op_t *o, const double *x, double *y) {
    orc_spmv(o->n, o->indptr, o->indices, o->data, o->fp32, x, y);
}
static void psolve(const op_t *o, const double *r, double *z) {
    if (o->line) orc_line_apply(o->n, 0, o->stride, o->seg, o->line, r, z);
    else if (o->inv) orc_bj_apply(o->n, o->bs, o->inv, r, z);
    else memcpy(z, r, sizeof(double) * o->n);
}

static int gmres_op(const op_t *op, const double *b, double *x, double rtol, double atol,
                    int restart, int64_t maxiter, int *info, orc_stats *st);

int orc_gmres(int64_t n, const int32_t *indptr, const int32_t *indices, const void *data,
              int fp32, const double *bj_inv, int bs, const double *b, double *x, double rtol,
              double atol, int restart, int64_t maxiter, int *info, orc_stats *st) {
    op_t o = {n, indptr, indices, data, fp32, bj_inv, bs, NULL, 0, 0};
    return gmres_op(&o, b, x, rtol, atol, restart, maxiter, info, st);
}

int orc_gmres_line(int64_t n, const int32_t *indptr, const int32_t *indices, const void *data,
                   int fp32, const double *line_f, int64_t stride, int64_t seg, const double *b,
                   double *x, double rtol, double atol, int restart, int64_t maxiter, int *info,
                   orc_stats *st) {
    op_t o = {n, indptr, indices, data, fp32, NULL, 0, line_f, stride, seg};
    return gmres_op(&o, b, x, rtol, atol, restart, maxiter, info, st);
}

static int gmres_op(const op_t *op, const double *b, double *x, double rtol, double atol,
                    int restart, int64_t maxiter, int *info, orc_stats *st) {
    const op_t o = *op;
    const int64_t n = o.n;
    memset(st, 0, sizeof(*st));
    double bnrm2 = nrm2(n, b);
    double rb = rtol * bnrm2;                        /* _get_atol_rtol :19 */
    atol = atol > rb ? atol : rb;
    if (bnrm2 == 0.0) { memcpy(x, b, sizeof(double) * n); *info = 0; return 0; }
    const double eps = DBL_EPSILON;
    if (maxiter <= 0) maxiter = n * 10;
    if (restart <= 0) restart = 20;
    if (restart > n) restart = (int)n;
    int m = restart;
    double *V = (double *)malloc(sizeof(double) * (size_t)(m + 1) * n);
    double *r = (double *)malloc(sizeof(double) * n);
    double *w = (double *)malloc(sizeof(double) * n);
    double *av = (double *)malloc(sizeof(double) * n);
    double *h = (double *)calloc((size_t)m * (m + 1), sizeof(double));
    double *giv = (double *)calloc((size_t)m * 2, sizeof(double));
    double *S = (double *)malloc(sizeof(double) * (m + 1));
    double *y = (double *)malloc(sizeof(double) * (m + 1));
#define H(c, k) h[(size_t)(c) * (m + 1) + (k)]

    psolve(&o, b, w);
    double Mb_nrm2 = nrm2(n, w);
    double ptol_max_factor = 1.0;
    double q = atol / bnrm2;
    double ptol = Mb_nrm2 * (ptol_max_factor < q ? ptol_max_factor : q);
    double presid = 0.0, rnorm = 0.0;
    int64_t inner = 0, it;
    int done_early = 0;
    for (it = 0; it < maxiter; ++it) {
        if (it == 0) {
            int any = 0;
            for (int64_t i = 0; i < n; ++i) if (x[i] != 0.0) { any = 1; break; }
            if (any) { matvec(&o, x, av); for (int64_t i = 0; i < n; ++i) r[i] = b[i] - av[i]; }
            else memcpy(r, b, sizeof(double) * n);
            if (nrm2(n, r) < atol) { done_early = 1; break; }
        }
        double *v0 = V;
        psolve(&o, r, v0);
        double tmp = nrm2(n, v0);
        double inv = 1.0 / tmp;
        for (int64_t i = 0; i < n; ++i) v0[i] *= inv;
        for (int k = 0; k <= m; ++k) S[k] = 0.0;
        S[0] = tmp;
        int breakdown = 0, col;
        for (col = 0; col < m; ++col) {
            matvec(&o, V + (size_t)col * n, av);
            psolve(&o, av, w);
            double h0 = nrm2(n, w);
            for (int k = 0; k <= col; ++k) {
                const double *vk = V + (size_t)k * n;
                double t = dot(n, vk, w);
                H(col, k) = t;
                for (int64_t i = 0; i < n; ++i) w[i] -= t * vk[i];
            }
            double h1 = nrm2(n, w);
            H(col, col + 1) = h1;
            double *vn = V + (size_t)(col + 1) * n;
            memcpy(vn, w, sizeof(double) * n);
            if (h1 <= eps * h0) { H(col, col + 1) = 0.0; breakdown = 1; }
            else { double ih = 1.0 / h1; for (int64_t i = 0; i < n; ++i) vn[i] *= ih; }
            for (int k = 0; k < col; ++k) {
                double c = giv[2 * k], s = giv[2 * k + 1];
                double n0 = H(col, k), n1 = H(col, k + 1);
                H(col, k) = c * n0 + s * n1;
                H(col, k + 1) = -s * n0 + c * n1;
            }
            double c, s, mag;
            orc_lartg(H(col, col), H(col, col + 1), &c, &s, &mag);
            giv[2 * col] = c; giv[2 * col + 1] = s;
            H(col, col) = mag; H(col, col + 1) = 0.0;
            double t = -s * S[col];
            S[col] = c * S[col];
            S[col + 1] = t;
            presid = fabs(t);
            inner++;
            if (presid <= ptol || breakdown) break;
        }
        if (col == m) col = m - 1;   /* python's loop variable keeps the last value */
        if (H(col, col) == 0.0) S[col] = 0.0;
        for (int k = 0; k <= col; ++k) y[k] = S[k];
        for (int k = col; k > 0; --k) {
            if (y[k] != 0.0) {
                y[k] /= H(k, k);
                double t = y[k];
                for (int i = 0; i < k; ++i) y[i] -= t * H(k, i);
            }
        }
        if (y[0] != 0.0) y[0] /= H(0, 0);
        for (int64_t i = 0; i < n; ++i) {
            double acc = 0.0;
            for (int k = 0; k <= col; ++k) acc += y[k] * V[(size_t)k * n + i];
            x[i] += acc;
        }
        matvec(&o, x, av);
        for (int64_t i = 0; i < n; ++i) r[i] = b[i] - av[i];
        rnorm = nrm2(n, r);
        st->restarts = it + 1;
        if (rnorm <= atol) break;
        else if (breakdown) break;
        else if (presid <= ptol) ptol_max_factor = eps > 0.25 * ptol_max_factor ? eps : 0.25 * ptol_max_factor;
        else ptol_max_factor = 1.0 < 1.5 * ptol_max_factor ? 1.0 : 1.5 * ptol_max_factor;
        double q2 = atol / rnorm;
        ptol = presid * (ptol_max_factor < q2 ? ptol_max_factor : q2);
    }
#undef H
    st->inner_iters = inner;
    st->presid = presid;
    st->rnorm = rnorm;
    *info = done_early ? 0 : (rnorm <= atol ? 0 : (int)maxiter);
    free(V); free(r); free(w); free(av); free(h); free(giv); free(S); free(y);
    return 0;
}
