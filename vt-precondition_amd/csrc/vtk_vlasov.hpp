// vtk_vlasov.hpp — entries of one row of the synthetic Vlasov operator.
//
// One definition, compiled both for the host generator (vtk_host.cpp) and for the gfx950
// generator kernels (vtk_kernels.hip), with -ffp-contract=off on both sides, so host- and
// device-assembled operators are bit-identical.  The expressions follow the operation order
// fixed by the spec (oracle/twin.py _rows_entries is the NumPy statement of the same spec).
#pragma once
#include <stdint.h>

#include "../../include/vtkrylov.h"

#if defined(__HIPCC__)
#define VTK_HD __host__ __device__
#else
#define VTK_HD
#endif

namespace vtk {

struct VlasovRow {
    int count;           // valid entries, sorted by column
    int64_t col[9];
    double val[9];
};

VTK_HD inline int64_t vl_pmod(int64_t a, int64_t m) {
    int64_t r = a % m;
    return r < 0 ? r + m : r;
}

VTK_HD inline double vl_abs(double x) { return __builtin_fabs(x); }

// Number of stored entries of row r (boundary rows of the velocity directions drop one).
VTK_HD inline int vlasov_row_count(const vtk_vlasov_params &p, int64_t r) {
    if (p.dim == 1) return 3;
    if (p.dim == 2) {
        const int64_t Nv = p.shape[1], j = r % Nv;
        return 5 - (j == 0) - (j == Nv - 1);
    }
    const int64_t Nvx = p.shape[2], Nvy = p.shape[3];
    const int64_t jy = r % Nvy, jx = (r / Nvy) % Nvx;
    return 9 - (jx == 0) - (jx == Nvx - 1) - (jy == 0) - (jy == Nvy - 1);
}

VTK_HD inline void vl_push(VlasovRow &o, int64_t c, double v) {
    // insertion into the sorted list (columns are distinct for Nx, Ny >= 3)
    int q = o.count++;
    while (q > 0 && o.col[q - 1] > c) {
        o.col[q] = o.col[q - 1];
        o.val[q] = o.val[q - 1];
        --q;
    }
    o.col[q] = c;
    o.val[q] = v;
}

VTK_HD inline void vlasov_row(const vtk_vlasov_params &p, int64_t r, VlasovRow &o) {
    const double vmax = p.vmax, E0 = p.E0, nu = p.nu, alpha = p.alpha, cfl = p.cfl;
    o.count = 0;
    if (p.dim == 1) {
        const int64_t n = p.shape[0];
        const double dx = 1.0 / (double)n;
        const double dt = cfl * dx / 1.0;
        const double cx = dt / dx;
        const double v = 1.0, av = 1.0;
        vl_push(o, vl_pmod(r - 1, n), cx * (-0.5 * v - alpha * av));
        vl_push(o, r, 1.0 + 2.0 * alpha * cx * av);
        vl_push(o, vl_pmod(r + 1, n), cx * (0.5 * v - alpha * av));
        return;
    }
    if (p.dim == 2) {
        const int64_t Nx = p.shape[0], Nv = p.shape[1];
        const int64_t i = r / Nv, j = r % Nv;
        const double dx = 1.0 / (double)Nx;
        const double dv = 2.0 * vmax / (double)Nv;
        const double dt = cfl * dx / vmax;
        const double cx = dt / dx, cv = dt / dv, d2 = nu * dt / (dv * dv);
        const double v = -vmax + ((double)j + 0.5) * dv;
        const double s = ((double)i + 0.5) / (double)Nx;
        const double E = E0 * (1.0 - 4.0 * vl_abs(s - 0.5));
        const double av = vl_abs(v), aE = vl_abs(E);
        vl_push(o, vl_pmod(i - 1, Nx) * Nv + j, cx * (-0.5 * v - alpha * av));
        if (j > 0) vl_push(o, r - 1, cv * (-0.5 * E - alpha * aE) - d2);
        vl_push(o, r, 1.0 + 2.0 * alpha * cx * av + 2.0 * alpha * cv * aE + 2.0 * d2);
        if (j < Nv - 1) vl_push(o, r + 1, cv * (0.5 * E - alpha * aE) - d2);
        vl_push(o, vl_pmod(i + 1, Nx) * Nv + j, cx * (0.5 * v - alpha * av));
        return;
    }
    const int64_t Nx = p.shape[0], Ny = p.shape[1], Nvx = p.shape[2], Nvy = p.shape[3];
    const int64_t jy = r % Nvy, t1 = r / Nvy;
    const int64_t jx = t1 % Nvx, t2 = t1 / Nvx;
    const int64_t iy = t2 % Ny, ix = t2 / Ny;
    const double dx = 1.0 / (double)Nx, dy = 1.0 / (double)Ny;
    const double dvx = 2.0 * vmax / (double)Nvx, dvy = 2.0 * vmax / (double)Nvy;
    const double dt = cfl * (dx < dy ? dx : dy) / vmax;
    const double cx = dt / dx, cy = dt / dy, cvx = dt / dvx, cvy = dt / dvy;
    const double d2x = nu * dt / (dvx * dvx), d2y = nu * dt / (dvy * dvy);
    const double vx = -vmax + ((double)jx + 0.5) * dvx;
    const double vy = -vmax + ((double)jy + 0.5) * dvy;
    const double sx = ((double)ix + 0.5) / (double)Nx, sy = ((double)iy + 0.5) / (double)Ny;
    const double Ex = E0 * (1.0 - 4.0 * vl_abs(sx - 0.5));
    const double Ey = E0 * (1.0 - 4.0 * vl_abs(sy - 0.5));
    const double avx = vl_abs(vx), avy = vl_abs(vy), aEx = vl_abs(Ex), aEy = vl_abs(Ey);
    const int64_t sxs = Ny * Nvx * Nvy, sys = Nvx * Nvy;
    const int64_t base = r - ix * sxs - iy * sys;
    vl_push(o, vl_pmod(ix - 1, Nx) * sxs + iy * sys + base, cx * (-0.5 * vx - alpha * avx));
    vl_push(o, vl_pmod(ix + 1, Nx) * sxs + iy * sys + base, cx * (0.5 * vx - alpha * avx));
    vl_push(o, ix * sxs + vl_pmod(iy - 1, Ny) * sys + base, cy * (-0.5 * vy - alpha * avy));
    vl_push(o, ix * sxs + vl_pmod(iy + 1, Ny) * sys + base, cy * (0.5 * vy - alpha * avy));
    if (jx > 0) vl_push(o, r - Nvy, cvx * (-0.5 * Ex - alpha * aEx) - d2x);
    if (jx < Nvx - 1) vl_push(o, r + Nvy, cvx * (0.5 * Ex - alpha * aEx) - d2x);
    if (jy > 0) vl_push(o, r - 1, cvy * (-0.5 * Ey - alpha * aEy) - d2y);
    if (jy < Nvy - 1) vl_push(o, r + 1, cvy * (0.5 * Ey - alpha * aEy) - d2y);
    vl_push(o, r, 1.0 + 2.0 * alpha * cx * avx + 2.0 * alpha * cy * avy + 2.0 * alpha * cvx * aEx
                      + 2.0 * alpha * cvy * aEy + 2.0 * d2x + 2.0 * d2y);
}

VTK_HD inline int64_t vlasov_n(const vtk_vlasov_params &p) {
    if (p.dim == 1) return p.shape[0];
    if (p.dim == 2) return p.shape[0] * p.shape[1];
    return p.shape[0] * p.shape[1] * p.shape[2] * p.shape[3];
}

VTK_HD inline int64_t vlasov_nnz(const vtk_vlasov_params &p) {
    const int64_t n = vlasov_n(p);
    if (p.dim == 1) return 3 * n;
    if (p.dim == 2) return 5 * n - 2 * p.shape[0];
    return 9 * n - 2 * (n / p.shape[2]) - 2 * (n / p.shape[3]);
}

VTK_HD inline uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

VTK_HD inline double rhs_value(uint64_t seed, int64_t i) {
    const double u = (double)(splitmix64(seed + (uint64_t)i) >> 11) * 0x1p-53;
    return 2.0 * u - 1.0;
}

}  // namespace vtk
