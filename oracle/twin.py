"""NumPy/SciPy oracle for the vtkrylov hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module.  Nothing in the product (``vt-precondition_amd/``) imports it.

Provenance / pinning
--------------------
* ``/root/reference`` (jwang1x/VT-precondition) contains no numerical code:
  the operator, RHS and solver parameters are the build's own spec, SURVEY.md Appendix A
  and §8(d).  The reference path the north_star names ("the reference scipy.sparse path")
  is SciPy 1.15.3 / NumPy 2.2.6 (third-party, present in this image):
    - SpMV      : ``scipy.sparse.csr_matrix @ x`` -> sparsetools ``csr_matvec``
                  (scipy/sparse/_compressed.py:518-530), serial per-row sum in column order.
    - GMRES     : ``scipy.sparse.linalg.gmres`` (scipy/sparse/linalg/_isolve/iterative.py:582,
                  body :692-841, tolerances ``_get_atol_rtol`` :10-21).
    - BJ        : ``numpy.linalg.inv`` on each bs x bs diagonal block, applied as
                  ``einsum('bij,bj->bi')`` inside a ``LinearOperator``.
* Golden vectors produced from this module + SciPy are committed under ``tests/golden``
  together with the script that made them (``tests/golden/make_golden.py``).  The
  reference itself pins nothing on this path ("parity unpinned by the reference");
  parity is anchored on SciPy's outputs.

Operator spec.  Every expression below is written in the exact
operation order used by the C restatement (``oracle/vtk_oracle.c``) and the product
generator (``vt-precondition_amd/csrc/vtk_generate.cpp``), all compiled with
``-ffp-contract=off``, so the three agree bit for bit.
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field

import numpy as np

# ---------------------------------------------------------------------------------------
# Configs (SURVEY.md §8 config key / Appendix A)
# ---------------------------------------------------------------------------------------


@dataclass(frozen=True)
class Vlasov:
    """Synthetic Vlasov operator parameters."""

    dim: int                      # 1, 2 or 4
    shape: tuple                  # (n,) | (Nx, Nv) | (Nx, Ny, Nvx, Nvy)
    vmax: float = 6.0
    E0: float = 0.5
    nu: float = 0.05
    alpha: float = 0.25
    cfl: float = 4.0
    fp32: bool = False            # store values as float32 (C4)

    @property
    def n(self) -> int:
        return int(np.prod(self.shape))

    @property
    def nnz(self) -> int:
        n = self.n
        if self.dim == 1:
            return 3 * n
        if self.dim == 2:
            Nx, Nv = self.shape
            return 5 * n - 2 * Nx
        Nx, Ny, Nvx, Nvy = self.shape
        return 9 * n - 2 * (n // Nvx) - 2 * (n // Nvy)


CONFIGS = {
    "C0": Vlasov(1, (10_000,)),
    "C1": Vlasov(2, (1250, 800)),
    "C2": Vlasov(2, (6250, 800)),
    "C3": Vlasov(2, (25_000, 800)),
    "C4": Vlasov(4, (200, 125, 50, 40), fp32=True),
    # small parity cases
    "S2": Vlasov(2, (64, 32)),
    "S4": Vlasov(4, (6, 5, 8, 8)),
    "S4F": Vlasov(4, (6, 5, 8, 8), fp32=True),
}

RHS_SEED = 0x5EED
M64 = np.uint64(0xFFFFFFFFFFFFFFFF)

# ---------------------------------------------------------------------------------------
# RHS: b[i] = 2 * ((splitmix64(seed + i) >> 11) * 2^-53) - 1      
# ---------------------------------------------------------------------------------------


def splitmix64(state: np.ndarray) -> np.ndarray:
    """splitmix64 output for the given states (uint64, wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        z = state.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def rhs(n: int, seed: int = RHS_SEED, r0: int = 0, r1: int | None = None) -> np.ndarray:
    r1 = n if r1 is None else r1
    st = np.uint64(seed) + np.arange(r0, r1, dtype=np.uint64)
    u = (splitmix64(st) >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)
    return 2.0 * u - 1.0


# ---------------------------------------------------------------------------------------
# Operator generator (canonical CSR, sorted columns, no duplicates)
# ---------------------------------------------------------------------------------------


def _rows_entries(p: Vlasov, r0: int, r1: int):
    """Return (cols[m,K], vals[m,K]) candidate entries for rows [r0, r1); invalid col = -1."""
    r = np.arange(r0, r1, dtype=np.int64)
    m = r1 - r0
    vmax, E0, nu, alpha, cfl = p.vmax, p.E0, p.nu, p.alpha, p.cfl
    if p.dim == 1:
        (n,) = p.shape
        dx = 1.0 / n
        dt = cfl * dx / 1.0
        cx = dt / dx
        v = 1.0
        av = 1.0
        diag = 1.0 + 2.0 * alpha * cx * av
        left = cx * (-0.5 * v - alpha * av)
        right = cx * (0.5 * v - alpha * av)
        cols = np.stack([(r - 1) % n, r, (r + 1) % n], axis=1)
        vals = np.empty((m, 3), dtype=np.float64)
        vals[:, 0] = left
        vals[:, 1] = diag
        vals[:, 2] = right
        return cols, vals
    if p.dim == 2:
        Nx, Nv = p.shape
        i = r // Nv
        j = r % Nv
        dx = 1.0 / Nx
        dv = 2.0 * vmax / Nv
        dt = cfl * dx / vmax
        cx = dt / dx
        cv = dt / dv
        d2 = nu * dt / (dv * dv)
        v = -vmax + (j + 0.5) * dv
        s = (i + 0.5) / Nx
        E = E0 * (1.0 - 4.0 * np.abs(s - 0.5))
        av = np.abs(v)
        aE = np.abs(E)
        diag = 1.0 + 2.0 * alpha * cx * av + 2.0 * alpha * cv * aE + 2.0 * d2
        xl = cx * (-0.5 * v - alpha * av)
        xr = cx * (0.5 * v - alpha * av)
        vl = cv * (-0.5 * E - alpha * aE) - d2
        vr = cv * (0.5 * E - alpha * aE) - d2
        cols = np.stack([((i - 1) % Nx) * Nv + j,
                         np.where(j > 0, r - 1, -1),
                         r,
                         np.where(j < Nv - 1, r + 1, -1),
                         ((i + 1) % Nx) * Nv + j], axis=1)
        vals = np.stack([xl, vl, diag, vr, xr], axis=1)
        return cols, vals
    # 4D
    Nx, Ny, Nvx, Nvy = p.shape
    jy = r % Nvy
    t = r // Nvy
    jx = t % Nvx
    t = t // Nvx
    iy = t % Ny
    ix = t // Ny
    dx = 1.0 / Nx
    dy = 1.0 / Ny
    dvx = 2.0 * vmax / Nvx
    dvy = 2.0 * vmax / Nvy
    dt = cfl * min(dx, dy) / vmax
    cx = dt / dx
    cy = dt / dy
    cvx = dt / dvx
    cvy = dt / dvy
    d2x = nu * dt / (dvx * dvx)
    d2y = nu * dt / (dvy * dvy)
    vx = -vmax + (jx + 0.5) * dvx
    vy = -vmax + (jy + 0.5) * dvy
    sx = (ix + 0.5) / Nx
    sy = (iy + 0.5) / Ny
    Ex = E0 * (1.0 - 4.0 * np.abs(sx - 0.5))
    Ey = E0 * (1.0 - 4.0 * np.abs(sy - 0.5))
    avx = np.abs(vx)
    avy = np.abs(vy)
    aEx = np.abs(Ex)
    aEy = np.abs(Ey)
    diag = (1.0 + 2.0 * alpha * cx * avx + 2.0 * alpha * cy * avy + 2.0 * alpha * cvx * aEx
            + 2.0 * alpha * cvy * aEy + 2.0 * d2x + 2.0 * d2y)
    sx_stride = Ny * Nvx * Nvy
    sy_stride = Nvx * Nvy
    base = r - ix * sx_stride - iy * sy_stride
    cols = np.stack([
        ((ix - 1) % Nx) * sx_stride + iy * sy_stride + base,
        ((ix + 1) % Nx) * sx_stride + iy * sy_stride + base,
        ix * sx_stride + ((iy - 1) % Ny) * sy_stride + base,
        ix * sx_stride + ((iy + 1) % Ny) * sy_stride + base,
        np.where(jx > 0, r - Nvy, -1),
        np.where(jx < Nvx - 1, r + Nvy, -1),
        np.where(jy > 0, r - 1, -1),
        np.where(jy < Nvy - 1, r + 1, -1),
        r], axis=1)
    vals = np.stack([
        cx * (-0.5 * vx - alpha * avx),
        cx * (0.5 * vx - alpha * avx),
        cy * (-0.5 * vy - alpha * avy),
        cy * (0.5 * vy - alpha * avy),
        cvx * (-0.5 * Ex - alpha * aEx) - d2x,
        cvx * (0.5 * Ex - alpha * aEx) - d2x,
        cvy * (-0.5 * Ey - alpha * aEy) - d2y,
        cvy * (0.5 * Ey - alpha * aEy) - d2y,
        diag], axis=1)
    return cols, vals


def generate_rows(p: Vlasov, r0: int, r1: int):
    """CSR rows [r0, r1) with local indptr (starting at 0) and global column indices."""
    cols, vals = _rows_entries(p, r0, r1)
    key = np.where(cols < 0, np.iinfo(np.int64).max, cols)
    order = np.argsort(key, axis=1, kind="stable")
    cols = np.take_along_axis(cols, order, axis=1)
    vals = np.take_along_axis(vals, order, axis=1)
    valid = cols >= 0
    counts = valid.sum(axis=1)
    indptr = np.zeros(r1 - r0 + 1, dtype=np.int64)
    np.cumsum(counts, out=indptr[1:])
    indices = cols[valid].astype(np.int32)
    data = vals[valid]
    if p.fp32:
        data = data.astype(np.float32)
    return indptr, indices, data


def generate(p: Vlasov):
    """Whole operator as (indptr int32, indices int32, data f64|f32)."""
    indptr, indices, data = generate_rows(p, 0, p.n)
    assert indptr[-1] == p.nnz
    assert p.nnz < 2 ** 31
    return indptr.astype(np.int32), indices, data


def csr_sha256(p: Vlasov, chunk: int = 1 << 20) -> dict:
    """SHA-256 of the indptr/indices/data byte streams, generated chunk by chunk."""
    hp, hi, hd = hashlib.sha256(), hashlib.sha256(), hashlib.sha256()
    off = 0
    hp.update(np.zeros(1, np.int32).tobytes())
    for r0 in range(0, p.n, chunk):
        r1 = min(p.n, r0 + chunk)
        ip, ix, dt = generate_rows(p, r0, r1)
        hp.update((ip[1:] + off).astype(np.int32).tobytes())
        hi.update(ix.tobytes())
        hd.update(dt.tobytes())
        off += int(ip[-1])
    return {"indptr": hp.hexdigest(), "indices": hi.hexdigest(), "data": hd.hexdigest(),
            "nnz": off}


# ---------------------------------------------------------------------------------------
# SpMV, block-Jacobi (NumPy/SciPy path)
# ---------------------------------------------------------------------------------------


def scipy_csr(indptr, indices, data, n):
    import scipy.sparse as sp
    A = sp.csr_matrix((data, indices, indptr), shape=(n, n))
    return A


def bj_blocks(indptr, indices, data, n, bs):
    """Dense diagonal blocks, f64[nb, bs, bs] (= the blocks of csr_matrix.toarray()); a short last
    block is padded with identity."""
    nb = (n + bs - 1) // bs
    B = np.zeros((nb, bs, bs), dtype=np.float64)
    ip = np.asarray(indptr, dtype=np.int64)
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(ip))
    cols = np.asarray(indices, dtype=np.int64)
    blk = rows // bs
    m = (cols // bs) == blk
    # duplicates (non-canonical CSR) add up in stored order, as csr_matrix.toarray() does
    np.add.at(B, (blk[m], rows[m] % bs, cols[m] % bs), np.asarray(data, dtype=np.float64)[m])
    tail = n - (nb - 1) * bs
    for t in range(tail, bs):
        B[nb - 1, t, t] = 1.0
    return B


def bj_inverse_numpy(indptr, indices, data, n, bs):
    """Oracle BJ setup: numpy.linalg.inv (LAPACK getrf/getri) on every diagonal block."""
    return np.linalg.inv(bj_blocks(indptr, indices, data, n, bs))


def bj_apply_numpy(Binv, r, n):
    nb, bs, _ = Binv.shape
    rp = np.zeros(nb * bs)
    rp[:n] = r
    return np.einsum("bij,bj->bi", Binv, rp.reshape(nb, bs)).reshape(-1)[:n]


def bj_operator(Binv, n):
    from scipy.sparse.linalg import LinearOperator
    return LinearOperator((n, n), matvec=lambda r: bj_apply_numpy(Binv, np.asarray(r).reshape(-1), n),
                          dtype=np.float64)


# ---------------------------------------------------------------------------------------
# Line Jacobi: x-direction line segments.  M keeps A's diagonal and the
# couplings of rows R, R +- stride whose line index R // stride lies in the same segment of
# `seg` consecutive lines, both rows in [row0, row0 + n).  Restated from the definition
# (SciPy: splu of that matrix) and as the Thomas sweeps oracle/vtk_oracle.c orc_line_setup /
# orc_line_apply perform (same IEEE operation order: bit-identical to the C restatement).
# ---------------------------------------------------------------------------------------


def _line_geometry(indptr, indices, n, stride, seg, row0):
    ip = np.asarray(indptr, dtype=np.int64)
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(ip)) + row0
    cols = np.asarray(indices, dtype=np.int64)
    R = np.arange(row0, row0 + n, dtype=np.int64)

    def has(d):
        Q = R + d * stride
        return (Q >= row0) & (Q < row0 + n) & ((Q // stride) // seg == (R // stride) // seg)

    return rows, cols, R, has(-1), has(1)


def line_matrix(indptr, indices, data, n, stride, seg, row0=0):
    """M as a SciPy CSR matrix (duplicates summed as toarray() does)."""
    import scipy.sparse as sp
    rows, cols, R, hl, hr = _line_geometry(indptr, indices, n, stride, seg, row0)
    r = rows - row0
    keep = (cols == rows) | ((cols == rows - stride) & hl[r]) | ((cols == rows + stride) & hr[r])
    M = sp.coo_matrix((np.asarray(data, np.float64)[keep], (r[keep], cols[keep] - row0)), shape=(n, n))
    return M.tocsr()


def line_factors_numpy(indptr, indices, data, n, stride, seg, row0=0):
    """Thomas factors f = [l | m | g] (vectorised over the lines, ascending line index)."""
    rows, cols, R, hl, hr = _line_geometry(indptr, indices, n, stride, seg, row0)
    v = np.asarray(data, np.float64)
    r = rows - row0
    b = np.zeros(n); a = np.zeros(n); c = np.zeros(n)
    mb = cols == rows
    ma = ~mb & (cols == rows - stride) & hl[r]
    mc = ~mb & ~ma & (cols == rows + stride) & hr[r]
    np.add.at(b, r[mb], v[mb])          # unbuffered: stored order, from 0.0
    np.add.at(a, r[ma], v[ma])
    np.add.at(c, r[mc], v[mc])
    l = np.zeros(n); u = np.zeros(n); m = np.zeros(n); g = np.zeros(n)
    i_lo, i_hi = row0 // stride, (row0 + n - 1) // stride
    with np.errstate(divide="ignore", invalid="ignore"):
        for i in range(i_lo, i_hi + 1):
            lo, hi = max(i * stride, row0) - row0, min((i + 1) * stride, row0 + n) - row0
            k = np.arange(lo, hi)
            first = ~hl[k]
            kp = np.where(first, k, k - stride)
            lv = np.where(first, 0.0, a[k] * m[kp])
            uv = np.where(first, b[k], b[k] - lv * np.where(first, 0.0, c[kp]))
            u[k] = uv
            l[k] = lv
            m[k] = 1.0 / uv
            g[k] = c[k] * m[k]
    bad = (u == 0) | ~np.isfinite(u) | ~np.isfinite(m)
    if n and bad.any():
        raise np.linalg.LinAlgError(f"zero or non-finite line pivot at row {row0 + int(np.argmax(bad))}")
    return np.concatenate([l, m, g])


def line_apply_numpy(f, r, stride, seg, row0=0):
    n = r.shape[0]
    l, m, g = f[:n], f[n:2 * n], f[2 * n:]
    R = np.arange(row0, row0 + n, dtype=np.int64)
    same = lambda d: ((R + d * stride >= row0) & (R + d * stride < row0 + n)
                      & (((R + d * stride) // stride) // seg == (R // stride) // seg))
    hl, hr = same(-1), same(1)
    d = np.zeros(n); z = np.zeros(n)
    i_lo, i_hi = row0 // stride, (row0 + n - 1) // stride
    sl = [np.arange(max(i * stride, row0) - row0, min((i + 1) * stride, row0 + n) - row0)
          for i in range(i_lo, i_hi + 1)]
    for k in sl:
        dp = np.where(hl[k], d[np.maximum(k - stride, 0)], 0.0)
        d[k] = r[k] - l[k] * dp
    for k in reversed(sl):
        zn = np.where(hr[k], z[np.minimum(k + stride, n - 1)], 0.0)
        z[k] = m[k] * d[k] - g[k] * zn
    return z


def line_operator(indptr, indices, data, n, stride, seg):
    """SciPy statement of the preconditioner: a LinearOperator solving with splu(M)."""
    from scipy.sparse.linalg import LinearOperator, splu
    lu = splu(line_matrix(indptr, indices, data, n, stride, seg).tocsc(), permc_spec="NATURAL")
    return LinearOperator((n, n), matvec=lambda r: lu.solve(np.asarray(r, np.float64).reshape(-1)),
                          dtype=np.float64)


@dataclass
class ScipySolve:
    x: np.ndarray
    info: int
    inner_iters: int
    true_resid: float
    b_norm: float
    seconds: float = 0.0
    extra: dict = field(default_factory=dict)


def scipy_gmres(A, b, Binv=None, *, rtol=1e-8, atol=0.0, restart=20, maxiter=None,
                inner_limit=None) -> ScipySolve:
    """The reference scipy.sparse path (iterative.py:582).  ``inner_limit`` bounds the work
    (legacy callback semantics: maxiter counts inner iterations, iterative.py:789-792)."""
    import time
    from scipy.sparse.linalg import gmres
    n = b.shape[0]
    if Binv is None or hasattr(Binv, "matvec"):
        M = Binv                      # None or a LinearOperator (e.g. line_operator)
    else:
        M = bj_operator(Binv, n)
    count = [0]

    def cb(_):
        count[0] += 1

    t0 = time.perf_counter()
    if inner_limit is None:
        x, info = gmres(A, b, rtol=rtol, atol=atol, restart=restart, maxiter=maxiter, M=M,
                        callback=cb, callback_type="pr_norm")
    else:
        x, info = gmres(A, b, rtol=rtol, atol=atol, restart=restart, maxiter=inner_limit, M=M,
                        callback=cb, callback_type="legacy")
    dt = time.perf_counter() - t0
    res = float(np.linalg.norm(b - A @ x))
    return ScipySolve(x=x, info=int(info), inner_iters=count[0], true_resid=res,
                      b_norm=float(np.linalg.norm(b)), seconds=dt)
