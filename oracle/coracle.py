"""ctypes wrapper over oracle/lib/libvtk_oracle.so — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module.  The C restatement it wraps (``oracle/vtk_oracle.c``) is the checker
the GPU parity tests run against on the GPU box, where ``/root/reference`` does not exist;
it is itself pinned to SciPy-generated golden vectors (``tests/golden``).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "lib", "libvtk_oracle.so")


class _Vlasov(C.Structure):
    _fields_ = [("dim", C.c_int), ("fp32", C.c_int), ("shape", C.c_int64 * 4),
                ("vmax", C.c_double), ("E0", C.c_double), ("nu", C.c_double),
                ("alpha", C.c_double), ("cfl", C.c_double)]


class _Stats(C.Structure):
    _fields_ = [("inner_iters", C.c_int64), ("restarts", C.c_int64),
                ("presid", C.c_double), ("rnorm", C.c_double)]


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = C.CDLL(_LIB)
        P = C.c_void_p
        L.orc_generate.argtypes = [C.POINTER(_Vlasov), C.c_int64, C.c_int64, P, P, P]
        L.orc_rhs.argtypes = [C.c_uint64, C.c_int64, C.c_int64, P]
        L.orc_spmv.argtypes = [C.c_int64, P, P, P, C.c_int, P, P]
        L.orc_bj_setup.argtypes = [C.c_int64, P, P, P, C.c_int, C.c_int, P]
        L.orc_bj_setup.restype = C.c_int64
        L.orc_bj_apply.argtypes = [C.c_int64, C.c_int, P, P, P]
        L.orc_lartg.argtypes = [C.c_double, C.c_double, C.POINTER(C.c_double),
                                C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.orc_gmres.argtypes = [C.c_int64, P, P, P, C.c_int, P, C.c_int, P, P, C.c_double,
                                C.c_double, C.c_int, C.c_int64, C.POINTER(C.c_int),
                                C.POINTER(_Stats)]
        L.orc_line_setup.argtypes = [C.c_int64, P, P, P, C.c_int, C.c_int64, C.c_int64, C.c_int64, P]
        L.orc_line_setup.restype = C.c_int64
        L.orc_line_apply.argtypes = [C.c_int64, C.c_int64, C.c_int64, C.c_int64, P, P, P]
        L.orc_gmres_line.argtypes = [C.c_int64, P, P, P, C.c_int, P, C.c_int64, C.c_int64, P, P,
                                     C.c_double, C.c_double, C.c_int, C.c_int64,
                                     C.POINTER(C.c_int), C.POINTER(_Stats)]
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _params(p) -> _Vlasov:
    s = (C.c_int64 * 4)(*(list(p.shape) + [0] * (4 - len(p.shape))))
    return _Vlasov(p.dim, int(p.fp32), s, p.vmax, p.E0, p.nu, p.alpha, p.cfl)


def generate(p, r0: int = 0, r1: int | None = None):
    r1 = p.n if r1 is None else r1
    # upper bound of the row block's nnz: 9 per row
    cap = (r1 - r0) * (3 if p.dim == 1 else 5 if p.dim == 2 else 9)
    indptr = np.empty(r1 - r0 + 1, np.int32)
    indices = np.empty(cap, np.int32)
    data = np.empty(cap, np.float32 if p.fp32 else np.float64)
    lib().orc_generate(C.byref(_params(p)), r0, r1, _ptr(indptr), _ptr(indices), _ptr(data))
    nnz = int(indptr[-1])
    return indptr, indices[:nnz].copy(), data[:nnz].copy()


def rhs(n: int, seed: int = 0x5EED, r0: int = 0, r1: int | None = None):
    r1 = n if r1 is None else r1
    b = np.empty(r1 - r0, np.float64)
    lib().orc_rhs(seed, r0, r1, _ptr(b))
    return b


def spmv(indptr, indices, data, x):
    n = indptr.shape[0] - 1
    y = np.empty(n, np.float64)
    lib().orc_spmv(n, _ptr(indptr), _ptr(indices), _ptr(data), int(data.dtype == np.float32),
                   _ptr(np.ascontiguousarray(x, np.float64)), _ptr(y))
    return y


def bj_setup(indptr, indices, data, bs: int):
    n = indptr.shape[0] - 1
    nb = (n + bs - 1) // bs
    inv = np.empty((nb, bs, bs), np.float64)
    rc = lib().orc_bj_setup(n, _ptr(indptr), _ptr(indices), _ptr(data),
                            int(data.dtype == np.float32), bs, _ptr(inv))
    if rc != 0:
        raise np.linalg.LinAlgError(f"singular diagonal block {-rc - 1}")
    return inv


def bj_apply(inv, r):
    nb, bs, _ = inv.shape
    n = r.shape[0]
    z = np.empty(n, np.float64)
    lib().orc_bj_apply(n, bs, _ptr(inv), _ptr(np.ascontiguousarray(r, np.float64)), _ptr(z))
    return z


class LineFactors:
    """Line-Jacobi factors ``f = [l | m | g]`` of rows [row0, row0+n) (orc_line_setup)."""

    def __init__(self, f, row0: int, stride: int, seg: int):
        self.f, self.row0, self.stride, self.seg = f, row0, stride, seg


def line_setup(indptr, indices, data, stride: int, seg: int, row0: int = 0) -> LineFactors:
    """``indices`` are GLOBAL columns of the row block [row0, row0 + n)."""
    n = indptr.shape[0] - 1
    f = np.empty(3 * max(n, 1), np.float64)[:3 * n]
    rc = lib().orc_line_setup(n, _ptr(indptr), _ptr(indices), _ptr(data),
                              int(data.dtype == np.float32), row0, stride, seg, _ptr(f))
    if rc != 0:
        raise np.linalg.LinAlgError(f"zero or non-finite line pivot at row {row0 - rc - 1}")
    return LineFactors(f, row0, stride, seg)


def line_apply(lf: LineFactors, r):
    n = r.shape[0]
    z = np.empty(n, np.float64)
    lib().orc_line_apply(n, lf.row0, lf.stride, lf.seg, _ptr(lf.f),
                         _ptr(np.ascontiguousarray(r, np.float64)), _ptr(z))
    return z


def lartg(f: float, g: float):
    c, s, r = C.c_double(), C.c_double(), C.c_double()
    lib().orc_lartg(f, g, C.byref(c), C.byref(s), C.byref(r))
    return c.value, s.value, r.value


@dataclass
class Solve:
    x: np.ndarray
    info: int
    inner_iters: int
    restarts: int
    presid: float
    rnorm: float


def gmres(indptr, indices, data, b, inv=None, *, x0=None, rtol=1e-5, atol=0.0, restart=20,
          maxiter=None) -> Solve:
    """``inv``: None, block inverses (bj_setup) or LineFactors (line_setup, row0 = 0)."""
    n = b.shape[0]
    x = np.zeros(n) if x0 is None else np.array(x0, np.float64, copy=True)
    if isinstance(inv, LineFactors):
        info = C.c_int()
        st = _Stats()
        lib().orc_gmres_line(n, _ptr(indptr), _ptr(indices), _ptr(data), int(data.dtype == np.float32),
                             _ptr(inv.f), inv.stride, inv.seg, _ptr(np.ascontiguousarray(b, np.float64)),
                             _ptr(x), rtol, atol, restart, 0 if maxiter is None else maxiter,
                             C.byref(info), C.byref(st))
        return Solve(x, info.value, st.inner_iters, st.restarts, st.presid, st.rnorm)
    bs = 0 if inv is None else inv.shape[1]
    info = C.c_int()
    st = _Stats()
    lib().orc_gmres(n, _ptr(indptr), _ptr(indices), _ptr(data), int(data.dtype == np.float32),
                    _ptr(inv), bs, _ptr(np.ascontiguousarray(b, np.float64)), _ptr(x), rtol, atol,
                    restart, 0 if maxiter is None else maxiter, C.byref(info), C.byref(st))
    return Solve(x, info.value, st.inner_iters, st.restarts, st.presid, st.rnorm)
