"""vtkrylov — MI355X-native preconditioned Krylov path (CSR SpMV + block-Jacobi + GMRES).

Drop-in for the north_star's "reference scipy.sparse path" (SURVEY.md §8b): the callables
below keep SciPy's names, argument meaning and error behaviour, and route every operation to
the gfx950 kernels of ``libvtkrylov.so`` through the C-ABI in ``include/vtkrylov.h``.

    scipy.sparse.csr_matrix((data, indices, indptr), shape)  ->  vtkrylov.csr_matrix(...)
    A @ x                                                    ->  A @ x   (vtk_spmv)
    LinearOperator(matvec=block-Jacobi)                      ->  vtkrylov.block_jacobi(A, bs)
    scipy.sparse.linalg.gmres(A, b, x0, rtol=, atol=,        ->  vtkrylov.gmres(...)
                              restart=, maxiter=, M=)           (iterative.py:582-841)

Vectors may be NumPy arrays (host; copied in and out) or torch CUDA tensors (device memory,
used in place).  There is no CPU fallback: without the library or a HIP device every call
raises.
"""
from __future__ import annotations

import atexit
import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _abi
from ._abi import check, lib

__all__ = ["Context", "default_context", "csr_matrix", "load_npz", "save_npz", "vlasov_operator", "block_jacobi",
           "gmres", "VlasovParams", "vlasov_params", "rhs_splitmix", "partition_rows",
           "halo_plan", "device_count", "SolveStats", "line_jacobi", "LineJacobi",
           "vlasov_line_stride"]

VlasovParams = _abi.VlasovParams

# At interpreter exit the finalizers below may run in any order (a context before the operators
# that use it); the process is ending, so they leave the native objects to the runtime.
_exiting = [False]
atexit.register(lambda: _exiting.__setitem__(0, True))


def vlasov_params(dim: int, shape, *, fp32=False, vmax=6.0, E0=0.5, nu=0.05, alpha=0.25,
                  cfl=4.0) -> VlasovParams:
    s = list(shape) + [0] * (4 - len(shape))
    return VlasovParams(int(dim), int(bool(fp32)), (C.c_int64 * 4)(*s), vmax, E0, nu, alpha, cfl)


def device_count() -> int:
    n = C.c_int()
    lib().vtk_device_count(C.byref(n))
    return n.value


def _np_ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def _is_torch_cuda(x) -> bool:
    t = type(x)
    return t.__module__.startswith("torch") and getattr(x, "is_cuda", False)


class _Vec:
    """A vector argument: NumPy (host, kind=HOST) or torch CUDA tensor (device, kind=DEVICE)."""

    def __init__(self, x, n: int, writable=False):
        if _is_torch_cuda(x):
            import torch
            if x.dtype != torch.float64 or not x.is_contiguous() or x.numel() != n:
                raise ValueError("device vectors must be contiguous float64 tensors of length n")
            torch.cuda.current_stream(x.device).synchronize()
            self.kind = _abi.PTR_DEVICE
            self.ptr = C.c_void_p(x.data_ptr())
            self.obj = x
        else:
            a = np.ascontiguousarray(x, dtype=np.float64).reshape(-1)
            if a.shape[0] != n:
                raise ValueError(f"vector has length {a.shape[0]}, expected {n}")
            if writable and not a.flags.writeable:
                a = a.copy()
            self.kind = _abi.PTR_HOST
            self.ptr = _np_ptr(a)
            self.obj = a


class Context:
    """One HIP device + stream (+ optional RCCL communicator).  ``vtk_ctx_create``."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        check(lib().vtk_ctx_create(int(device), C.byref(h)))
        self._h = h
        self.device = device
        self.rank, self.world = 0, 1

    @property
    def handle(self):
        return self._h

    def stream_ptr(self) -> int:
        s = C.c_void_p()
        check(lib().vtk_ctx_stream(self._h, C.byref(s)), self._h)
        return s.value or 0

    def synchronize(self):
        check(lib().vtk_ctx_synchronize(self._h), self._h)

    def comm_init(self, rank: int, world: int, unique_id: bytes | None):
        buf = None if unique_id is None else C.create_string_buffer(bytes(unique_id), 128)
        check(lib().vtk_comm_init(self._h, rank, world, buf), self._h)
        self.rank, self.world = rank, world

    def rccl_ranks(self) -> int:
        """Ranks of the RCCL communicator (ncclCommCount); 0 without one."""
        n = C.c_int()
        check(lib().vtk_comm_rccl_count(self._h, C.byref(n)), self._h)
        return n.value

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        check(lib().vtk_comm_unique_id(buf))
        return buf.raw

    def comm_init_host(self, rank: int, world: int, group=None):
        """Host-staged communicator over torch.distributed (tests; ranks may share a GPU)."""
        from .comm import init_host
        return init_host(self, rank, world, group)

    def profile(self, on: bool = True):
        """Enable (and clear) / disable the per-kernel-class event profile."""
        check(lib().vtk_profile_enable(self._h, int(bool(on))), self._h)

    def profile_read(self) -> dict:
        """{class: {launches, seconds, bytes, avg_us, gbs}} from the event profile."""
        n = C.c_int()
        check(lib().vtk_profile_read(self._h, None, 0, C.byref(n)), self._h)
        arr = (_abi.KernelProfile * max(n.value, 1))()
        check(lib().vtk_profile_read(self._h, arr, n.value, C.byref(n)), self._h)
        out = {}
        for e in arr[:n.value]:
            if e.launches:
                out[e.name.decode()] = {"launches": e.launches, "seconds": e.seconds, "bytes": e.bytes,
                                        "avg_us": e.seconds / e.launches * 1e6,
                                        "gbs": e.bytes / e.seconds / 1e9 if e.seconds > 0 else 0.0}
        return out

    orth = _abi.ORTH_AUTO

    def set_orth(self, orth: int):
        check(lib().vtk_gmres_set_orth(self._h, int(orth)), self._h)
        self.orth = int(orth)

    def set_tuning(self, key: str, value: int):
        """A/B and test switch of this context (``vtk_ctx_set_tuning``; keys in
        include/vtkrylov.h).  Seeded from ``VTK_<KEY>`` when the context was created."""
        check(lib().vtk_ctx_set_tuning(self._h, key.encode(), int(value)), self._h)

    def get_tuning(self, key: str) -> int:
        v = C.c_int()
        check(lib().vtk_ctx_get_tuning(self._h, key.encode(), C.byref(v)), self._h)
        return v.value

    def tuning(self, **kv):
        """``with ctx.tuning(band_lsv=0): ...`` -- set switches for a block, then restore."""
        import contextlib

        @contextlib.contextmanager
        def cm():
            old = {k: self.get_tuning(k) for k in kv}
            try:
                for k, v in kv.items():
                    self.set_tuning(k, v)
                yield self
            finally:
                for k, v in old.items():
                    self.set_tuning(k, v)
        return cm()

    band = True

    def set_band(self, on: bool):
        """Allow (default) or forbid the line-band DCGS2 step (see csr_matrix.set_line_band)."""
        check(lib().vtk_gmres_set_band(self._h, 1 if on else 0), self._h)
        self.band = bool(on)

    def close(self):
        if getattr(self, "_h", None):
            lib().vtk_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        if _exiting[0]:
            return
        try:
            self.close()
        except Exception:
            pass


_default = {}


def default_context(device: int = 0) -> Context:
    if device not in _default:
        _default[device] = Context(device)
    return _default[device]


class CsrOperator:
    """Device-resident CSR operator (this rank's row block).  ``vtk_csr_create``."""

    def __init__(self, handle, ctx: Context, fp32: bool):
        self._h = handle
        self.ctx = ctx
        self.fp32 = bool(fp32)
        ng, rb, re_, nnz, nh = (C.c_int64() for _ in range(5))
        check(lib().vtk_csr_info(handle, C.byref(ng), C.byref(rb), C.byref(re_), C.byref(nnz),
                                 C.byref(nh)), ctx.handle)
        self.n_global, self.row_begin, self.row_end = ng.value, rb.value, re_.value
        self.nnz, self.n_halo = nnz.value, nh.value
        self.n_local = self.row_end - self.row_begin
        self.shape = (self.n_global, self.n_global)
        self.dtype = np.dtype(np.float64)

    @property
    def handle(self):
        return self._h

    LAYOUTS = {"auto": 0, "csr": 1, "sell": 2, "sell32": 3}

    def set_layout(self, layout: str):
        """SpMV layout: "sell" (SELL-64 copy, columns dictionary-coded per 64-row chunk),
        "sell32" (SELL-64 with int32 columns), "csr" (CSR-stream tiles) or "auto" ("sell" when
        its padding is <= 25 % of nnz).  Results are bit-identical in every layout."""
        check(lib().vtk_csr_set_layout(self._h, self.LAYOUTS[layout]), self.ctx.handle)

    @property
    def layout(self) -> str:
        v = C.c_int()
        check(lib().vtk_csr_get_layout(self._h, C.byref(v)), self.ctx.handle)
        return {1: "csr", 2: "sell", 3: "sell32"}[v.value]

    def set_line_band(self, line_len: int):
        """Declare the line-band structure: rows form x-lines of ``line_len`` rows and every
        column lies in the lines x-1..x+1 (periodic) of its row's line (checked on the device;
        0 clears it).  The 2D Vlasov operators get it automatically (line_len = Nv).  gmres then
        fuses each DCGS2 update pass with the next step's SpMV + BJ + dots (one basis read per
        step); results stay within the DCGS2 bars."""
        check(lib().vtk_csr_set_line_band(self._h, int(line_len)), self.ctx.handle)

    @property
    def line_band(self) -> int:
        v = C.c_int64()
        check(lib().vtk_csr_get_line_band(self._h, C.byref(v)), self.ctx.handle)
        return v.value

    @property
    def line_separable(self) -> bool:
        """True when the band step reads the values from per-position / per-line tables (the
        operator's x couplings depend only on v, its v couplings only on x; checked bit for bit
        when the band was set -- vtk_csr_get_line_values)."""
        return self.line_values > 0

    @property
    def line_values(self) -> int:
        """0: SELL values; 1: line-separable values; 2: also canonical rows (no column codes read
        by the band step) -- vtk_csr_get_line_values."""
        v = C.c_int()
        check(lib().vtk_csr_get_line_values(self._h, C.byref(v)), self.ctx.handle)
        return v.value

    def set_grid4(self, Ny: int, Nvx: int, Nvy: int):
        """Declare the 4D phase-space grid structure (vtk_csr_set_grid4; checked on the device, Ny 0
        clears it).  The 4D Vlasov operators get it automatically, also when uploaded as a CSR."""
        check(lib().vtk_csr_set_grid4(self._h, int(Ny), int(Nvx), int(Nvy)), self.ctx.handle)

    @property
    def grid4(self) -> tuple:
        """(Ny, Nvx, Nvy) of the verified 4D grid structure, (0, 0, 0) when not set."""
        v = (C.c_int64 * 3)()
        check(lib().vtk_csr_get_grid4(self._h, v), self.ctx.handle)
        return tuple(int(t) for t in v)

    def layout_info(self) -> dict:
        """Layout in use, bytes of the operator one SpMV reads in it, SELL chunk counts."""
        li = _abi.LayoutInfo()
        check(lib().vtk_csr_layout_info(self._h, C.byref(li)), self.ctx.handle)
        d = {k: getattr(li, k) for k, _ in li._fields_}
        d["layout"] = {1: "csr", 2: "sell", 3: "sell32"}[d["layout"]]
        return d

    def matvec(self, x):
        """y = A x on this rank's rows (sparsetools csr_matvec, bit-identical)."""
        vx = _Vec(x, self.n_local)
        if vx.kind == _abi.PTR_DEVICE:
            import torch
            y = torch.empty_like(vx.obj)
            check(lib().vtk_spmv(self._h, vx.ptr, C.c_void_p(y.data_ptr()), vx.kind), self.ctx.handle)
            self.ctx.synchronize()
            return y
        y = np.empty(self.n_local)
        check(lib().vtk_spmv(self._h, vx.ptr, _np_ptr(y), vx.kind), self.ctx.handle)
        return y

    def __matmul__(self, x):
        return self.matvec(x)

    def dot(self, x):
        return self.matvec(x)

    def precond_matvec(self, M, x):
        """w = M^-1 (A x) through the launch the solver's split DCGS2 step uses for this operator
        (SciPy: ``M.matvec(A @ x)``; vtk_precond_matvec).  M: a BlockJacobi / LineJacobi of this
        operator, or None (w = A x)."""
        vx = _Vec(x, self.n_local)
        mh = M.handle if M is not None else None
        if vx.kind == _abi.PTR_DEVICE:
            import torch
            w = torch.empty_like(vx.obj)
            check(lib().vtk_precond_matvec(self._h, mh, vx.ptr, C.c_void_p(w.data_ptr()), vx.kind), self.ctx.handle)
            self.ctx.synchronize()
            return w
        w = np.empty(self.n_local)
        check(lib().vtk_precond_matvec(self._h, mh, vx.ptr, _np_ptr(w), vx.kind), self.ctx.handle)
        return w

    def download(self):
        """(indptr, indices[global], data) of this rank's rows, as stored on the device."""
        ip = np.empty(self.n_local + 1, np.int32)
        ix = np.empty(max(self.nnz, 1), np.int32)
        d = np.empty(max(self.nnz, 1), np.float32 if self.fp32 else np.float64)
        check(lib().vtk_csr_download(self._h, _np_ptr(ip), _np_ptr(ix), _np_ptr(d)), self.ctx.handle)
        return ip, ix[:self.nnz], d[:self.nnz]

    def close(self):
        if getattr(self, "_h", None):
            lib().vtk_csr_destroy(self._h)
            self._h = None

    def __del__(self):
        if _exiting[0]:
            return
        try:
            self.close()
        except Exception:
            pass


def _is_device(a) -> bool:
    return getattr(a, "is_cuda", False) is True


def _apply_line_len(A: CsrOperator, line_len):
    """line_len None: keep what vtk_csr_create detected (the 2D Vlasov x-lines are found in
    the CSR itself); 0: no line band; L: require the line band of L rows (ValueError if the
    operator does not have it)."""
    if line_len is None:
        return A
    if int(line_len) != A.line_band:
        A.set_line_band(int(line_len))
    return A


def csr_matrix(arg, shape=None, *, ctx: Context | None = None, offsets=None, line_len=None) -> CsrOperator:
    """Build a device CSR operator from ``(data, indices, indptr)`` or a SciPy sparse matrix.

    With ``offsets`` (world+1 row boundaries) the arrays are this rank's row block with
    global column indices (multi-GPU); otherwise the whole matrix.  The library looks for the
    x-line structure of the 2D Vlasov operators in the CSR (``line_len=None``, the default) and
    then runs the same fused solver as for a generated operator; ``line_len=0`` turns that off,
    an explicit ``line_len`` requires it (see :meth:`CsrOperator.set_line_band`)."""
    ctx = ctx or default_context()
    if hasattr(arg, "tocsr"):
        # stored order kept: csr_matvec sums each row in stored order, so must the device
        m = arg.tocsr()
        data, indices, indptr = m.data, m.indices, m.indptr
        shape = m.shape
    else:
        data, indices, indptr = arg
    if shape is None or shape[0] != shape[1]:
        raise ValueError("a square shape is required")
    if _is_device(data) or _is_device(indices) or _is_device(indptr):
        # CSR already in HBM (torch tensors on the context's device): no host round trip; the
        # library validates indptr (host copy) and the column range (device reduction)
        import torch
        if not (_is_device(data) and _is_device(indices) and _is_device(indptr)):
            raise TypeError("csr_matrix: data, indices and indptr must all be device tensors or all host arrays")
        for t in (data, indices, indptr):
            if t.device.index != ctx.device:
                raise ValueError(f"csr_matrix: tensor on {t.device}, the context is on cuda:{ctx.device}")
        fp32 = data.dtype == torch.float32
        data = data.contiguous().to(torch.float32 if fp32 else torch.float64)
        indices = indices.contiguous().to(torch.int32)
        indptr = indptr.contiguous().to(torch.int32)
        # the conversions above run on torch's current stream; the library copies with
        # hipMemcpy on its own: let them finish first
        torch.cuda.current_stream(data.device).synchronize()
        nnz = int(indptr[-1].item())   # the CSR may carry spare capacity beyond indptr[-1]
        offs = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.int64)
        # the library copies nnz entries device to device: never past the tensors' ends
        n_rows = int(shape[0]) if offs is None else int(offs[ctx.rank + 1] - offs[ctx.rank])
        if indptr.numel() != n_rows + 1:
            raise ValueError(f"csr_matrix: indptr has {indptr.numel()} entries, expected {n_rows + 1}")
        if nnz < 0 or nnz > indices.numel() or nnz > data.numel():
            raise ValueError(f"csr_matrix: indptr[-1] = {nnz} exceeds the {indices.numel()} indices / "
                             f"{data.numel()} values given")
        h = C.c_void_p()
        check(lib().vtk_csr_create(ctx.handle, int(shape[0]), None if offs is None else _np_ptr(offs),
                                   nnz, C.c_void_p(indptr.data_ptr()),
                                   C.c_void_p(indices.data_ptr()), C.c_void_p(data.data_ptr()),
                                   int(fp32), _abi.PTR_DEVICE, C.byref(h)), ctx.handle)
        return _apply_line_len(CsrOperator(h, ctx, fp32), line_len)
    data = np.asarray(data)
    fp32 = data.dtype == np.float32
    data = np.ascontiguousarray(data, dtype=np.float32 if fp32 else np.float64)
    indices = np.ascontiguousarray(indices, dtype=np.int32)
    indptr = np.ascontiguousarray(indptr, dtype=np.int32)
    offs = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.int64)
    nnz = int(indptr[-1])
    n_rows = int(shape[0]) if offs is None else int(offs[ctx.rank + 1] - offs[ctx.rank])
    if indptr.shape[0] != n_rows + 1:
        raise ValueError(f"csr_matrix: indptr has {indptr.shape[0]} entries, expected {n_rows + 1}")
    if nnz < 0 or nnz > indices.shape[0] or nnz > data.shape[0]:
        raise ValueError(f"csr_matrix: indptr[-1] = {nnz} exceeds the {indices.shape[0]} indices / "
                         f"{data.shape[0]} values given")
    h = C.c_void_p()
    check(lib().vtk_csr_create(ctx.handle, int(shape[0]), None if offs is None else _np_ptr(offs),
                               nnz, _np_ptr(indptr), _np_ptr(indices), _np_ptr(data),
                               int(fp32), _abi.PTR_HOST, C.byref(h)), ctx.handle)
    return _apply_line_len(CsrOperator(h, ctx, fp32), line_len)


def load_npz(file, *, ctx: Context | None = None, offsets=None, line_len=None) -> CsrOperator:
    """``scipy.sparse.load_npz`` for CSR archives, straight to the device: with ``offsets``
    (world+1 row boundaries) each rank reads only its row block (``ctx.rank``).  ``line_len``
    as in :func:`csr_matrix`."""
    from .npz import load_npz_arrays
    ctx = ctx or default_context()
    rows = None
    if offsets is not None:
        offs = np.asarray(offsets, dtype=np.int64)
        if offs.shape != (ctx.world + 1,):
            raise ValueError("offsets must have world+1 entries")
        rows = (int(offs[ctx.rank]), int(offs[ctx.rank + 1]))
    indptr, indices, data, shape = load_npz_arrays(file, rows)
    return csr_matrix((data, indices, indptr), shape=shape, ctx=ctx, offsets=offsets, line_len=line_len)


def save_npz(file, A: CsrOperator, compressed: bool = True) -> None:
    """``scipy.sparse.save_npz`` of a whole (single-rank) device operator, entries in stored
    order; a row-sharded operator is saved per rank with ``npz.save_npz_arrays`` on
    ``A.download()`` (global column ids) and concatenated by the caller."""
    from .npz import save_npz_arrays
    if A.n_local != A.n_global:
        raise ValueError("save_npz needs the whole matrix on this rank (row-sharded operator)")
    indptr, indices, data = A.download()
    save_npz_arrays(file, indptr, indices, data, A.shape, compressed)


def vlasov_operator(params: VlasovParams, *, ctx: Context | None = None, offsets=None) -> CsrOperator:
    """Generate the Appendix-A Vlasov operator directly in device memory."""
    ctx = ctx or default_context()
    offs = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.int64)
    h = C.c_void_p()
    check(lib().vtk_csr_create_vlasov(ctx.handle, C.byref(params),
                                      None if offs is None else _np_ptr(offs), C.byref(h)), ctx.handle)
    return CsrOperator(h, ctx, bool(params.fp32))


BJ_MODES = {"auto": 0, "inverse": 1, "tridiag": 2}


class BlockJacobi:
    """Block-Jacobi preconditioner M = blockdiag(A)^-1 (SciPy: a LinearOperator whose matvec
    applies the bs x bs diagonal-block inverses).  ``vtk_bjacobi_create``.

    ``mode``: how M^-1 is applied (same operator either way): "inverse" multiplies by the
    block inverses (bit-identical to the oracle with setup "exact"), "tridiag" solves with the LU factors of
    tridiagonal blocks (bs 2/4/8; 24 B/row instead of 8*bs), "auto" (default) takes "tridiag"
    when every block is tridiagonal and its factors pass the setup check.

    ``setup``: how the inverses are computed: "exact" (default, as ``vtk_bjacobi_create``:
    Gauss-Jordan with partial pivoting, bit-identical to the oracle), "mfma" (bs 16 / 32: blocked
    Gauss-Jordan with the rank-4 panel updates on the fp64 matrix cores; same pivot rule,
    rounding-level differences) or "auto" ("mfma" for bs 16 and 32, 2.3x / 4.7x faster at C3,
    else "exact")."""

    SETUPS = {"exact": 0, "mfma": 1, "auto": 2}

    def __init__(self, A: CsrOperator, bs: int = 8, mode: str = "auto", setup: str = "exact"):
        if mode not in BJ_MODES:
            raise ValueError(f"mode must be one of {sorted(BJ_MODES)}")
        if setup not in self.SETUPS:
            raise ValueError(f"setup must be one of {sorted(self.SETUPS)}")
        h = C.c_void_p()
        check(lib().vtk_bjacobi_create_ex(A.handle, int(bs), self.SETUPS[setup], C.byref(h)), A.ctx.handle)
        self._h = h
        self.A = A
        self.bs = bs
        self.shape = A.shape
        self.dtype = np.dtype(np.float64)
        self.set_mode(mode)

    def set_mode(self, mode: str):
        check(lib().vtk_bjacobi_set_mode(self._h, BJ_MODES[mode]), self.A.ctx.handle)

    @property
    def mode(self) -> str:
        """The apply in use: "inverse" or "tridiag"."""
        m = C.c_int()
        check(lib().vtk_bjacobi_get_mode(self._h, C.byref(m), None), self.A.ctx.handle)
        return {1: "inverse", 2: "tridiag"}[m.value]

    @property
    def tridiag_available(self) -> bool:
        t = C.c_int()
        check(lib().vtk_bjacobi_get_mode(self._h, None, C.byref(t)), self.A.ctx.handle)
        return bool(t.value)

    @property
    def handle(self):
        return self._h

    def inverse(self) -> np.ndarray:
        nb = (self.A.n_local + self.bs - 1) // self.bs
        inv = np.empty((nb, self.bs, self.bs))
        check(lib().vtk_bjacobi_inverse(self._h, _np_ptr(inv), _abi.PTR_HOST), self.A.ctx.handle)
        return inv

    def matvec(self, r):
        vr = _Vec(r, self.A.n_local)
        if vr.kind == _abi.PTR_DEVICE:
            import torch
            z = torch.empty_like(vr.obj)
            check(lib().vtk_bjacobi_apply(self._h, vr.ptr, C.c_void_p(z.data_ptr()), vr.kind), self.A.ctx.handle)
            self.A.ctx.synchronize()
            return z
        z = np.empty(self.A.n_local)
        check(lib().vtk_bjacobi_apply(self._h, vr.ptr, _np_ptr(z), vr.kind), self.A.ctx.handle)
        return z

    def __matmul__(self, r):
        return self.matvec(r)

    def close(self):
        if getattr(self, "_h", None):
            lib().vtk_prec_destroy(self._h)
            self._h = None

    def __del__(self):
        if _exiting[0]:
            return
        try:
            self.close()
        except Exception:
            pass


def block_jacobi(A: CsrOperator, bs: int = 8, mode: str = "auto", setup: str = "exact") -> BlockJacobi:
    return BlockJacobi(A, bs, mode, setup)


class LineJacobi:
    """Line-Jacobi preconditioner (line-implicit x-direction solve):
    M = A's diagonal + the couplings between rows R and R +- ``stride`` within segments of
    ``seg`` consecutive line indices R // stride (and within this rank's rows).  SciPy
    statement: ``LinearOperator(matvec=splu(M).solve)``.  ``vtk_linejacobi_create``.

    For the Vlasov operators ``stride`` = 1 (1D), Nv (2D), Ny*Nvx*Nvy (4D): see
    :func:`vlasov_line_stride`.  Choose ``seg`` dividing Nx / world so that M does not depend
    on the number of ranks."""

    def __init__(self, A: CsrOperator, stride: int, seg: int = 25):
        h = C.c_void_p()
        check(lib().vtk_linejacobi_create(A.handle, int(stride), int(seg), C.byref(h)), A.ctx.handle)
        self._h = h
        self.A = A
        self.stride = int(stride)
        self.seg = int(seg)
        self.shape = A.shape
        self.dtype = np.dtype(np.float64)

    @property
    def handle(self):
        return self._h

    @property
    def compact(self) -> bool:
        """Apply forms l and g from the lines' constant x-couplings (reads only m)."""
        u = C.c_int()
        check(lib().vtk_linejacobi_get_compact(self._h, C.byref(u), None), self.A.ctx.handle)
        return bool(u.value)

    @property
    def compact_available(self) -> bool:
        a = C.c_int()
        check(lib().vtk_linejacobi_get_compact(self._h, None, C.byref(a)), self.A.ctx.handle)
        return bool(a.value)

    def set_compact(self, on: bool):
        check(lib().vtk_linejacobi_set_compact(self._h, int(bool(on))), self.A.ctx.handle)

    def factors(self) -> np.ndarray:
        """l | m | g, 3 * n_local doubles (the oracle's orc_line_setup layout)."""
        f = np.empty(3 * self.A.n_local)
        check(lib().vtk_linejacobi_factors(self._h, _np_ptr(f), _abi.PTR_HOST), self.A.ctx.handle)
        return f

    def matvec(self, r):
        vr = _Vec(r, self.A.n_local)
        if vr.kind == _abi.PTR_DEVICE:
            import torch
            z = torch.empty_like(vr.obj)
            check(lib().vtk_prec_apply(self._h, vr.ptr, C.c_void_p(z.data_ptr()), vr.kind), self.A.ctx.handle)
            self.A.ctx.synchronize()
            return z
        z = np.empty(self.A.n_local)
        check(lib().vtk_prec_apply(self._h, vr.ptr, _np_ptr(z), vr.kind), self.A.ctx.handle)
        return z

    def __matmul__(self, r):
        return self.matvec(r)

    def close(self):
        if getattr(self, "_h", None):
            lib().vtk_prec_destroy(self._h)
            self._h = None

    def __del__(self):
        if _exiting[0]:
            return
        try:
            self.close()
        except Exception:
            pass


def line_jacobi(A: CsrOperator, stride: int, seg: int = 25) -> LineJacobi:
    return LineJacobi(A, stride, seg)


def vlasov_line_stride(params) -> int:
    """Rows between x-neighbours of a Vlasov operator: 1 (1D), Nv (2D), Ny*Nvx*Nvy (4D)."""
    dim = int(params.dim)
    sh = [int(v) for v in params.shape]
    if dim == 1:
        return 1
    if dim == 2:
        return sh[1]
    return sh[1] * sh[2] * sh[3]


@dataclass
class SolveStats:
    inner_iters: int
    restarts: int
    presid: float
    rnorm: float
    bnorm: float
    atol_eff: float
    t_solve: float
    bytes_moved: float
    breakdown: int
    orth: int
    band: int = 0   # 1: the line-band DCGS2 step ran


_last_stats: SolveStats | None = None


def last_stats() -> SolveStats | None:
    return _last_stats


def gmres(A, b, x0=None, *, rtol=1e-5, atol=0., restart=None, maxiter=None, M=None,
          callback=None, callback_type=None, orth=None):
    """``scipy.sparse.linalg.gmres`` on the GPU (iterative.py:582-841, left-preconditioned
    restarted GMRES: SciPy's control flow, ptol schedule, ``dlartg`` Givens rotations and
    ``info`` convention).  Returns ``(x, info)``.

    Orthogonalisation: the DEFAULT (``orth=None``/``"auto"`` with the context left at auto) is
    DCGS2 -- delayed classical Gram-Schmidt with re-orthogonalisation, one global reduction per
    Arnoldi step -- whenever ``restart <= 32``, else MGS.  DCGS2 builds the same Krylov basis in
    exact arithmetic but not SciPy's floating-point sequence: info matches and the inner
    iteration count may differ by one.  ``orth="mgs"`` runs SciPy's exact
    modified Gram-Schmidt sequence (iterative.py:755-759); ``orth="dcgs2"`` forces DCGS2.

    ``A``: a :class:`CsrOperator` or any SciPy sparse matrix (uploaded).  ``M``: None, a
    :class:`BlockJacobi` or a :class:`LineJacobi` built on ``A``; any other preconditioner raises TypeError (no CPU
    fallback).  ``callback`` is not supported (the Arnoldi loop never returns to the host).
    ``restart``/``maxiter``: None = SciPy's defaults (20 / 10 n); explicit values must be
    positive integers (ValueError otherwise).
    """
    global _last_stats
    if callback is not None:
        raise NotImplementedError("vtkrylov.gmres: callbacks would force a host round trip per "
                                  "Arnoldi step and are not supported")
    if M is not None and not isinstance(M, (BlockJacobi, LineJacobi)):
        raise TypeError("vtkrylov.gmres: M must be None, vtkrylov.BlockJacobi or vtkrylov.LineJacobi")
    if not isinstance(A, CsrOperator):
        A = csr_matrix(A)
    if atol == "legacy" or atol is None or atol < 0:
        raise ValueError(f"'scipy.sparse.linalg.gmres' called with invalid `atol`={atol}; "
                         "if set, `atol` must be a real, non-negative number.")
    for name, v in (("restart", restart), ("maxiter", maxiter)):
        if v is not None and (int(v) != v or int(v) <= 0):
            raise ValueError(f"vtkrylov.gmres: {name} must be a positive integer or None, got {v!r}")
    n = A.n_local
    vb = _Vec(b, n)
    if x0 is None:
        if vb.kind == _abi.PTR_DEVICE:
            import torch
            x = torch.zeros_like(vb.obj)
        else:
            x = np.zeros(n)
    else:
        if vb.kind == _abi.PTR_DEVICE:
            x = x0.clone()
        else:
            x = np.array(x0, dtype=np.float64, copy=True).reshape(-1)
    vx = _Vec(x, n, writable=True)
    x = vx.obj
    info = C.c_int()
    st = _abi.Stats()
    prev = None
    if orth is not None:
        prev = A.ctx.orth
        A.ctx.set_orth(_abi.ORTH[orth])
    try:
        check(lib().vtk_gmres(A.handle, None if M is None else M.handle, vb.ptr, vx.ptr,
                              float(rtol), float(atol), 0 if restart is None else int(restart),
                              0 if maxiter is None else int(maxiter), vb.kind, C.byref(info),
                              C.byref(st)), A.ctx.handle)
    finally:
        if prev is not None:
            A.ctx.set_orth(prev)
    _last_stats = SolveStats(**st.as_dict())
    return x, info.value


def rhs_splitmix(n: int, seed: int = 0x5EED, r0: int = 0, r1: int | None = None) -> np.ndarray:
    r1 = n if r1 is None else r1
    b = np.empty(r1 - r0)
    check(lib().vtk_rhs_splitmix(seed, r0, r1, _np_ptr(b)))
    return b


def vlasov_generate_host(params: VlasovParams, r0: int = 0, r1: int | None = None):
    """Host assembly of rows [r0, r1) (the same entry code the device generator runs)."""
    n, nnz = C.c_int64(), C.c_int64()
    check(lib().vtk_vlasov_size(C.byref(params), C.byref(n), C.byref(nnz)))
    r1 = n.value if r1 is None else r1
    per = {1: 3, 2: 5, 4: 9}[params.dim]
    cap = max(1, (r1 - r0) * per)
    ip = np.empty(r1 - r0 + 1, np.int32)
    ix = np.empty(cap, np.int32)
    d = np.empty(cap, np.float32 if params.fp32 else np.float64)
    check(lib().vtk_vlasov_generate(C.byref(params), r0, r1, _np_ptr(ip), _np_ptr(ix), _np_ptr(d)))
    k = int(ip[-1])
    return ip, ix[:k].copy(), d[:k].copy()


def partition_rows(n: int, world: int, align: int = 1, indptr=None) -> np.ndarray:
    offs = np.empty(world + 1, np.int64)
    ip = None if indptr is None else np.ascontiguousarray(indptr, np.int32)
    check(lib().vtk_partition_rows(n, None if ip is None else _np_ptr(ip), world, align, _np_ptr(offs)))
    return offs


def halo_plan(n_global: int, offsets, rank: int, indices):
    """(local_indices, halo_cols, halo_count_per_rank) of one rank's row block."""
    offs = np.ascontiguousarray(offsets, np.int64)
    world = offs.shape[0] - 1
    idx = np.ascontiguousarray(indices, np.int32)
    nh = C.c_int64()
    check(lib().vtk_halo_plan(n_global, _np_ptr(offs), world, rank, idx.shape[0], _np_ptr(idx),
                              None, C.byref(nh), None, None))
    loc = np.empty(idx.shape[0], np.int32)
    cols = np.empty(max(nh.value, 1), np.int64)
    cnt = np.empty(world, np.int64)
    check(lib().vtk_halo_plan(n_global, _np_ptr(offs), world, rank, idx.shape[0], _np_ptr(idx),
                              _np_ptr(loc), C.byref(nh), _np_ptr(cols), _np_ptr(cnt)))
    return loc, cols[:nh.value], cnt
