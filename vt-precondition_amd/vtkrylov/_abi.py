"""Raw ctypes binding of libvtkrylov.so (include/vtkrylov.h).

This is the reference-side binding INTEGRATION.md describes: the thin layer a caller of the
scipy.sparse path adds to reach the gfx950 kernels.  It loads the in-tree library
(``vtkrylov/lib/libvtkrylov.so``) and nothing else; there is no CPU fallback — if the
library is missing or no HIP device is visible, calls fail loudly.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libvtkrylov.so")

OK = 0
ERR_ARG = -1
ERR_HIP = -2
ERR_RCCL = -3
ERR_SINGULAR = -4
ERR_NOMEM = -5
ERR_STATE = -6
ERR_NODEVICE = -7
ERR_PEER = -8       # a peer rank failed mid-solve; this rank left the solve at the same step

PTR_HOST = 0
PTR_DEVICE = 1

ORTH_MGS = 0
ORTH_DCGS2 = 1
ORTH_AUTO = 2
ORTH = {"mgs": 0, "dcgs2": 1, "auto": 2}


class VlasovParams(C.Structure):
    _fields_ = [("dim", C.c_int), ("fp32", C.c_int), ("shape", C.c_int64 * 4),
                ("vmax", C.c_double), ("E0", C.c_double), ("nu", C.c_double),
                ("alpha", C.c_double), ("cfl", C.c_double)]


class Stats(C.Structure):
    _fields_ = [("inner_iters", C.c_int64), ("restarts", C.c_int64), ("presid", C.c_double),
                ("rnorm", C.c_double), ("bnorm", C.c_double), ("atol_eff", C.c_double),
                ("t_solve", C.c_double), ("bytes_moved", C.c_double), ("breakdown", C.c_int),
                ("orth", C.c_int), ("band", C.c_int)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


P = C.c_void_p
I32P = C.POINTER(C.c_int32)
I64P = C.POINTER(C.c_int64)

# name -> (restype, argtypes); must cover every function declared in include/vtkrylov.h
PROTOTYPES = {
    "vtk_abi_version": (C.c_int, []),
    "vtk_build_id": (C.c_char_p, []),
    "vtk_ctx_set_tuning": (C.c_int, [P, C.c_char_p, C.c_int]),
    "vtk_ctx_get_tuning": (C.c_int, [P, C.c_char_p, C.POINTER(C.c_int)]),
    "vtk_status_string": (C.c_char_p, [C.c_int]),
    "vtk_last_error": (C.c_int, [P, C.c_char_p, C.c_size_t]),
    "vtk_vlasov_size": (C.c_int, [C.POINTER(VlasovParams), I64P, I64P]),
    "vtk_vlasov_generate": (C.c_int, [C.POINTER(VlasovParams), C.c_int64, C.c_int64, P, P, P]),
    "vtk_rhs_splitmix": (C.c_int, [C.c_uint64, C.c_int64, C.c_int64, P]),
    "vtk_partition_rows": (C.c_int, [C.c_int64, P, C.c_int, C.c_int, P]),
    "vtk_halo_plan": (C.c_int, [C.c_int64, P, C.c_int, C.c_int, C.c_int64, P, P, I64P, P, P]),
    "vtk_line_band_plan": (C.c_int, [C.c_int64, C.c_int64, C.c_int, C.c_void_p]),
    "vtk_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "vtk_ctx_create": (C.c_int, [C.c_int, C.POINTER(P)]),
    "vtk_ctx_destroy": (None, [P]),
    "vtk_ctx_stream": (C.c_int, [P, C.POINTER(P)]),
    "vtk_ctx_synchronize": (C.c_int, [P]),
    "vtk_comm_unique_id": (C.c_int, [P]),
    "vtk_comm_init": (C.c_int, [P, C.c_int, C.c_int, P]),
    "vtk_comm_info": (C.c_int, [P, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "vtk_comm_rccl_count": (C.c_int, [P, C.POINTER(C.c_int)]),
    # vtk_comm_init_host: prototype registered by vtkrylov/comm.py (needs the hook struct)
    "vtk_comm_init_host": (C.c_int, [P, C.c_int, C.c_int, P]),
    "vtk_csr_create": (C.c_int, [P, C.c_int64, P, C.c_int64, P, P, P, C.c_int, C.c_int, C.POINTER(P)]),
    "vtk_csr_create_vlasov": (C.c_int, [P, C.POINTER(VlasovParams), P, C.POINTER(P)]),
    "vtk_csr_info": (C.c_int, [P, I64P, I64P, I64P, I64P, I64P]),
    "vtk_csr_download": (C.c_int, [P, P, P, P]),
    "vtk_csr_destroy": (None, [P]),
    "vtk_spmv": (C.c_int, [P, P, P, C.c_int]),
    "vtk_bjacobi_create": (C.c_int, [P, C.c_int, C.POINTER(P)]),
    "vtk_bjacobi_inverse": (C.c_int, [P, P, C.c_int]),
    "vtk_bjacobi_apply": (C.c_int, [P, P, P, C.c_int]),
    "vtk_bjacobi_set_mode": (C.c_int, [P, C.c_int]),
    "vtk_csr_set_layout": (C.c_int, [P, C.c_int]),
    "vtk_csr_get_layout": (C.c_int, [P, C.POINTER(C.c_int)]),
    "vtk_csr_layout_info": (C.c_int, [P, C.c_void_p]),
    "vtk_csr_set_line_band": (C.c_int, [P, C.c_int64]),
    "vtk_csr_get_line_band": (C.c_int, [P, I64P]),
    "vtk_csr_get_line_values": (C.c_int, [P, C.POINTER(C.c_int)]),
    "vtk_csr_set_grid4": (C.c_int, [P, C.c_int64, C.c_int64, C.c_int64]),
    "vtk_csr_get_grid4": (C.c_int, [P, I64P]),
    "vtk_bjacobi_get_mode": (C.c_int, [P, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "vtk_prec_destroy": (None, [P]),
    "vtk_linejacobi_create": (C.c_int, [P, C.c_int64, C.c_int64, C.POINTER(P)]),
    "vtk_linejacobi_factors": (C.c_int, [P, P, C.c_int]),
    "vtk_prec_apply": (C.c_int, [P, P, P, C.c_int]),
    "vtk_linejacobi_set_compact": (C.c_int, [P, C.c_int]),
    "vtk_linejacobi_get_compact": (C.c_int, [P, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "vtk_prec_kind_of": (C.c_int, [P, C.POINTER(C.c_int)]),
    "vtk_precond_matvec": (C.c_int, [P, P, P, P, C.c_int]),
    "vtk_gmres": (C.c_int, [P, P, P, P, C.c_double, C.c_double, C.c_int, C.c_int64, C.c_int,
                            C.POINTER(C.c_int), C.POINTER(Stats)]),
    "vtk_gmres_set_orth": (C.c_int, [P, C.c_int]),
    "vtk_gmres_set_band": (C.c_int, [P, C.c_int]),
    "vtk_bjacobi_create_ex": (C.c_int, [P, C.c_int, C.c_int, C.c_void_p]),
    "vtk_profile_enable": (C.c_int, [P, C.c_int]),
    "vtk_profile_read": (C.c_int, [P, P, C.c_int, C.POINTER(C.c_int)]),
}


ABI_VERSION = 6   # include/vtkrylov.h VTK_ABI_VERSION


class BandGeometry(C.Structure):
    _fields_ = [("parts", C.c_int), ("wg_per_range", C.c_int), ("waves_per_wg", C.c_int),
                ("ranges", C.c_int), ("lines", C.c_int64)]


class LayoutInfo(C.Structure):
    _fields_ = [("layout", C.c_int), ("matrix_bytes", C.c_double), ("sell_chunks", C.c_int64),
                ("sell_entries", C.c_int64), ("wide_chunks", C.c_int64)]


class KernelProfile(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("launches", C.c_int64), ("seconds", C.c_double),
                ("bytes", C.c_double)]

_lib = None


class VtkError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"{msg} (status {status})")
        self.status = status


def lib() -> C.CDLL:
    """Load libvtkrylov.so (build it with ``make -C vt-precondition_amd/csrc``)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch's libtorch_hip NEEDs "libamdhip64.so" while this
        # library NEEDs the SONAME "libamdhip64.so.7"; if torch is present it must be loaded
        # first so both resolve to the same runtime (otherwise torch finds no GPU).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        path = os.environ.get("VTK_LIB", LIB_PATH)   # VTK_LIB: another build of the same ABI (A/B runs)
        if not os.path.exists(path):
            raise ImportError(f"libvtkrylov.so not built: {path} (run __graft_entry__.build())")
        L = C.CDLL(path)
        for name, (res, args) in PROTOTYPES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if L.vtk_abi_version() != ABI_VERSION:
            raise ImportError("libvtkrylov.so ABI version mismatch")
        _lib = L
    return _lib


CSRC = os.path.join(os.path.dirname(_HERE), "csrc")
HEADER = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "vtkrylov.h")


def source_build_id(csrc: str = CSRC, header: str = HEADER, extra: str = "") -> str | None:
    """The build id csrc/Makefile compiles into vtk_build_id(): SHA-256 (16 hex digits) of the
    .hip/.hpp/.cpp sources in name order, the public header, the Makefile and EXTRA.  None when
    the sources are not present."""
    if not os.path.isdir(csrc) or not os.path.exists(header):
        return None
    names = sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".hpp", ".cpp")))
    h = hashlib.sha256()
    for path in [os.path.join(csrc, f) for f in names] + [header, os.path.join(csrc, "Makefile")]:
        with open(path, "rb") as f:
            h.update(f.read())
    h.update(extra.encode())
    return h.hexdigest()[:16]


def build_id() -> str:
    return lib().vtk_build_id().decode()


class StaleBuildError(RuntimeError):
    pass


def check_build_id(built: str | None = None, sources: str | None = None) -> str:
    """Raise StaleBuildError when the loaded libvtkrylov.so was not built from the checked-out
    sources (the GPU box runs the binary pushed from the build container).  An explicit VTK_LIB
    (A/B builds of other variants) is not checked.  Returns the build id."""
    built = build_id() if built is None else built
    if os.environ.get("VTK_LIB") and built is not None:
        return built
    sources = source_build_id() if sources is None else sources
    if sources is not None and built != sources:
        raise StaleBuildError(f"libvtkrylov.so build id {built} does not match the sources ({sources}): "
                              "rebuild with __graft_entry__.build() / make -C vt-precondition_amd/csrc")
    return built


def last_error(ctx=None) -> str:
    buf = C.create_string_buffer(1024)
    lib().vtk_last_error(ctx, buf, len(buf))
    return buf.value.decode(errors="replace")


def check(status: int, ctx=None):
    if status == OK:
        return
    import numpy as np
    msg = last_error(ctx)
    if status == ERR_SINGULAR:
        raise np.linalg.LinAlgError(msg)
    if status == ERR_ARG:
        raise ValueError(msg)
    raise VtkError(status, msg or lib().vtk_status_string(status).decode())
