"""Plain-SpMV timing of a given libvtkrylov.so build (any ABI >= 1: only vtk_ctx_create,
vtk_csr_create_vlasov, vtk_ctx_stream and vtk_spmv are used), for bisecting the plain SpMV across
rounds: C3 operator assembled on the device, 50 back-to-back vtk_spmv launches timed with HIP
events on the library's stream, median of rounds.

    python tools/spmv_lib_time.py --lib tools/bin/lib_r03/libvtkrylov.so [--config C3] [--rounds 6]

Prints one JSON line {lib, median_us, us}."""
import argparse
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]


class VlasovParams(C.Structure):
    _fields_ = [("dim", C.c_int), ("fp32", C.c_int), ("shape", C.c_int64 * 4),
                ("vmax", C.c_double), ("E0", C.c_double), ("nu", C.c_double),
                ("alpha", C.c_double), ("cfl", C.c_double)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    import torch   # first: one HIP runtime for torch and the library
    from oracle import twin
    L = C.CDLL(os.path.abspath(a.lib))
    P = C.c_void_p
    L.vtk_ctx_create.argtypes = [C.c_int, C.POINTER(P)]
    L.vtk_csr_create_vlasov.argtypes = [P, C.POINTER(VlasovParams), P, C.POINTER(P)]
    L.vtk_spmv.argtypes = [P, P, P, C.c_int]
    L.vtk_ctx_stream.argtypes = [P, C.POINTER(P)]
    p = twin.CONFIGS[a.config]
    ctx, A, st = P(), P(), P()
    assert L.vtk_ctx_create(0, C.byref(ctx)) == 0
    sh = list(p.shape) + [0] * (4 - len(p.shape))
    prm = VlasovParams(p.dim, int(p.fp32), (C.c_int64 * 4)(*sh), p.vmax, p.E0, p.nu, p.alpha, p.cfl)
    assert L.vtk_csr_create_vlasov(ctx, C.byref(prm), None, C.byref(A)) == 0
    assert L.vtk_ctx_stream(ctx, C.byref(st)) == 0
    dev = torch.device("cuda", 0)
    x = torch.from_numpy(twin.rhs(p.n, seed=0xC0FFEE)).to(dev)
    y = torch.empty_like(x)
    torch.cuda.synchronize()
    stream = torch.cuda.ExternalStream(st.value, device=dev)
    us = []
    for r in range(a.rounds + 1):
        for _ in range(3):
            assert L.vtk_spmv(A, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), 1) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(a.reps):
            L.vtk_spmv(A, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), 1)
        e1.record(stream)
        e1.synchronize()
        if r:
            us.append(round(e0.elapsed_time(e1) * 1e3 / a.reps, 2))
    print(json.dumps({"lib": a.lib, "config": a.config, "median_us": statistics.median(us), "us": us}))


if __name__ == "__main__":
    main()
