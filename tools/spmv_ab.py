"""In-process A/B of the plain SpMV (vtk_spmv, the measured half of the metric) over context
tuning settings: one operator, alternating settings, HIP-event timing on the library's stream.

    python tools/spmv_ab.py --config C3 --settings "layout=sell;layout=csr"

A setting is `layout=sell|csr` (vtk_csr_set_layout: the switch that reaches vtk_spmv; the
solver's tuning keys -- sell_canon, grid4, ... -- are compiled out of the plain SpMV)
or a context tuning key=value, comma-separated.

Prints one JSON line: per setting the per-launch microseconds of every round and their median,
and the algorithmic GB/s (layout bytes + x + y)."""
import argparse
import ctypes as C
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vt-precondition_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--settings", default="layout=sell;layout=csr")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    import torch

    import vtkrylov as vk
    from oracle import twin
    p = twin.CONFIGS[a.config]
    ctx = vk.default_context(0)
    A = vk.vlasov_operator(vk.vlasov_params(p.dim, p.shape, fp32=p.fp32), ctx=ctx)
    dev = torch.device("cuda", 0)
    x = torch.from_numpy(vk.rhs_splitmix(p.n, seed=0xC0FFEE)).to(dev)
    y = torch.empty_like(x)
    y0 = None
    torch.cuda.synchronize()
    lib = vk._abi.lib()
    stream = torch.cuda.ExternalStream(ctx.stream_ptr(), device=dev)
    sets = [dict((kv.split("=")[0], kv.split("=")[1]) for kv in s.split(",") if kv) for s in a.settings.split(";")]
    nbytes = {}
    times = {i: [] for i in range(len(sets))}
    for r in range(a.rounds + 1):
        order = range(len(sets)) if r % 2 == 0 else reversed(range(len(sets)))
        for i in order:
            for k, v in sets[i].items():
                if k == "layout":
                    A.set_layout(v)
                else:
                    ctx.set_tuning(k, int(v))
            nbytes[i] = A.layout_info()["matrix_bytes"] + 16 * A.n_local
            for _ in range(3):
                vk._abi.check(lib.vtk_spmv(A.handle, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), 1))
            ctx.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.reps):
                vk._abi.check(lib.vtk_spmv(A.handle, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), 1))
            e1.record(stream)
            e1.synchronize()
            if r > 0:
                times[i].append(round(e0.elapsed_time(e1) * 1e3 / a.reps, 2))
            yh = y.cpu().numpy()
            if y0 is None:
                y0 = yh
            assert np.array_equal(yh, y0), "SpMV bits changed with a tuning setting"
    out = {"config": a.config, "settings": {}}
    for i, s in enumerate(sets):
        med = statistics.median(times[i])
        out["settings"][a.settings.split(";")[i]] = {"median_us": med, "bytes": nbytes[i], "gbs": nbytes[i] / med / 1e3,
                                                    "us": times[i]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
