"""In-process A/B of a library environment switch (one operator, one allocation, alternating
settings): the band step's rate varies ~5 % between processes with the physical placement of
the same allocations (profiles/r03_membench_walk.txt), so A/Bs across processes need many reps.

    python tools/ab_env.py --env band --values 1,0 --rounds 6 [--config C3] [--slab 8 --comm-solo]

Prints one JSON line: per value the solve wall times (ms) and their median.  The switch is a
context tuning key (vtk_ctx_set_tuning: band, band_lsv, sell_canon, ...; a VTK_<KEY> name is
accepted too), set on the context between solves."""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vt-precondition_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", required=True)
    ap.add_argument("--values", default="1,0")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--rtol", type=float, default=1e-8)
    ap.add_argument("--prec", default="bj", choices=["bj", "line"])
    ap.add_argument("--seg", type=int, default=25)
    ap.add_argument("--slab", type=int, default=1, help="one rank's x-slab at this many GPUs (as bench.py --slab)")
    ap.add_argument("--comm-solo", action="store_true", help="the distributed code path on one rank (bench.py --comm-solo)")
    ap.add_argument("--perj", action="store_true", help="also one profiled solve per value: band step us per j")
    ap.add_argument("--set", default="", help="fixed tuning for every value, e.g. band_opt=1,lsv_ring=0")
    ap.add_argument("--maxiter", type=int, default=None,
                    help="restart cycles per solve (timing-only variants whose numerics do not converge)")
    a = ap.parse_args()
    import vtkrylov as vk
    from oracle import twin
    p = twin.CONFIGS[a.config]
    ctx = vk.default_context(0)
    if a.comm_solo:
        ctx.set_tuning("comm_solo", 1)
        ctx.comm_init(0, 1, vk.Context.unique_id())
    shape = (p.shape[0] // a.slab,) + tuple(p.shape[1:])
    n = int(np.prod(shape))
    A = vk.vlasov_operator(vk.vlasov_params(p.dim, shape, fp32=p.fp32), ctx=ctx)
    params = vk.vlasov_params(p.dim, shape, fp32=p.fp32)
    M = vk.line_jacobi(A, vk.vlasov_line_stride(params), a.seg) if a.prec == "line" else vk.block_jacobi(A, 8)
    import torch
    b = torch.from_numpy(vk.rhs_splitmix(n)).to(torch.device("cuda", 0))   # device-resident, as bench.py
    torch.cuda.synchronize()
    key = a.env[4:].lower() if a.env.startswith("VTK_") else a.env
    for kv in filter(None, a.set.split(",")):
        k, v = kv.split("=")
        ctx.set_tuning(k, int(v))
    vals = a.values.split(",")
    times = {v: [] for v in vals}
    iters = {}
    for r in range(a.rounds + 1):
        for v in (vals if r % 2 == 0 else vals[::-1]):
            ctx.set_tuning(key, int(v))
            t = time.perf_counter()
            _, info = vk.gmres(A, b, rtol=a.rtol, M=M, maxiter=a.maxiter)
            dt = (time.perf_counter() - t) * 1e3
            st = vk.last_stats()
            iters[v] = (st.inner_iters, st.band, info)
            if r > 0:   # round 0: warm-up
                times[v].append(round(dt, 3))
    perj = {}
    if a.perj:
        ctx.set_tuning("prof_perj", 1)
        for v in vals:
            ctx.set_tuning(key, int(v))
            ctx.profile(True)
            vk.gmres(A, b, rtol=a.rtol, M=M, maxiter=a.maxiter)
            pr = ctx.profile_read()
            ctx.profile(False)
            perj[v] = {k: round(e["avg_us"], 1) for k, e in sorted(pr.items())
                       if k.startswith("band_step") or k in ("dc_scalar", "dc_update", "spmv_resid_bj", "spmv_bj_dc",
                                                             "line_dc", "spmv_lsv", "xupdate", "spmv_bj",
                                                             "dc_dots", "spmv_resid")}
        ctx.set_tuning("prof_perj", 0)
    out = {"config": a.config, "set": a.set, "perj_us": perj, "prec": a.prec, "slab": a.slab, "comm_solo": a.comm_solo, "env": a.env, "iters_band_info": iters,
           "median_ms": {v: statistics.median(t) for v, t in times.items()}, "ms": times}
    print(json.dumps(out))
    M.close()
    A.close()


if __name__ == "__main__":
    main()
