"""Benchmark: preconditioned-GMRES iterations/s (+ CSR SpMV achieved HBM GB/s) on the C3
20M-row synthetic Vlasov operator (BASELINE.json configs[3], the north_star's target), one
rank per MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3] [--no-cpu-baseline]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

With --gpus N > 1 and no launcher (WORLD_SIZE unset) the script starts its own N ranks: the
parent process never touches the GPU, it spawns N fresh children (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set, one GPU each), passes rank 0's JSON line
through and exits non-zero if any rank fails.

A step = one full solve: x0 = 0 -> ||b - A x|| <= 1e-8 ||b|| with GMRES(20) + block-Jacobi(8)
(SURVEY.md §8d).  value = inner (Arnoldi) iterations of the K timed solves / the max-over-ranks
wall time of those solves.  The problem is fixed as N grows (strong scaling; rows sharded in
contiguous x-slabs, RCCL halo exchange + all-reduce).  Operator, RHS and BJ inverses are built
on the device before the timed region; b and x live in HBM (torch tensors passed through the
C-ABI as device pointers).

Printed: ONE JSON line on rank 0 (the driver's contract), with `roofline` (the dominant
kernel, timed live with HIP events on the context's stream) and `cpu_baseline` (SciPy, the
north_star's reference scipy.sparse path: one full solve of the same operator and RHS to the
same tolerance on the box's host cores; --cpu-sample bounds it to the first --cpu-inner inner
iterations instead).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "vt-precondition_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)

CONFIGS = {  # name -> (dim, shape, fp32)   SURVEY.md Appendix A
    "C1": (2, (1250, 800), False),
    "C2": (2, (6250, 800), False),
    "C3": (2, (25_000, 800), False),
    "C4": (4, (200, 125, 50, 40), True),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def spmv_bytes(nnz, n, fp32):
    # B_spmv = 12 nnz + 4 (n+1) + 8 n (x once) + 8 n (y)   (fp32 values: 8 nnz)   SURVEY §8d
    return (8 if fp32 else 12) * nnz + 4 * (n + 1) + 16 * n


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(cfg_name, A_host, b, bs, rtol, inner_limit, line=None, full=True, gpu_iters=None):
    """SciPy 1.15.3 (the reference scipy.sparse path) on the host cores (BASELINE.md "CPU-baseline
    plan"): one full GMRES solve to the GPU's tolerance (time to solution and inner iterations/s;
    `full=False`: only the first `inner_limit` inner iterations), and csr_matvec's median over
    20 reps.  BLAS threads = the box's CPU share (OMP_NUM_THREADS, 16 on the GPU box; the
    affinity set is the whole machine's), csr_matvec itself is single-threaded."""
    import numpy as np
    import scipy.sparse as sp

    from oracle import twin
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, len(os.sched_getaffinity(0)))
    try:
        from threadpoolctl import threadpool_info, threadpool_limits
        limiter = threadpool_limits(share)
        blas_threads = max([d.get("num_threads", 1) for d in threadpool_info()] or [1])
    except Exception:
        limiter, blas_threads = None, 1
    ip, ix, d = A_host
    n = ip.shape[0] - 1
    A = sp.csr_matrix((d, ix, ip), shape=(n, n))
    x = twin.rhs(n, seed=0xC0FFEE)
    A @ x
    reps = []
    for _ in range(20):
        t = time.perf_counter()
        A @ x
        reps.append(time.perf_counter() - t)
    t_spmv = sorted(reps)[len(reps) // 2]
    if line is None:
        Mop, mname = twin.bj_inverse_numpy(ip, ix, d, n, bs), f"BJ({bs})"
    else:   # (stride, seg): SciPy's splu of the line matrix as the LinearOperator
        Mop, mname = twin.line_operator(ip, ix, d, n, line[0], line[1]), f"Line(stride={line[0]}, seg={line[1]}) splu"
    s = twin.scipy_gmres(A, b, Mop, rtol=rtol, inner_limit=None if full else inner_limit)
    if limiter is not None:
        limiter.restore_original_limits()
    what = (f"one full solve to rtol={rtol} (info {s.info}, {s.inner_iters} inner iterations, "
            f"true residual {s.true_resid / s.b_norm:.2e} ||b||)" if full else
            f"the first {s.inner_iters} inner iterations (one restart cycle, legacy maxiter bound)")
    out = {
        "value": s.inner_iters / s.seconds,
        "unit": "iters/s",
        "cores": int(blas_threads),
        "kind": "reference",
        "sample": (f"scipy.sparse.linalg.gmres(restart=20, M={mname} LinearOperator) on the same "
                   f"{cfg_name} operator/RHS, {what} in {s.seconds:.1f} s; csr_matvec is single-threaded, "
                   f"np.dot uses {blas_threads} BLAS threads (the box's CPU share); host cpus in affinity: "
                   f"{len(os.sched_getaffinity(0))}; cpu: {cpu_model()}"),
        "spmv_gbs": spmv_bytes(ip[-1], n, d.dtype == np.float32) / t_spmv / 1e9,
        "spmv_median_ms": t_spmv * 1e3,
        "spmv_reps": len(reps),
    }
    if full:
        out.update({"full_solve_s": s.seconds, "inner_iters": s.inner_iters, "info": s.info,
                    "true_rel_residual": s.true_resid / s.b_norm})
        if gpu_iters is not None:
            out["inner_iters_gpu"] = gpu_iters
    return out


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n: int) -> int:
    """Start ranks 0..n-1 of this same command as child processes (the torch.distributed.run
    environment contract) and wait for them.  Called before anything initialises the GPU; a
    failing rank ends the others (exact PIDs), so a half-dead job cannot hang the barrier."""
    import signal
    import subprocess
    env0 = dict(os.environ)
    env0.update({"WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1",
                 "MASTER_PORT": str(free_port()), "GROUP_RANK": "0", "VTK_BENCH_SPAWNED": "1"})
    env0.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = []
    for r in range(n):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                log(f"[launcher] rank {procs.index(p)} exited with {code}: stopping the other ranks")
                for q in live:
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.2)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C3", choices=sorted(CONFIGS))
    ap.add_argument("--bs", type=int, default=8)
    ap.add_argument("--rtol", type=float, default=1e-8)
    ap.add_argument("--restart", type=int, default=20)
    ap.add_argument("--spmv-reps", type=int, default=50)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-inner", type=int, default=20,
                    help="with --cpu-sample: inner iterations of the bounded SciPy sample")
    ap.add_argument("--cpu-sample", action="store_true",
                    help="CPU baseline on the first --cpu-inner inner iterations instead of a full solve")
    ap.add_argument("--orth", default="auto", choices=["auto", "mgs", "dcgs2"],
                    help="orthogonalisation: auto (library default: dcgs2 for restart <= 32), "
                         "mgs (SciPy's sequence) or dcgs2 (one reduction per step)")
    ap.add_argument("--bj-mode", default="auto", choices=["auto", "inverse", "tridiag"],
                    help="block-Jacobi apply: auto (tridiagonal-block LU factors when every block is "
                         "tridiagonal, as on the Vlasov operators), inverse (bit-exact inv*r), tridiag")
    ap.add_argument("--layout", default="auto", choices=["auto", "sell", "sell32", "csr"],
                    help="SpMV layout: auto (SELL-64 when its padding is small), sell (dictionary-coded "
                         "columns), sell32 (int32 columns), csr (CSR-stream tiles)")
    ap.add_argument("--prec", default="bj", choices=["bj", "line"],
                    help="preconditioner: bj (block-Jacobi(bs), SURVEY §8d, the metric's config) or line "
                         "(line-Jacobi along x, segments of --seg x-points, SURVEY §8f-4)")
    ap.add_argument("--seg", type=int, default=25, help="line-Jacobi segment length (x-points)")
    ap.add_argument("--operator", default="generated", choices=["generated", "upload", "npz"],
                    help="generated: assembled on the device (vtk_csr_create_vlasov); upload: the same "
                         "CSR handed over as host arrays (vtkrylov.csr_matrix, the drop-in path); npz: "
                         "written with save_npz and read back with vtkrylov.load_npz")
    ap.add_argument("--comm-solo", action="store_true",
                    help="one GPU through the distributed code paths (one-rank RCCL communicator)")
    ap.add_argument("--slab", type=int, default=1,
                    help="run one rank's slab of the config at this GPU count (Nx / SLAB x-columns; "
                         "with --comm-solo: the per-rank distributed step on one GPU)")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "host"],
                    help="rccl (production) or host-staged hooks over gloo (testing: ranks may share a GPU)")
    ap.add_argument("--check-launch", action="store_true",
                    help="rank plumbing only (no GPU): init the process group, all-reduce the ranks, "
                         "rank 0 prints one JSON line")
    ap.add_argument("--check-launch-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(launch_ranks(args.gpus))   # no GPU call has happened in this process

    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    if args.check_launch:
        if rank == args.check_launch_fail_rank:
            raise SystemExit(3)
        t = torch.tensor([rank, 1], dtype=torch.int64)
        if dist is not None:
            dist.all_reduce(t)
        if rank == 0:
            print(json.dumps({"check_launch": True, "n_gpus": world, "rank_sum": int(t[0]), "ranks": int(t[1]),
                              "local_rank": local, "launcher": os.environ.get("VTK_BENCH_SPAWNED") and "bench.py"}),
                  flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return

    import vtkrylov as vk
    from vtkrylov import comm as vkcomm
    # the GPU box runs the libvtkrylov.so pushed with the tree: refuse a binary that was not built
    # from these sources (a stale build would be measured as this code)
    build_id = vk._abi.check_build_id()
    ndev = vk.device_count()
    device = local % max(ndev, 1)
    ctx = vk.Context(device)
    if world > 1:
        if args.comm == "rccl":
            vkcomm.init_rccl(ctx, rank, world)
        else:
            vkcomm.init_host(ctx, rank, world)
    elif args.comm_solo:
        ctx.set_tuning("comm_solo", 1)
        ctx.comm_init(0, 1, vk.Context.unique_id())
    ctx.set_orth(vk._abi.ORTH[args.orth])
    torch.cuda.set_device(device)
    dev = torch.device("cuda", device)

    dim, shape, fp32 = CONFIGS[args.config]
    if args.slab > 1:
        # one rank's share of the config at --slab GPUs: the x-direction cut by that many (the
        # same periodic operator on Nx / P columns), run through the distributed code paths
        # (--comm-solo): the per-rank step time of a P-GPU run without its xGMI transfers
        if world != 1 or shape[0] % args.slab:
            raise SystemExit("--slab needs one rank and Nx divisible by it")
        shape = (shape[0] // args.slab,) + tuple(shape[1:])
    params = vk.vlasov_params(dim, shape, fp32=fp32)
    n_glob = int(np.prod(shape))
    align = shape[-1] if dim == 2 else shape[-1] * shape[-2] * shape[-3]   # x-slab boundaries
    offsets = vk.partition_rows(n_glob, world, align) if world > 1 else None
    t0 = time.time()
    A = vk.vlasov_operator(params, ctx=ctx, offsets=offsets)
    if args.operator != "generated":
        # the drop-in path: the operator arrives as a CSR (this rank's rows, global columns), the
        # way the reference's scipy.sparse path would hand it; the library finds its structure
        ip_h, ix_h, d_h = A.download()
        A.close()
        if args.operator == "npz":
            import tempfile
            from vtkrylov import npz as vknpz
            tmpd = tempfile.mkdtemp(prefix="vtk_bench_")
            f = os.path.join(tmpd, f"A_rank{rank}.npz")
            vknpz.save_npz_arrays(f, ip_h, ix_h, d_h, (A.row_end - A.row_begin, n_glob), compressed=False)
            del ip_h, ix_h, d_h
            ip_h, ix_h, d_h, _ = vknpz.load_npz_arrays(f)
            os.remove(f)
            os.rmdir(tmpd)
        A = vk.csr_matrix((d_h, ix_h, ip_h), shape=(n_glob, n_glob), ctx=ctx, offsets=offsets)
        del ip_h, ix_h, d_h
    A.set_layout(args.layout)
    if args.prec == "line":
        M = vk.line_jacobi(A, vk.vlasov_line_stride(params), args.seg)
        mdesc, mmode = f"Line({args.seg})", "line"
    else:
        M = vk.block_jacobi(A, args.bs, mode=args.bj_mode)
        mdesc, mmode = f"BJ({args.bs})", M.mode
    b_host = vk.rhs_splitmix(n_glob, r0=A.row_begin, r1=A.row_end)
    b = torch.from_numpy(b_host).to(dev)
    torch.cuda.synchronize()
    log(f"[rank {rank}] setup {time.time() - t0:.1f}s: n_local={A.n_local} nnz_local={A.nnz} halo={A.n_halo}")

    def barrier():
        if dist is not None:
            dist.barrier()

    def solve():
        x, info = vk.gmres(A, b, rtol=args.rtol, restart=args.restart, M=M)
        return x, info, vk.last_stats()

    for _ in range(args.warmup):
        _, info, st = solve()
    barrier()
    torch.cuda.synchronize()
    t = time.perf_counter()
    iters = 0
    infos = []
    per_solve = []   # vtk_gmres returns synchronised: wall time per solve (SURVEY §8d median)
    for _ in range(args.steps):
        ts = time.perf_counter()
        x, info, st = solve()
        per_solve.append(time.perf_counter() - ts)
        iters += st.inner_iters
        infos.append(info)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    # true residual of the last solve, on the device (vtk_spmv), reduced over ranks
    r = b - A @ x
    rn2 = torch.tensor([float(torch.dot(r, r).item()), float(torch.dot(b, b).item())], dtype=torch.float64)
    if dist is not None:
        dist.all_reduce(rn2)
    rel_res = float((rn2[0] / rn2[1]).sqrt())

    # ---- SpMV kernel, live HIP-event timing on the context's stream ----------------------
    import ctypes as C
    lib = vk._abi.lib()
    xs = torch.from_numpy(vk.rhs_splitmix(n_glob, seed=0xC0FFEE, r0=A.row_begin, r1=A.row_end)).to(dev)
    ys = torch.empty_like(xs)
    torch.cuda.synchronize()
    stream = torch.cuda.ExternalStream(ctx.stream_ptr(), device=dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        vk._abi.check(lib.vtk_spmv(A.handle, C.c_void_p(xs.data_ptr()), C.c_void_p(ys.data_ptr()), 1))
    ctx.synchronize()
    ev0.record(stream)
    for _ in range(args.spmv_reps):
        vk._abi.check(lib.vtk_spmv(A.handle, C.c_void_p(xs.data_ptr()), C.c_void_p(ys.data_ptr()), 1))
    ev1.record(stream)
    ev1.synchronize()
    t_spmv = ev0.elapsed_time(ev1) / 1e3 / args.spmv_reps
    # bytes the SpMV reads/writes in the layout in use (dictionary-coded SELL columns are
    # 0.5 B + 1 B/row instead of 4 B per entry); csr_equiv: SURVEY §8d's CSR figure
    linfo = A.layout_info()
    B = linfo["matrix_bytes"] + 16 * A.n_local
    B_csr = spmv_bytes(A.nnz, A.n_local, fp32)
    spmv_gbs = B / t_spmv / 1e9
    # cold: median of single reps with the 256 MB Infinity Cache flushed in between
    flush = torch.empty(512 * 2**20 // 8, dtype=torch.float64, device=dev)
    cold = []
    with torch.cuda.stream(stream):
        for _ in range(max(20, min(2 * args.spmv_reps, 100))):   # 100 flushed reps
            flush.fill_(1.0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            vk._abi.check(lib.vtk_spmv(A.handle, C.c_void_p(xs.data_ptr()), C.c_void_p(ys.data_ptr()), 1))
            e1.record(stream)
            e1.synchronize()
            cold.append(e0.elapsed_time(e1) / 1e3)
        # device-copy reference bandwidth: 1 GiB D2D copy (read + write)
        src = torch.empty(2**27, dtype=torch.float64, device=dev).fill_(1.0)
        dst = torch.empty_like(src)
        dst.copy_(src)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(5):
            dst.copy_(src)
        e1.record(stream)
        e1.synchronize()
    copy_gbs = 2 * src.numel() * 8 * 5 / (e0.elapsed_time(e1) / 1e3) / 1e9
    # device-read reference: a torch reduction over the same 1 GiB (read-only stream)
    with torch.cuda.stream(stream):
        src.sum()
        e0.record(stream)
        for _ in range(5):
            src.sum()
        e1.record(stream)
        e1.synchronize()
    read_gbs = src.numel() * 8 * 5 / (e0.elapsed_time(e1) / 1e3) / 1e9
    t_cold = sorted(cold)[len(cold) // 2]
    del flush, src, dst

    # ---- per-kernel profile of one more solve (outside the timed region): HIP events around
    #      every launch on the context's stream, algorithmic bytes per launch
    ctx.profile(True)
    solve()
    kprof = ctx.profile_read()
    ctx.profile(False)
    tot_s = sum(v["seconds"] for v in kprof.values()) or 1.0
    dom = max(kprof, key=lambda k: kprof[k]["seconds"])
    traffic, traffic_src = pmc_traffic(dom, args.config, world)
    traffic_spmv, traffic_spmv_src = pmc_traffic("spmv", args.config, world)
    dk = kprof[dom]

    # ---- the same solve with the line-implicit x preconditioner, outside the
    #      headline metric: fewer, slightly cheaper iterations -> time to solution
    alt = None
    if args.prec == "bj":
        ML = vk.line_jacobi(A, vk.vlasov_line_stride(params), args.seg)
        vk.gmres(A, b, rtol=args.rtol, restart=args.restart, M=ML)
        barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        it_l, inf_l, reps_l = 0, [], 3
        for _ in range(reps_l):
            _, inf = vk.gmres(A, b, rtol=args.rtol, restart=args.restart, M=ML)
            it_l += vk.last_stats().inner_iters
            inf_l.append(inf)
        torch.cuda.synchronize()
        barrier()
        el_l = time.perf_counter() - t
        if dist is not None:
            tt = torch.tensor([el_l], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el_l = float(tt.item())
        # one profiled line solve: per-class launches, mean time and rate
        ctx.profile(True)
        vk.gmres(A, b, rtol=args.rtol, restart=args.restart, M=ML)
        kprof_l = ctx.profile_read()
        ctx.profile(False)
        tot_l = sum(v["seconds"] for v in kprof_l.values()) or 1.0
        ML.close()
        alt = {"prec": f"Line({args.seg}), compact apply", "info": inf_l,
               "inner_iters_per_solve": it_l / reps_l, "ms_per_solve": el_l / reps_l * 1e3,
               "iters_per_s": it_l / el_l,
               "time_to_solution_speedup_vs_bj": (elapsed / args.steps) / (el_l / reps_l),
               "kernels": {k: {"avg_us": round(v["avg_us"], 2), "gbs": round(v["gbs"], 1),
                               "launches": v["launches"], "share": round(v["seconds"] / tot_l, 4)}
                           for k, v in sorted(kprof_l.items(), key=lambda kv: -kv[1]["seconds"])}}

    ms = elapsed / args.steps * 1e3
    # ---- reconciliation with SURVEY §8(d)'s byte model (MGS, inverse BJ(bs), CSR int32 columns):
    # (1) the dominant kernel with its SELL matrix bytes replaced by CSR's (same algorithm,
    #     §8(d)'s matrix encoding); (2) the whole solve's actual algorithmic bytes (every
    #     profiled class) / ms_per_step; (3) the whole solve under §8(d)'s formulas / ms_per_step
    #     (above 1.0 of peak is possible: DCGS2 reads the basis twice per step instead of MGS's
    #     2j+8 vector passes, tridiagonal BJ reads 8 B/row instead of 64, codes instead of int32
    #     columns, no residual SpMV for x0 = 0 -- fewer bytes, not skipped work)
    n_loc, nnz_loc = A.n_local, A.nnz
    csr_matrix_bytes = (4 if fp32 else 8) * nnz_loc + 4 * nnz_loc + 4 * (n_loc + 1)
    # the band step reads the SELL codes and -- line-separable operators (A.line_separable) --
    # 8 B of values per row from the diagonal table instead of the SELL values (vtk_api.cpp b_band)
    lv = A.line_values   # 2: canonical rows, the band step reads only the diagonal table
    band_matrix = 8.0 * n_loc if lv == 2 else \
        linfo["matrix_bytes"] - (8.0 * linfo["sell_entries"] - 8.0 * n_loc if lv == 1 else 0.0)
    d_matrix = csr_matrix_bytes - (band_matrix if dom == "band_step" else linfo["matrix_bytes"])
    dom_csr = dk["bytes"] / dk["launches"] + (d_matrix if dom.startswith("spmv") or dom == "band_step" else 0.0)
    solve_bytes = sum(v["bytes"] for v in kprof.values())
    it_solve = int(round(iters / args.steps))
    m = args.restart
    cycles = -(-it_solve // m)
    B_spmv = spmv_bytes(nnz_loc, n_loc, fp32)
    B_pc = 8 * args.bs * n_loc + 16 * n_loc
    sec8d = sum(B_spmv + B_pc + 8 * n_loc * (2 * (k % m) + 8) for k in range(it_solve)) \
        + cycles * (B_spmv + 24 * n_loc + B_pc + 24 * n_loc + 8 * n_loc * (m + 2))
    t_solve = ms / 1e3
    # (round 2's "unfused-equivalent" band rate is no longer reported: with p_j recomputed and
    # the line-separable values the band step's bytes per launch differ from the two kernels' by
    # more than one basis read, and the per-j mix of a solve is not in the aggregate profile)
    band_equiv = None
    recon = {
        "note": "SURVEY 8(d) reconciliation; per rank (n_local rows); frac = GB/s / 8000",
        "dominant_kernel_csr_equiv": {"kernel": dom, "bytes_per_launch": dom_csr,
                                      "gbs": dom_csr / (dk["avg_us"] * 1e-6) / 1e9,
                                      "frac": dom_csr / (dk["avg_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS,
                                      "matrix_bytes_layout": band_matrix if dom == "band_step" else linfo["matrix_bytes"],
                                      "matrix_bytes_csr_int32": csr_matrix_bytes},
        "solve_actual": {"bytes": solve_bytes, "gbs": solve_bytes / t_solve / 1e9,
                         "frac": solve_bytes / t_solve / 1e9 / HBM_PEAK_GBS,
                         "note": "algorithmic bytes of every profiled kernel of one solve / ms_per_step"},
        "solve_sec8d_model": {"bytes": sec8d, "gbs": sec8d / t_solve / 1e9,
                              "frac": sec8d / t_solve / 1e9 / HBM_PEAK_GBS,
                              "inner_iters": it_solve, "cycles": cycles,
                              "note": "MGS + inverse BJ + CSR int32 byte model of 8(d) / ms_per_step"},
    }
    out = {
        "metric": "precond-GMRES iters/sec + CSR SpMV achieved-HBM-GB/s, 1/2/4/8 MI355X",
        "value": iters / elapsed,
        "unit": "iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64" if not fp32 else "f32-values/f64",
        "data": "synthetic (SURVEY.md Appendix A Vlasov operator, splitmix64 RHS), " +
                {"generated": "generated on device", "upload": "uploaded as a host CSR (vtkrylov.csr_matrix)",
                 "npz": "read from a save_npz archive (vtkrylov.load_npz)"}[args.operator],
        "config": {"workload": f"{args.config}{'/' + str(args.slab) + ' slab' if args.slab > 1 else ''}: "
                               f"GMRES({args.restart}, {args.orth})+{mdesc} to rtol={args.rtol}, "
                               f"n={n_glob}, row-sharded over {world} GPU(s)",
                   "n": n_glob, "nnz": int(params_nnz(dim, shape)), "restart": args.restart,
                   "prec": args.prec, "bs": args.bs if args.prec == "bj" else None, "operator": args.operator,
                   "line_band": A.line_band, "line_values": A.line_values,
                   "seg": args.seg if args.prec == "line" else None, "bj_apply": mmode, "layout": A.layout, "rtol": args.rtol, "orth": args.orth,
                   "parallelism": f"row-slab x{world}",
                   "comm": args.comm if world > 1 else ("rccl-solo" if args.comm_solo else None),
                   "launcher": ("bench.py" if os.environ.get("VTK_BENCH_SPAWNED") else "external") if world > 1 else None},
        "rccl_ranks": ctx.rccl_ranks(),
        "build_id": build_id,
        "inner_iters_per_solve": iters / args.steps,
        "solves_per_s": args.steps / elapsed,
        "solve_ms_median": sorted(per_solve)[len(per_solve) // 2] * 1e3,
        "info": infos,
        "true_rel_residual": rel_res,
        "spmv": {"gbs": spmv_gbs, "hbm_frac": spmv_gbs / HBM_PEAK_GBS, "us": t_spmv * 1e6, "bytes": B,
                 "layout": linfo["layout"], "wide_chunks": linfo["wide_chunks"],
                 "csr_equiv_bytes": B_csr, "csr_equiv_gbs": B_csr / t_spmv / 1e9,
                 "cold_median_us": t_cold * 1e6, "cold_gbs": B / t_cold / 1e9,
                 "device_copy_gbs": copy_gbs, "frac_of_copy": spmv_gbs / copy_gbs,
                 "device_read_gbs": read_gbs, "frac_of_read": spmv_gbs / read_gbs},
        "roofline": {"kernel": dom, "bound": "hbm", "achieved": dk["gbs"], "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": dk["gbs"] / HBM_PEAK_GBS,
                     "traffic": traffic, "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": dk["bytes"] / dk["launches"],
                     "avg_us": dk["avg_us"], "launches": dk["launches"],
                     "share_of_solve": dk["seconds"] / tot_s},
        "roofline_band_unfused_equiv": band_equiv,
        "roofline_spmv": {"kernel": f"spmv ({linfo['layout']}, vtk_spmv)", "bound": "hbm",
                          "achieved": spmv_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": spmv_gbs / HBM_PEAK_GBS, "traffic": traffic_spmv,
                          "traffic_source": traffic_spmv_src,
                          "algorithmic_bytes_per_launch": B},
        "sec8d_reconciliation": recon,
        "kernels": {k: {"avg_us": round(v["avg_us"], 2), "gbs": round(v["gbs"], 1),
                        "launches": v["launches"], "share": round(v["seconds"] / tot_s, 4)}
                    for k, v in sorted(kprof.items(), key=lambda kv: -kv[1]["seconds"])},
        "cpu_baseline": None,
        "line_precond_solve": alt,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            A_host = A.download()
            out["cpu_baseline"] = cpu_baseline(args.config, A_host, b_host, args.bs, args.rtol,
                                               args.cpu_inner,
                                               (vk.vlasov_line_stride(params), args.seg) if args.prec == "line" else None,
                                               full=not args.cpu_sample, gpu_iters=iters / args.steps)
            cb = out["cpu_baseline"]
            if "full_solve_s" in cb:   # same-tolerance time to solution, GPU vs the reference path
                cb["gpu_solve_s"] = out["solve_ms_median"] / 1e3
                cb["time_to_solution_speedup"] = cb["full_solve_s"] / cb["gpu_solve_s"]
        except Exception as e:  # reported, never silently replaced
            out["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


# every source whose text reaches device code: the kernels, the headers they include (geometry
# constants and launch structs live in vtk_internal.hpp, the generator in vtk_vlasov.hpp)
KERNEL_SOURCES = ("vtk_kernels.hip", "vtk_band.hip", "vtk_device.hpp", "vtk_scalar.hpp", "vtk_internal.hpp",
                  "vtk_vlasov.hpp")


def kernels_sha16():
    """SHA-256 (16 hex digits) of the device sources, in a fixed order (tools/pmc_summary.py
    stamps its summaries with the same hash)."""
    import hashlib
    h = hashlib.sha256()
    for name in KERNEL_SOURCES:
        with open(os.path.join(ROOT, "vt-precondition_amd", "csrc", name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def pmc_traffic(cls, config, world):
    """(HBM bytes per launch of kernel class `cls`, source) from the newest committed rocprofv3
    PMC summary (profiles/rNN[_tag]_pmc_traffic.json, tools/pmc_summary.py) taken on the same
    config at one GPU AND on the same kernel source (its `kernels_sha16` must equal the hash of
    the vtk_kernels.hip being benched).  (None, why) otherwise: a summary of other kernels is
    never reported as this run's traffic."""
    import glob
    import re
    if world != 1:
        return None, "no PMC summary for multi-GPU runs"
    sha = kernels_sha16()
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")), reverse=True)
    stale = None
    for path in files:
        with open(path) as f:
            rec = json.load(f)
        m = re.match(r"r\d+_(c\d)_pmc_traffic\.json$", os.path.basename(path))
        cfg = rec.get("config") or (m.group(1).upper() if m else "C3")
        if cfg != config:
            continue
        if rec.get("kernels_sha16") != sha:
            stale = stale or os.path.basename(path)
            continue
        k = rec["kernels"].get(cls)
        if k is not None:
            return k["hbm_bytes_per_launch"], f"{os.path.basename(path)} (kernels {sha})"
    return None, (f"newest {config} summary {stale} profiles other kernel sources than {sha}" if stale
                  else f"no {config} PMC summary")


def params_nnz(dim, shape):
    import numpy as np
    n = int(np.prod(shape))
    if dim == 2:
        return 5 * n - 2 * shape[0]
    return 9 * n - 2 * (n // shape[2]) - 2 * (n // shape[3])


if __name__ == "__main__":
    main()
