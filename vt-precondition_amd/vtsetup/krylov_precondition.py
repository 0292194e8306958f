"""vtsetup entry for the preconditioned-Krylov path.

Mirrors the reference's step-object convention — a class whose ``main()`` runs a fixed
sequence (hypervisor.py:589-594: deploy -> network -> tools -> vms -> env) — with the
solver's sequence: generate operator -> set up preconditioner -> solve -> report.  Errors
surface as exceptions that ``test_main`` turns into a return code, as in
vt_precondition.py:66-79.

    python -m vtsetup.krylov_precondition [--config C1] [--xml path] [--report out.json]
                                          [--operator-file matrix.npz] [--gpus N] [--comm host]

``run/gpus`` > 1 (or ``--gpus``): ``test_main`` starts one process per rank before anything
touches a GPU (the torch.distributed.run environment contract: RANK, WORLD_SIZE, MASTER_*);
each rank builds its x-slab of the operator (``vtkrylov.partition_rows`` on whole x-lines /
x-planes), joins the communicator (RCCL, or the host-staged transport with ``run/comm`` =
host, which lets ranks share one GPU) and solves its rows; rank 0 writes the report with the
max-over-ranks solve time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


class KrylovPrecondition:
    def __init__(self, cfg, ctx=None, rank: int = 0, world: int = 1, group=None):
        self.cfg = cfg
        self.ctx = ctx
        self.rank, self.world, self.group = rank, world, group
        self.offsets = None
        self.A = self.M = self.b = self.x = None
        self.result = {}

    def partition(self):
        """Row blocks of the ranks (world + 1 offsets on whole x-slabs; None on one rank)."""
        import vtkrylov as vk
        c = self.cfg
        if self.world == 1:
            return None
        if c.operator_file:
            from vtkrylov.npz import npz_shape
            n = npz_shape(c.operator_file)[0]
        else:
            n = 1
            for e in c.shape:
                n *= e
        return vk.partition_rows(n, self.world, c.slab_align())

    def generate_operator(self):
        """The config's Vlasov operator assembled on the device, or the SciPy archive named by
        operator/file (vtkrylov.load_npz) -- this rank's row block when there are several."""
        import vtkrylov as vk
        c = self.cfg
        self.ctx = self.ctx or vk.Context(c.device)
        t = time.perf_counter()
        self.offsets = self.partition()
        if c.operator_file:
            # the x-line structure of a 2D Vlasov archive is found by the library (line_len None)
            # and runs the fused band step, as a generated operator does; operator/line_len
            # requires (L) or refuses (0) it
            self.A = vk.load_npz(c.operator_file, ctx=self.ctx, offsets=self.offsets, line_len=c.line_len)
        else:
            p = vk.vlasov_params(c.dim, c.shape, fp32=c.fp32, **c.physics)
            self.A = vk.vlasov_operator(p, ctx=self.ctx, offsets=self.offsets)
            if c.line_len is not None and c.line_len != self.A.line_band:
                self.A.set_line_band(c.line_len)
        self.result["operator"] = {"n": self.A.n_global, "nnz": self._sum(self.A.nnz),
                                   "source": c.operator_file or f"vlasov {c.config}",
                                   "line_band": self.A.line_band, "line_values": self.A.line_values,
                                   "t_assemble_s": self._max(time.perf_counter() - t)}
        if self.world > 1:
            self.result["operator"]["rows_per_rank"] = [int(self.offsets[q + 1] - self.offsets[q])
                                                        for q in range(self.world)]

    def setup_preconditioner(self):
        import vtkrylov as vk
        t = time.perf_counter()
        c = self.cfg
        info = {"type": c.preconditioner}
        if c.preconditioner == "block_jacobi":
            self.M = vk.block_jacobi(self.A, c.block_size)
            info["block_size"] = c.block_size
        elif c.preconditioner == "line_jacobi":
            stride = c.line_stride
            if stride <= 0:
                if c.operator_file:
                    # the detected x-line length is the line stride of a 2D operator
                    stride = self.A.line_band
                    if stride <= 0:
                        raise ValueError("line_jacobi on an operator file without a detected x-line "
                                         "structure needs preconditioner/line_stride")
                else:
                    stride = vk.vlasov_line_stride(vk.vlasov_params(c.dim, c.shape))
            self.M = vk.line_jacobi(self.A, stride, c.line_segment)
            info.update(line_stride=stride, line_segment=c.line_segment)
        info["t_setup_s"] = self._max(time.perf_counter() - t)
        self.result["preconditioner"] = info

    def solve(self):
        import vtkrylov as vk
        c = self.cfg
        self.b = vk.rhs_splitmix(self.A.n_global, seed=c.seed, r0=self.A.row_begin, r1=self.A.row_end)
        self._barrier()
        self.x, info = vk.gmres(self.A, self.b, rtol=c.rtol, atol=c.atol, restart=c.restart,
                                maxiter=c.maxiter or None, M=self.M, orth=c.orth)
        st = vk.last_stats()
        t_solve = self._max(st.t_solve)
        self.result["solve"] = {"info": info, "inner_iters": st.inner_iters,
                                "restarts": st.restarts, "rnorm": st.rnorm, "bnorm": st.bnorm,
                                "t_solve_s": t_solve, "band_step": bool(st.band),
                                "iters_per_s": st.inner_iters / t_solve if t_solve else None}

    def gather_x(self):
        """The whole solution on rank 0 (None on the others; the local x on one rank)."""
        import numpy as np
        x = np.asarray(self.x)
        if self.world == 1:
            return x
        import torch.distributed as dist
        parts = [None] * self.world if self.rank == 0 else None
        dist.gather_object(x, parts, dst=0, group=self.group)
        return np.concatenate(parts) if self.rank == 0 else None

    def report(self):
        self.result["config"] = self.cfg.config
        self.result["ranks"] = self.world
        if self.world > 1:
            self.result["comm"] = self.cfg.comm
        if self.cfg.report and self.rank == 0:
            with open(self.cfg.report, "w") as f:
                json.dump(self.result, f, indent=1)
        return self.result

    def main(self):
        self.generate_operator()
        self.setup_preconditioner()
        self.solve()
        return self.report()

    # ---- collectives over the launch's process group (gloo; nothing on one rank) ----------
    def _reduce(self, v: float, op) -> float:
        if self.world == 1:
            return v
        import torch
        import torch.distributed as dist
        t = torch.tensor([float(v)], dtype=torch.float64)
        dist.all_reduce(t, op=op, group=self.group)
        return float(t[0])

    def _max(self, v: float) -> float:
        if self.world == 1:
            return v
        import torch.distributed as dist
        return self._reduce(v, dist.ReduceOp.MAX)

    def _sum(self, v) -> int:
        if self.world == 1:
            return v
        import torch.distributed as dist
        return int(self._reduce(v, dist.ReduceOp.SUM))

    def _barrier(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.barrier(group=self.group)


def launch_ranks(n: int, argv: list[str]) -> int:
    """One child process per rank running this entry with ``argv`` (the torch.distributed.run
    environment), started before this process touches a GPU.  A failing rank stops the others
    (exact PIDs).  Returns the first non-zero exit code (0 when all succeed)."""
    import signal
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env0 = dict(os.environ)
    env0.update({"WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1",
                 "MASTER_PORT": str(port), "PYTHONPATH": os.pathsep.join([pkg] + [p for p in
                 env0.get("PYTHONPATH", "").split(os.pathsep) if p])})
    env0.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = [subprocess.Popen([sys.executable, "-m", "vtsetup.krylov_precondition"] + list(argv),
                              env=dict(env0, RANK=str(r), LOCAL_RANK=str(r)))
             for r in range(n)]
    rc, live = 0, list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                if code != 1:   # 1: a rank finished without convergence (info != 0), not a failure
                    for q in live:
                        q.send_signal(signal.SIGTERM)
        time.sleep(0.1)
    return rc


def _rank_main(cfg, a) -> int:
    """One rank of a multi-rank run (WORLD_SIZE set by launch_ranks or torch.distributed.run)."""
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    try:
        if a.dry_run:   # the plumbing alone (no GPU): the partition every rank would build
            step = KrylovPrecondition(cfg, rank=rank, world=world)
            offs = step.partition()
            out = {"rank": rank, "world": world, "offsets": None if offs is None else [int(v) for v in offs],
                   "rows": None if offs is None else [int(offs[rank]), int(offs[rank + 1])]}
            outs = [None] * world if rank == 0 else None
            dist.gather_object(out, outs, dst=0)
            if rank == 0:
                print(json.dumps({"dry_run": True, "ranks": outs}))
            return 0
        import vtkrylov as vk
        from vtkrylov import comm as vkcomm
        ndev = max(vk.device_count(), 1)
        ctx = vk.Context((cfg.device + local) % ndev)
        if cfg.comm == "rccl":
            vkcomm.init_rccl(ctx, rank, world)
        else:
            vkcomm.init_host(ctx, rank, world)
        step = KrylovPrecondition(cfg, ctx=ctx, rank=rank, world=world)
        res = step.main()
        x = step.gather_x()
        if rank == 0:
            if a.x_out:
                import numpy as np
                np.save(a.x_out, x)
            print(json.dumps(res))
        return 0 if res["solve"]["info"] == 0 else 1
    finally:
        dist.destroy_process_group()


def test_main(argv=None) -> int:
    from .config import DEFAULT_XML, SolverConfig
    argv = sys.argv[1:] if argv is None else list(argv)
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--xml", default=DEFAULT_XML)
    ap.add_argument("--config")
    ap.add_argument("--report")
    ap.add_argument("--operator-file", help="SciPy save_npz CSR archive to solve")
    ap.add_argument("--preconditioner", choices=["block_jacobi", "line_jacobi", "none"])
    ap.add_argument("--orth", choices=["auto", "mgs", "dcgs2"])
    ap.add_argument("--gpus", type=int, help="ranks (overrides run/gpus)")
    ap.add_argument("--comm", choices=["rccl", "host"], help="transport (overrides run/comm)")
    ap.add_argument("--x-out", help="write the whole solution (.npy) from rank 0")
    ap.add_argument("--dry-run", action="store_true", help="ranks and partition only; no GPU")
    a = ap.parse_args(argv)
    try:
        cfg = SolverConfig.load(a.xml, config=a.config, report=a.report, operator_file=a.operator_file,
                                preconditioner=a.preconditioner, orth=a.orth, gpus=a.gpus, comm=a.comm)
        if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1:
            return _rank_main(cfg, a)
        if cfg.gpus > 1:
            return launch_ranks(cfg.gpus, argv)   # nothing has touched a GPU in this process
        if a.dry_run:
            print(json.dumps({"dry_run": True, "ranks": [{"rank": 0, "world": 1, "offsets": None}]}))
            return 0
        step = KrylovPrecondition(cfg)
        res = step.main()
        if a.x_out:
            import numpy as np
            np.save(a.x_out, np.asarray(step.x))
        print(json.dumps(res))
        return 0 if res["solve"]["info"] == 0 else 1
    except Exception as e:   # vt_precondition.py:70-71 style: report and fail
        print(f"vtsetup.krylov_precondition failed: {type(e).__name__}: {e}", file=sys.stderr)
        return 2


if __name__ == "__main__":
    sys.exit(test_main())
