"""World-size-2/3 gloo tests on the CPU (no GPU): the N>1 path's host logic.

* the product's row partition and halo plan (vtk_partition_rows / vtk_halo_plan), driven
  through the same schedule the device driver uses (halo send/recv before every SpMV, one
  all-reduce per Arnoldi scalar), with the oracle's local SpMV / BJ apply as the arithmetic:
  the distributed GMRES must reproduce the single-rank oracle (SciPy's algorithm);
* the host-staged communicator hooks (vtkrylov.comm.HostComm) the multi-rank GPU test uses.
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class DistOps:
    """Distributed SpMV / BJ / dot of one rank, mirroring vtk_api.cpp's multi-rank schedule."""

    def __init__(self, vk, dist, p, offs, rank, world, prec="bj", seg=0):
        from oracle import coracle
        self.dist, self.rank, self.world = dist, rank, world
        self.rb, self.re = int(offs[rank]), int(offs[rank + 1])
        ip, ix, d = coracle.generate(p, self.rb, self.re)
        self.ip, self.d = ip, d
        self.loc, self.halo_cols, self.recv_cnt = vk.halo_plan(p.n, offs, rank, ix)
        self.loc = self.loc.astype(np.int32)
        # everyone learns what it must send (counts allgather), then the requested ids travel
        # to their owners (alltoallv) — setup_halo() in vtk_api.cpp
        import torch
        cnt = torch.from_numpy(self.recv_cnt.astype(np.int64))
        allc = [torch.empty(world, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allc, cnt)
        self.send_cnt = np.array([int(allc[q][rank]) for q in range(world)])
        req = torch.from_numpy(self.halo_cols.astype(np.int64))
        got = torch.empty(int(self.send_cnt.sum()), dtype=torch.int64)
        dist.all_to_all_single(got, req, self.send_cnt.tolist(), self.recv_cnt.tolist())
        self.send_idx = got.numpy() - self.rb
        assert np.all((self.send_idx >= 0) & (self.send_idx < self.re - self.rb))
        self.inv = coracle.bj_setup(ip, self.loc, d, 8)   # blocks never reach halo columns
        # line Jacobi: rank-local lines (vtk_linejacobi_create cuts segments at the row block)
        self.lf = None
        if prec == "line":
            stride = 1 if p.dim == 1 else (p.shape[1] if p.dim == 2 else p.n // p.shape[0])
            self.lf = coracle.line_setup(ip, ix, d, stride, seg, row0=self.rb)

    def halo(self, xl):
        import torch
        out = torch.empty(len(self.halo_cols), dtype=torch.float64)
        self.dist.all_to_all_single(out, torch.from_numpy(xl[self.send_idx].copy()),
                                    self.recv_cnt.tolist(), self.send_cnt.tolist())
        return out.numpy()

    def matvec(self, xl):
        from oracle import coracle
        return coracle.spmv(self.ip, self.loc, self.d, np.concatenate([xl, self.halo(xl)]))

    def psolve(self, r):
        from oracle import coracle
        if self.lf is not None:
            return coracle.line_apply(self.lf, r)
        return coracle.bj_apply(self.inv, r)

    def dot(self, a, b):
        import torch
        t = torch.tensor([float(np.dot(a, b))], dtype=torch.float64)
        self.dist.all_reduce(t)
        return float(t.item())


def dist_gmres(ops, b, rtol, restart=20, maxiter=1000):
    """iterative.py:692-841 with every dot/norm all-reduced and every matvec halo-exchanged."""
    from oracle import coracle
    eps = np.finfo(float).eps
    nrm = lambda v: np.sqrt(ops.dot(v, v))
    bnrm2 = nrm(b)
    atol = rtol * bnrm2
    x = np.zeros_like(b)
    Mb = nrm(ops.psolve(b))
    pmf = 1.0
    ptol = Mb * min(pmf, atol / bnrm2)
    V = np.empty((restart + 1, b.shape[0]))
    h = np.zeros((restart, restart + 1))
    giv = np.zeros((restart, 2))
    inner = 0
    r = b - ops.matvec(x)
    for it in range(maxiter):
        V[0] = ops.psolve(r)
        t = nrm(V[0])
        V[0] *= 1.0 / t
        S = np.zeros(restart + 1)
        S[0] = t
        brk = False
        for col in range(restart):
            w = ops.psolve(ops.matvec(V[col]))
            h0 = nrm(w)
            for k in range(col + 1):
                hk = ops.dot(V[k], w)
                h[col, k] = hk
                w -= hk * V[k]
            h1 = nrm(w)
            h[col, col + 1] = h1
            V[col + 1] = w
            if h1 <= eps * h0:
                h[col, col + 1] = 0
                brk = True
            else:
                V[col + 1] *= 1.0 / h1
            for k in range(col):
                c, s = giv[k]
                n0, n1 = h[col, k], h[col, k + 1]
                h[col, k], h[col, k + 1] = c * n0 + s * n1, -s * n0 + c * n1
            c, s, mag = coracle.lartg(h[col, col], h[col, col + 1])
            giv[col] = c, s
            h[col, col], h[col, col + 1] = mag, 0
            tmp = -s * S[col]
            S[col], S[col + 1] = c * S[col], tmp
            presid = abs(tmp)
            inner += 1
            if presid <= ptol or brk:
                break
        if h[col, col] == 0:
            S[col] = 0
        y = S[:col + 1].copy()
        for k in range(col, 0, -1):
            if y[k] != 0:
                y[k] /= h[k, k]
                y[:k] -= y[k] * h[k, :k]
        if y[0] != 0:
            y[0] /= h[0, 0]
        x += y @ V[:col + 1]
        r = b - ops.matvec(x)
        rnorm = nrm(r)
        if rnorm <= atol or brk:
            break
        pmf = max(eps, 0.25 * pmf) if presid <= ptol else min(1.0, 1.5 * pmf)
        ptol = presid * min(pmf, atol / rnorm)
    return x, (0 if rnorm <= atol else maxiter), inner


def _worker(rank, world, port, case, outdir, prec="bj", seg=0):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import vtkrylov as vk
    from oracle import twin
    p = twin.CONFIGS[case]
    align = p.shape[-1] if p.dim == 2 else (8 if p.dim == 1 else p.shape[-1] * p.shape[-2])
    offs = vk.partition_rows(p.n, world, align)
    ops = DistOps(vk, dist, p, offs, rank, world, prec, seg)
    b = twin.rhs(p.n)[ops.rb:ops.re]
    x, info, inner = dist_gmres(ops, b, 1e-8)
    # the host-staged communicator hooks, called the way the library calls them
    from vtkrylov.comm import HostComm
    hc = HostComm()
    buf = np.array([rank + 1.0, 2.0 * rank])
    assert hc._allreduce(None, buf.ctypes.data_as(C.POINTER(C.c_double)), 2) == 0
    tri = world * (world + 1) / 2
    assert buf.tolist() == [tri, float(world * (world - 1))]
    scnt = np.array([q + 1 for q in range(world)], np.int64)         # q+1 doubles to rank q
    soff = np.concatenate([[0], np.cumsum(scnt)[:-1]]).astype(np.int64)
    rcnt = np.full(world, rank + 1, np.int64)                         # rank+1 doubles from each
    roff = np.concatenate([[0], np.cumsum(rcnt)[:-1]]).astype(np.int64)
    sb = np.concatenate([np.full(q + 1, 100.0 * rank + q) for q in range(world)])
    rbuf = np.zeros(int(rcnt.sum()))
    P64 = lambda a: a.ctypes.data_as(C.POINTER(C.c_int64))
    assert hc._alltoallv(None, sb.ctypes.data, P64(scnt), P64(soff), rbuf.ctypes.data,
                         P64(rcnt), P64(roff), 8) == 0
    exp = np.concatenate([np.full(rank + 1, 100.0 * q + rank) for q in range(world)])
    assert np.array_equal(rbuf, exp), (rbuf, exp)
    g_in = np.array([rank * 10, rank * 10 + 1], np.int64)
    g_out = np.zeros(2 * world, np.int64)
    assert hc._allgather(None, g_in.ctypes.data, g_out.ctypes.data, 16) == 0
    assert g_out.tolist() == [v for q in range(world) for v in (q * 10, q * 10 + 1)]
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), x=x, info=info, inner=inner, rb=ops.rb, re=ops.re,
             halo=len(ops.halo_cols))
    dist.destroy_process_group()


@pytest.mark.parametrize("case,world", [("S2", 2), ("S4", 2), ("C0", 3)])
def test_distributed_gmres_matches_single_rank(tmp_path, case, world):
    import torch.multiprocessing as mp

    from oracle import coracle, twin
    mp.spawn(_worker, args=(world, _free_port(), case, str(tmp_path)), nprocs=world, join=True)
    p = twin.CONFIGS[case]
    ip, ix, d = coracle.generate(p)
    ref = coracle.gmres(ip, ix, d, twin.rhs(p.n), coracle.bj_setup(ip, ix, d, 8), rtol=1e-8)
    x = np.zeros(p.n)
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        assert int(z["halo"]) > 0
        assert int(z["info"]) == ref.info == 0
        assert abs(int(z["inner"]) - ref.inner_iters) <= 1
        x[int(z["rb"]):int(z["re"])] = z["x"]
    assert np.linalg.norm(x - ref.x) / np.linalg.norm(ref.x) <= 1e-10


@pytest.mark.parametrize("case,world,seg", [("S2", 2, 8), ("S4", 2, 3)])
def test_distributed_line_jacobi_matches_single_rank(tmp_path, case, world, seg):
    """Line Jacobi with segments that divide every rank's x-range: the rank-local M equals the
    single-rank M, so the distributed solve reproduces the single-rank oracle."""
    import torch.multiprocessing as mp

    from oracle import coracle, twin
    mp.spawn(_worker, args=(world, _free_port(), case, str(tmp_path), "line", seg), nprocs=world, join=True)
    p = twin.CONFIGS[case]
    ip, ix, d = coracle.generate(p)
    stride = p.shape[1] if p.dim == 2 else p.n // p.shape[0]
    ref = coracle.gmres(ip, ix, d, twin.rhs(p.n), coracle.line_setup(ip, ix, d, stride, seg), rtol=1e-8)
    x = np.zeros(p.n)
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        assert int(z["info"]) == ref.info == 0
        assert abs(int(z["inner"]) - ref.inner_iters) <= 1
        x[int(z["rb"]):int(z["re"])] = z["x"]
    assert np.linalg.norm(x - ref.x) / np.linalg.norm(ref.x) <= 1e-10


class _FakeCtx:
    """Stands in for vtkrylov.Context in init_rccl: rank 0's unique id, every rank's comm_init."""

    def __init__(self, rank):
        self.rank = rank
        self.init_args = None

    def unique_id(self):
        assert self.rank == 0, "only rank 0 creates the RCCL unique id"
        return bytes((7 * i + 3) % 256 for i in range(128))

    def comm_init(self, rank, world, uid):
        self.init_args = (rank, world, uid)


def _rccl_uid_worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vtkrylov import comm
    ctx = _FakeCtx(rank)
    comm.init_rccl(ctx, rank, world)
    r, w, uid = ctx.init_args
    with open(os.path.join(outdir, f"uid{rank}.bin"), "wb") as f:
        f.write(bytes([r, w]) + uid)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_init_rccl_broadcasts_rank0_unique_id(tmp_path, world):
    """bench.py's N>1 set-up (vtkrylov.comm.init_rccl over the gloo group the launcher makes):
    every rank calls vtk_comm_init with its own rank, the world size and rank 0's 128-byte RCCL
    unique id -- the host half of the RCCL path the driver's multi-GPU run is the first to use."""
    import torch.multiprocessing as mp
    mp.spawn(_rccl_uid_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    want = bytes((7 * i + 3) % 256 for i in range(128))
    for r in range(world):
        got = (tmp_path / f"uid{r}.bin").read_bytes()
        assert got[0] == r and got[1] == world and got[2:] == want, r
