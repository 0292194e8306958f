"""Communicator set-up for multi-rank runs (one rank per GPU).

* ``init_rccl(ctx, rank, world, pg)`` — production: rank 0 creates the RCCL unique id, the
  torch.distributed process group (any backend; used only for this broadcast) carries it,
  every rank calls ``vtk_comm_init``.  Data-path collectives are RCCL calls the library
  issues on its own stream (halo send/recv over xGMI, scalar all-reduces).
* ``HostComm`` — test transport: the library's ``vtk_host_comm`` hooks implemented with
  torch.distributed on CPU tensors (gloo).  It lets several ranks share one GPU (which RCCL
  refuses), so the multi-rank device code runs on the single-GPU test box.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi
from ._abi import check, lib

ALLRED = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_int64)
A2AV = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                   C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.c_int64)
AGATH = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64)


class _HostCommStruct(C.Structure):
    _fields_ = [("user", C.c_void_p), ("allreduce_sum_f64", ALLRED), ("alltoallv", A2AV),
                ("allgather", AGATH)]




def _bytes_view(ptr, nbytes):
    if nbytes == 0:
        return np.empty(0, np.uint8)
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), shape=(nbytes,))


class HostComm:
    """vtk_host_comm hooks over a torch.distributed process group (CPU tensors)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.errors = []
        # every communicator operation the library issued, in order: ("allreduce", count),
        # ("alltoallv", elem_bytes, send counts per peer, recv counts per peer), ("allgather",
        # bytes) -- the sequence the RCCL transport would issue at the same points (DESIGN.md §6:
        # every rank must issue the same collectives, and matched send/recv pairs)
        self.log = []
        self._cbs = (ALLRED(self._allreduce), A2AV(self._alltoallv), AGATH(self._allgather))
        self.struct = _HostCommStruct(None, *self._cbs)

    def _guard(self, fn, *a):
        try:
            fn(*a)
            return 0
        except Exception as e:  # surfaced by the library as VTK_ERR_STATE
            self.errors.append(repr(e))
            return 1

    def _allreduce(self, user, buf, count):
        self.log.append(("allreduce", int(count)))

        def go():
            import torch
            a = np.ctypeslib.as_array(buf, shape=(count,))
            t = torch.from_numpy(a)
            self.dist.all_reduce(t, group=self.group)
        return self._guard(go)

    def _alltoallv(self, user, sb, scnt, soff, rb, rcnt, roff, eb):
        self.log.append(("alltoallv", int(eb), [int(scnt[q]) for q in range(self.world)],
                         [int(rcnt[q]) for q in range(self.world)]))

        def go():
            import torch
            W = self.world
            sc = [int(scnt[q]) * eb for q in range(W)]
            rc = [int(rcnt[q]) * eb for q in range(W)]
            for q in range(1, W):   # the library packs contiguously
                assert soff[q] == soff[q - 1] + scnt[q - 1] and roff[q] == roff[q - 1] + rcnt[q - 1]
            sv = torch.from_numpy(_bytes_view(sb, sum(sc)).copy())
            out = torch.empty(sum(rc), dtype=torch.uint8)
            self.dist.all_to_all_single(out, sv, rc, sc, group=self.group)
            _bytes_view(rb, sum(rc))[:] = out.numpy()
        return self._guard(go)

    def _allgather(self, user, sb, rb, nbytes):
        self.log.append(("allgather", int(nbytes)))

        def go():
            import torch
            W = self.world
            mine = torch.from_numpy(_bytes_view(sb, nbytes).copy())
            outs = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(W)]
            self.dist.all_gather(outs, mine, group=self.group)
            rv = _bytes_view(rb, nbytes * W)
            for q in range(W):
                rv[q * nbytes:(q + 1) * nbytes] = outs[q].numpy()
        return self._guard(go)


def check_sequences(logs) -> int:
    """Every rank's communicator log (HostComm.log, rank order) describes one run that RCCL could
    execute: the same operation kinds and sizes at every position on every rank, and at every
    alltoallv each send count matched by the peer's receive count (a rank with no neighbours
    takes part with zero counts).  Returns the number of operations; AssertionError otherwise."""
    W = len(logs)
    n = len(logs[0])
    assert all(len(lg) == n for lg in logs), [len(lg) for lg in logs]
    for i in range(n):
        ops = [lg[i] for lg in logs]
        kind = ops[0][0]
        assert all(o[0] == kind for o in ops), (i, [o[0] for o in ops])
        if kind == "alltoallv":
            assert all(o[1] == ops[0][1] for o in ops), (i, "element size")
            for r in range(W):
                for q in range(W):
                    assert ops[r][2][q] == ops[q][3][r], (i, r, q, ops[r][2][q], ops[q][3][r])
        else:
            assert all(o[1] == ops[0][1] for o in ops), (i, kind, [o[1] for o in ops])
    return n


def init_host(ctx, rank: int, world: int, group=None) -> HostComm:
    hc = HostComm(group)
    check(lib().vtk_comm_init_host(ctx.handle, rank, world, C.byref(hc.struct)), ctx.handle)
    ctx.rank, ctx.world = rank, world
    ctx._host_comm = hc   # keep the callbacks alive with the context
    return hc


def init_rccl(ctx, rank: int, world: int, group=None):
    import torch
    import torch.distributed as dist
    uid = ctx.unique_id() if rank == 0 else bytes(128)
    t = torch.tensor(list(uid), dtype=torch.uint8)
    dist.broadcast(t, 0, group=group)
    ctx.comm_init(rank, world, bytes(t.tolist()))
