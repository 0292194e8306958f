"""Multi-rank device path on the single-GPU test box: W processes share cuda:0 and talk through
the library's host-staged communicator (vtk_comm_init_host over gloo), so the row partition,
device-side column remap, halo exchange and the all-reduced Arnoldi scalars all run in the
real kernels.  (RCCL itself refuses several ranks on one GPU; the production bench uses it.)
Checks against the single-rank oracle:
  * each rank's SpMV rows and BJ blocks: bit-identical (halo columns keep the row order);
  * the distributed GMRES: same info, inner iterations +-1, ||x - x_ref|| / ||x_ref|| <= 1e-9.
"""
import json
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, case, outdir, from_host, orth):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import vtkrylov as vk
    from oracle import coracle, twin
    ctx = vk.Context(0)
    hc = ctx.comm_init_host(rank, world)
    p = twin.CONFIGS[case]
    align = p.shape[-1] if p.dim == 2 else (8 if p.dim == 1 else p.shape[-1] * p.shape[-2])
    planes = isinstance(from_host, str) and from_host.startswith("planes")
    if planes:   # slabs of whole x planes: the 4D grid rows hold across ranks (halo planes)
        align = p.shape[1] * p.shape[2] * p.shape[3]
        if from_host == "planes_ring":   # the LDS-ring step across ranks, 64 workgroups
            ctx.set_tuning("g4_ring", 64)
        elif from_host.startswith("planes_ring512"):   # ... and in 512-row groups, dots apart
            ctx.set_tuning("g4_ring", 2)
            ctx.set_tuning("g4_gr", 512)
        else:                            # the SELL grid-row split step (interior / boundary groups)
            ctx.set_tuning("g4_ring", 0)
    offs = vk.partition_rows(p.n, world, align)
    if from_host == "planes_ring512_uneven":   # slabs of 2 and 4 planes: rank-dependent ring grids
        offs = np.array([0, 2 * align, p.n], dtype=np.int64)
    rb, re_ = int(offs[rank]), int(offs[rank + 1])
    if from_host == "npz":   # this rank's row block of a SciPy archive (vtkrylov.load_npz)
        A = vk.load_npz(os.path.join(outdir, "A.npz"), ctx=ctx, offsets=offs)
    elif from_host:   # host CSR row block with global columns (vtk_csr_create path)
        ip, ix, d = coracle.generate(p, rb, re_)
        A = vk.csr_matrix((d, ix, ip), shape=(p.n, p.n), ctx=ctx, offsets=offs)
    else:           # device assembly of this rank's rows
        A = vk.vlasov_operator(vk.vlasov_params(p.dim, p.shape, fp32=p.fp32), ctx=ctx, offsets=offs)
    if planes:
        assert A.grid4 == tuple(p.shape[1:]), A.grid4
    # the line band is found in the CSR on every path (device assembly, host row blocks, npz)
    assert A.line_band == (p.shape[1] if p.dim == 2 else 0), A.line_band
    x = twin.rhs(p.n, seed=0xC0FFEE)
    y = A @ x[rb:re_]
    M = vk.block_jacobi(A, 8)
    inv = M.inverse()
    b = twin.rhs(p.n)
    ctx.profile(True)
    xs, info = vk.gmres(A, b[rb:re_], rtol=1e-8, M=M, orth=orth)
    st = vk.last_stats()
    classes = sorted(k for k, e in ctx.profile_read().items() if e["launches"] > 0)
    ctx.profile(False)
    gip, gix, gd = A.download()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), y=y, inv=inv, x=xs, info=info,
             iters=st.inner_iters, rb=rb, re=re_, halo=A.n_halo, gip=gip, gix=gix, gd=gd, band=st.band,
             line_band=A.line_band, line_values=A.line_values,
             errors=np.array(hc.errors, dtype=object).astype(str), classes=json.dumps(classes),
             commlog=json.dumps(hc.log))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("case,world,from_host,orth", [("S2", 2, False, "mgs"), ("S4", 3, False, "dcgs2"),
                                                       ("S2", 3, True, "dcgs2"), ("S4", 2, "npz", "dcgs2"),
                                                       ("C1", 2, False, "mgs"),
                                                       ("C1", 2, False, "dcgs2"), ("C1", 3, False, "dcgs2"),
                                                       ("S2", 2, True, "dcgs2"), ("S2", 4, False, "dcgs2"),
                                                       ("S4", 3, "planes", "dcgs2"), ("S4", 2, "planes_ring", "dcgs2"),
                                                       ("S4", 3, "planes_ring", "dcgs2"), ("S4F", 2, "planes_ring", "mgs"),
                                                       ("S4", 2, "planes_ring512", "dcgs2"),
                                                       ("S4", 2, "planes_ring512_uneven", "dcgs2"), ("S4", 2, "planes", "dcgs2")])
def test_ranks_sharing_one_gpu(tmp_path, case, world, from_host, orth):
    import torch.multiprocessing as mp

    from oracle import coracle, twin
    if from_host == "npz":
        from vtkrylov import npz
        p = twin.CONFIGS[case]
        ip, ix, d = coracle.generate(p)
        npz.save_npz_arrays(tmp_path / "A.npz", ip, ix, d, (p.n, p.n))
    mp.spawn(_worker, args=(world, _free_port(), case, str(tmp_path), from_host, orth), nprocs=world, join=True)
    p = twin.CONFIGS[case]
    ip, ix, d = coracle.generate(p)
    inv_ref = coracle.bj_setup(ip, ix, d, 8)
    y_ref = coracle.spmv(ip, ix, d, twin.rhs(p.n, seed=0xC0FFEE))
    b = twin.rhs(p.n)
    ref = coracle.gmres(ip, ix, d, b, inv_ref, rtol=1e-8)
    xs = np.zeros(p.n)
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz", allow_pickle=False)
        rb, re_ = int(z["rb"]), int(z["re"])
        assert z["errors"].size == 0, z["errors"]
        if world > 1 and re_ > rb:
            assert int(z["halo"]) > 0
        assert np.array_equal(z["gix"], ix[ip[rb]:ip[re_]])          # download maps back to global
        assert np.array_equal(z["y"], y_ref[rb:re_])                  # bitwise SpMV rows
        assert np.array_equal(z["inv"], inv_ref[rb // 8:(re_ + 7) // 8])
        # 2D operators under DCGS2 run the line-band step across ranks (ghost lines exchanged)
        expect_band = p.dim == 2 and orth == "dcgs2"
        assert int(z["band"]) == int(expect_band), (int(z["band"]), int(z["line_band"]))
        if p.dim == 2:   # separable values AND canonical rows on every rank (the halo lines' place
            # in the global column order: canon_order_xv's xord), so every rank runs the code-free step
            assert int(z["line_values"]) == 2, (r, int(z["line_values"]))
        assert int(z["info"]) == ref.info == 0
        assert abs(int(z["iters"]) - ref.inner_iters) <= 1
        xs[rb:re_] = z["x"]
    rel = np.linalg.norm(xs - ref.x) / np.linalg.norm(ref.x)
    assert rel <= 1e-9, rel
    # the step kernel that ran: the 4D ring across ranks books its boundary
    # planes as spmv_bj_bd, the SELL split step as spmv_bj_dc_bd
    for r in range(world):
        cls = set(json.loads(str(np.load(tmp_path / f"rank{r}.npz", allow_pickle=False)["classes"])))
        if orth != "dcgs2":   # (MGS: SciPy's sequence, precond_matvec's launches)
            continue
        if isinstance(from_host, str) and from_host.startswith("planes_ring"):
            assert "spmv_bj_bd" in cls and "spmv_bj_dc_bd" not in cls, sorted(cls)
        elif from_host == "planes":
            assert "spmv_bj_dc_bd" in cls and "spmv_bj_bd" not in cls, sorted(cls)
    # every rank issued the communicator sequence RCCL could run
    from vtkrylov.comm import check_sequences
    check_sequences([json.loads(str(np.load(tmp_path / f"rank{r}.npz", allow_pickle=False)["commlog"]))
                     for r in range(world)])


def _fail_worker(rank, world, port, case, outdir, fail_rank, fail_step, planes):
    """One rank of a solve in which rank `fail_rank` fails its DCGS2 step `fail_step` (the
    fail_step test hook: as if that step's launch had been refused), then a clean solve on the
    same communicator."""
    import time
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import vtkrylov as vk
    from oracle import twin
    ctx = vk.Context(0)
    hc = ctx.comm_init_host(rank, world)
    p = twin.CONFIGS[case]
    if planes:   # whole x planes: the 4D ring step across ranks (halo planes, split launches)
        align = p.shape[1] * p.shape[2] * p.shape[3]
        ctx.set_tuning("g4_ring", 64)
    else:
        align = p.shape[-1]
    offs = vk.partition_rows(p.n, world, align)
    rb, re_ = int(offs[rank]), int(offs[rank + 1])
    A = vk.vlasov_operator(vk.vlasov_params(p.dim, p.shape, fp32=p.fp32), ctx=ctx, offsets=offs)
    M = vk.block_jacobi(A, 8)
    b = twin.rhs(p.n)[rb:re_]
    if rank == fail_rank:
        ctx.set_tuning("fail_step", fail_step)
    t = time.perf_counter()
    status, msg = 0, ""
    try:
        vk.gmres(A, b, rtol=1e-8, M=M, orth="dcgs2")
    except vk._abi.VtkError as e:
        status, msg = e.status, str(e)
    elapsed = time.perf_counter() - t
    ops_failed = len(hc.log)
    ctx.set_tuning("fail_step", -1)
    x2, info2 = vk.gmres(A, b, rtol=1e-8, M=M, orth="dcgs2")
    st = vk.last_stats()
    # the kernel-level pin of the step's launch: the ring kernel across ranks in the
    # solver's interior / boundary form == the SELL grid-row SpMV + BJ epilogue, bit for bit
    xr = twin.rhs(p.n, seed=0xC0FFEE)[rb:re_]
    w_step = A.precond_matvec(M, xr)
    with ctx.tuning(g4_ring=0):
        w_sell = A.precond_matvec(M, xr)
    np.savez(os.path.join(outdir, f"fail{rank}.npz"), status=status, msg=msg, elapsed=elapsed, x2=x2, info2=info2,
             iters2=st.inner_iters, band=st.band, rb=rb, re=re_, ops_failed=ops_failed, w_step=w_step, w_sell=w_sell,
             errors=np.array(hc.errors, dtype=object).astype(str), commlog=json.dumps(hc.log))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("case,world,fail_rank,fail_step,planes", [("S2", 2, 1, 3, False), ("C1", 3, 0, 5, False),
                                                                   ("S4", 2, 1, 2, True), ("S4", 3, 2, 0, True)])
def test_peer_failure_is_contained(tmp_path, case, world, fail_rank, fail_step, planes):
    """A rank whose DCGS2 step fails mid-solve: it votes the failure into the
    step's all-reduce and keeps issuing the same collectives, so every rank leaves the solve at
    that step -- the failing one with its own error, the others with VTK_ERR_PEER -- within a
    bounded time and with the communicator sequence intact; the next solve on the same
    communicator converges as a clean one does."""
    import torch.multiprocessing as mp

    import vtkrylov as vk
    from oracle import coracle, twin
    mp.spawn(_fail_worker, args=(world, _free_port(), case, str(tmp_path), fail_rank, fail_step, planes),
             nprocs=world, join=True)
    p = twin.CONFIGS[case]
    ip, ix, d = coracle.generate(p)
    ref = coracle.gmres(ip, ix, d, twin.rhs(p.n), coracle.bj_setup(ip, ix, d, 8), rtol=1e-8)
    z = [np.load(tmp_path / f"fail{r}.npz", allow_pickle=False) for r in range(world)]
    xs = np.zeros(p.n)
    for r in range(world):
        assert z[r]["errors"].size == 0, z[r]["errors"]
        st, msg = int(z[r]["status"]), str(z[r]["msg"])
        if r == fail_rank:
            assert st == vk._abi.ERR_HIP and "injected failure" in msg, (st, msg)
        else:
            assert st == vk._abi.ERR_PEER and "peer rank failed" in msg, (st, msg)
        assert float(z[r]["elapsed"]) < 30.0
        assert int(z[r]["band"]) == int(p.dim == 2)
        assert int(z[r]["info2"]) == 0 and abs(int(z[r]["iters2"]) - ref.inner_iters) <= 1
        xs[int(z[r]["rb"]):int(z[r]["re"])] = z[r]["x2"]
        assert np.array_equal(z[r]["w_step"], z[r]["w_sell"]), r
    assert np.linalg.norm(xs - ref.x) / np.linalg.norm(ref.x) <= 1e-9
    # every rank left the failed solve after the same collectives, and the whole run (failed solve
    # + clean solve) is one sequence RCCL could execute
    assert len({int(q["ops_failed"]) for q in z}) == 1
    from vtkrylov.comm import check_sequences
    check_sequences([json.loads(str(q["commlog"])) for q in z])
