"""Row-partitioned solves at the headline sizes (VERDICT r2 "next" 1, r3 "next" 1; SURVEY §8e,
BASELINE configs 4 and 5): C3 (20M rows) on 2, 4 and 8 ranks and C4 (50M rows, fp32 values) on
2, 4 and 8 ranks -- the geometries the driver's 8-GPU scaling run executes (C3/8: 3 125 x-lines
per rank; C4/8: 25 x-planes per rank, 2 MB halos per side) --
every rank its x-slab of the operator assembled on the device, all ranks sharing the one GPU
of the test box through the library's host-staged communicator (vtk_comm_init_host over gloo:
the same partition, halo plan, device column remap, per-step all-reduce and -- on C3 -- the
line-band step's per-step ghost-line exchange as the RCCL path; RCCL itself refuses several
ranks on one GPU).

Bars: the same as tests/test_gpu_large.py against tests/golden/golden_large.json (SciPy
1.15.3's GMRES(20) + BJ(8) at C3 and C4): info 0 on every
rank, inner iterations +-1, ||x|| relative 1e-9, x[:8], x[-8:] and the 64 strided entries
within 1e-8 of max|x| (1e-6 when the counts differ by one), and the true residual of the
assembled x recomputed on the host by the oracle's SpMV <= rtol ||b||.  C3 also asserts that
the band step ran across the ranks (stats.band, halo = the two neighbour lines).
"""
import json
import os
import socket

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, case, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import vtkrylov as vk
    from oracle import twin
    ctx = vk.Context(0)
    hc = ctx.comm_init_host(rank, world)
    p = twin.CONFIGS[case]
    align = p.shape[-1] if p.dim == 2 else int(np.prod(p.shape[1:]))   # whole x-lines / x-planes
    offs = vk.partition_rows(p.n, world, align)
    rb, re_ = int(offs[rank]), int(offs[rank + 1])
    A = vk.vlasov_operator(vk.vlasov_params(p.dim, p.shape, fp32=p.fp32), ctx=ctx, offsets=offs)
    M = vk.block_jacobi(A, 8)
    b = vk.rhs_splitmix(p.n, r0=rb, r1=re_)
    x, info = vk.gmres(A, b, rtol=1e-8, M=M)
    st = vk.last_stats()
    np.save(os.path.join(outdir, f"x{rank}.npy"), x)
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), info=info, iters=st.inner_iters, band=st.band,
             rb=rb, re=re_, halo=A.n_halo, line_band=A.line_band, mode=M.mode, layout=A.layout_info()["layout"],
             separable=A.line_separable, line_values=A.line_values,
             errors=np.array(hc.errors, dtype=object).astype(str), commlog=json.dumps(hc.log))
    M.close()
    A.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("case,world", [("C3", 2), ("C3", 4), ("C3", 8), ("C4", 2), ("C4", 4), ("C4", 8)])
def test_row_partitioned_full_size(tmp_path, golden_large, case, world):
    import torch.multiprocessing as mp

    from oracle import coracle, twin
    mp.spawn(_worker, args=(world, _free_port(), case, str(tmp_path)), nprocs=world, join=True)
    p = twin.CONFIGS[case]
    g = golden_large[case]["gmres_bj8"]
    x = np.empty(p.n)
    iters = []
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz", allow_pickle=False)
        rb, re_ = int(z["rb"]), int(z["re"])
        assert z["errors"].size == 0, z["errors"]
        assert int(z["info"]) == g["info"] == 0
        assert str(z["layout"]) == "sell" and str(z["mode"]) == "tridiag"
        if p.dim == 2:   # the line-band step across ranks: halo = the two neighbour lines
            assert int(z["line_band"]) == p.shape[1] and int(z["halo"]) == 2 * p.shape[1]
            assert int(z["band"]) == 1
            assert bool(z["separable"])   # the distributed line-separable tables (halo lines)
            assert int(z["line_values"]) == 2, (r, int(z["line_values"]))   # ... and canonical rows
        else:            # 4D: the halo is the two neighbour x-planes
            assert int(z["halo"]) == 2 * int(np.prod(p.shape[1:]))
        iters.append(int(z["iters"]))
        x[rb:re_] = np.load(tmp_path / f"x{r}.npy", allow_pickle=False)
    assert len(set(iters)) == 1, iters          # every rank ran the same Arnoldi steps
    # the communicator sequence the RCCL transport would issue -- the same
    # collectives in the same order on every rank, every send matched by the peer's receive
    from vtkrylov.comm import check_sequences
    logs = [json.loads(str(np.load(tmp_path / f"rank{r}.npz", allow_pickle=False)["commlog"])) for r in range(world)]
    nops = check_sequences(logs)
    kinds = {op[0] for op in logs[0]}
    assert nops > 2 * iters[0] and "allreduce" in kinds and "alltoallv" in kinds, (nops, kinds)
    assert g["source"].startswith("scipy.sparse.linalg.gmres")
    it = iters[0]
    assert abs(it - g["inner_iters"]) <= 1, (it, g["inner_iters"])
    assert np.linalg.norm(x) == pytest.approx(g["x_norm2"], rel=1e-9)
    scale = max(np.max(np.abs(g["x_sample"])), np.max(np.abs(g["x_first8"])))
    tol = (1e-8 if it == g["inner_iters"] else 1e-6) * scale
    np.testing.assert_allclose(x[:8], g["x_first8"], rtol=0, atol=tol)
    np.testing.assert_allclose(x[-8:], g["x_last8"], rtol=0, atol=tol)
    s = g["x_sample_stride"]
    np.testing.assert_allclose(x[::s][:64], g["x_sample"], rtol=0, atol=tol)
    ip, ix, d = coracle.generate(p)
    b = twin.rhs(p.n)
    res = np.linalg.norm(b - coracle.spmv(ip, ix, d, x))
    assert res <= 1e-8 * g["b_norm2"], (res, g["b_norm2"])
