"""The production RCCL transport on the one-GPU box: a one-rank RCCL communicator
(VTK_COMM_SOLO=1) runs every distributed code path of the library — halo plan and (empty)
grouped send/recv on the comm stream, interior/boundary split launches with their events,
in-place all-reduces of the partial vectors, DCGS2's finalize + all-reduce of the scalars —
through ncclCommInitRank / ncclAllReduce / ncclAllGather / ncclSend / ncclRecv.  Results must
meet the single-GPU bars.  (Several ranks on one GPU go through the host-staged transport in
test_gpu_multirank.py: RCCL refuses duplicate GPUs.)"""
import numpy as np
import pytest

from oracle import coracle, twin

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def solo(vk_lib):
    import os
    os.environ["VTK_COMM_SOLO"] = "1"
    try:
        ctx = vk_lib.Context(0)
        ctx.comm_init(0, 1, vk_lib.Context.unique_id())
    finally:
        del os.environ["VTK_COMM_SOLO"]
    return ctx


@pytest.mark.parametrize("layout", ["sell", "csr"])
@pytest.mark.parametrize("orth", ["mgs", "dcgs2"])
def test_rccl_solo_gmres(vk_lib, solo, layout, orth):
    vk = vk_lib
    p = twin.CONFIGS["C1"]
    A = vk.vlasov_operator(vk.vlasov_params(p.dim, p.shape), ctx=solo)
    A.set_layout(layout)
    assert A.n_halo == 0
    ip, ix, d = coracle.generate(p)
    x = twin.rhs(p.n, seed=0xC0FFEE)
    assert np.array_equal(A @ x, coracle.spmv(ip, ix, d, x))
    M = vk.block_jacobi(A, 8)
    b = twin.rhs(p.n)
    ref = coracle.gmres(ip, ix, d, b, coracle.bj_setup(ip, ix, d, 8), rtol=1e-8)
    solo.profile(True)
    xs, info = vk.gmres(A, b, rtol=1e-8, M=M, orth=orth)
    prof = solo.profile_read()
    solo.profile(False)
    st = vk.last_stats()
    assert info == ref.info == 0
    assert abs(st.inner_iters - ref.inner_iters) <= 1
    assert np.linalg.norm(xs - ref.x) / np.linalg.norm(ref.x) <= 1e-9
    assert "allreduce" in prof and prof["allreduce"]["launches"] > 0   # the RCCL path ran
    if orth == "dcgs2":
        # the distributed step (interior launch + finalize + all-reduce); one rank has no halo
        # and no boundary rows, so no exchange and no boundary launch
        assert "dc_finalize" in prof and "spmv_bj_dc" in prof
        assert "spmv_bj_dc_bd" not in prof and "halo" not in prof


@pytest.mark.parametrize("name", ["S4", "S4F"])
def test_rccl_solo_grid4(vk_lib, solo, name):
    """The 4D grid rows on the one-rank RCCL communicator: no neighbour planes, so the one-rank
    (periodic) form of the grid and of k_g4_ring runs inside the distributed code paths, x0 != 0
    so that the cycles start with the ring residual."""
    vk = vk_lib
    p = twin.CONFIGS[name]
    A = vk.vlasov_operator(vk.vlasov_params(p.dim, p.shape, fp32=p.fp32), ctx=solo)
    assert A.grid4 == tuple(p.shape[1:])
    ip, ix, d = coracle.generate(p)
    M = vk.block_jacobi(A, 8)
    b = twin.rhs(p.n)
    x0 = twin.rhs(p.n, seed=0xB0B) * 1e-3
    ref = coracle.gmres(ip, ix, d, b, coracle.bj_setup(ip, ix, d, 8), x0=x0, rtol=1e-8, restart=5)
    xs, info = vk.gmres(A, b, x0=x0, rtol=1e-8, M=M, restart=5)
    st = vk.last_stats()
    assert info == ref.info == 0
    assert abs(st.inner_iters - ref.inner_iters) <= 1
    assert np.linalg.norm(xs - ref.x) / np.linalg.norm(ref.x) <= 1e-9
