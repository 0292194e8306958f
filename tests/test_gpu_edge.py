"""Edge cases of the device path: 1x1 and n < bs systems (padded BJ blocks), a partial last
block under the tridiagonal BJ mode, n below one SELL chunk, an empty system, b = 0; every
layout and BJ mode against the oracle."""
import numpy as np
import pytest

from oracle import coracle, twin

pytestmark = pytest.mark.gpu


def tridiag(n, seed=1):
    rng = np.random.default_rng(seed)
    rows, cols, vals = [], [], []
    for i in range(n):
        for c in (i - 1, i, i + 1):
            if 0 <= c < n:
                rows.append(i)
                cols.append(c)
                vals.append(4.0 + rng.random() if c == i else -1.0 + 0.2 * rng.random())
    ip = np.zeros(n + 1, np.int32)
    np.add.at(ip, np.asarray(rows) + 1, 1)
    return np.cumsum(ip).astype(np.int32), np.asarray(cols, np.int32), np.asarray(vals)


@pytest.mark.parametrize("n,bs", [(1, 8), (5, 8), (7, 4), (63, 8), (65, 4), (130, 2)])
@pytest.mark.parametrize("layout", ["sell", "sell32", "csr"])
@pytest.mark.parametrize("mode", ["inverse", "tridiag"])
def test_small_systems(gpu, vk_lib, n, bs, layout, mode):
    vk = vk_lib
    ip, ix, d = tridiag(n)
    A = vk.csr_matrix((d, ix, ip), shape=(n, n), ctx=gpu)
    A.set_layout(layout)
    x = twin.rhs(n, seed=0xC0FFEE)
    assert np.array_equal(A @ x, coracle.spmv(ip, ix, d, x))
    M = vk.block_jacobi(A, bs, mode=mode)
    assert M.mode == mode
    inv = coracle.bj_setup(ip, ix, d, bs)
    assert np.array_equal(M.inverse(), inv)
    b = twin.rhs(n)
    z = M @ b
    ref_z = coracle.bj_apply(inv, b)
    if mode == "inverse":
        assert np.array_equal(z, ref_z)
    else:
        np.testing.assert_allclose(z, ref_z, rtol=1e-12, atol=1e-14 * np.abs(ref_z).max())
    ref = coracle.gmres(ip, ix, d, b, inv, rtol=1e-10)
    xs, info = vk.gmres(A, b, rtol=1e-10, M=M)
    assert info == ref.info == 0
    assert abs(vk.last_stats().inner_iters - ref.inner_iters) <= 1
    np.testing.assert_allclose(xs, ref.x, rtol=1e-8, atol=1e-12)


def test_zero_rhs_and_empty(gpu, vk_lib):
    vk = vk_lib
    ip, ix, d = tridiag(100)
    A = vk.csr_matrix((d, ix, ip), shape=(100, 100), ctx=gpu)
    x, info = vk.gmres(A, np.zeros(100), M=vk.block_jacobi(A, 4))
    assert info == 0 and not x.any()                       # iterative.py: b = 0 -> x = 0
    E = vk.csr_matrix((np.zeros(0), np.zeros(0, np.int32), np.zeros(1, np.int32)), shape=(0, 0), ctx=gpu)
    assert (E @ np.zeros(0)).shape == (0,)
    with pytest.raises(ValueError):
        vk.gmres(E, np.zeros(0))


def test_device_csr_input(gpu, vk_lib):
    """CSR arrays already in HBM (VTK_PTR_DEVICE): the same operator as the host path, and a
    column index out of [0, n) is rejected by the device range check instead of
    reaching the SpMV gathers."""
    import torch
    vk = vk_lib
    n = 300
    ip, ix, d = tridiag(n)
    dev = torch.device("cuda", 0)
    A = vk.csr_matrix((torch.from_numpy(d).to(dev), torch.from_numpy(ix).to(dev), torch.from_numpy(ip).to(dev)),
                      shape=(n, n), ctx=gpu)
    x = twin.rhs(n, seed=0xC0FFEE)
    assert np.array_equal(A @ x, coracle.spmv(ip, ix, d, x))
    for bad in (n, -1, 1 << 30):
        ixb = ix.copy()
        ixb[n // 2] = bad
        with pytest.raises(ValueError, match="column index out of range"):
            vk.csr_matrix((torch.from_numpy(d).to(dev), torch.from_numpy(ixb).to(dev), torch.from_numpy(ip).to(dev)),
                          shape=(n, n), ctx=gpu)
        with pytest.raises(ValueError, match="column index out of range"):
            vk.csr_matrix((d, ixb, ip), shape=(n, n), ctx=gpu)


def test_device_csr_spare_capacity_and_stream(gpu, vk_lib):
    """Device CSR whose indices / data carry spare capacity past indptr[-1]: nnz is
    taken from indptr, the spare entries are ignored; the conversions run on a non-default torch
    stream and are complete before the library copies them."""
    import torch
    vk = vk_lib
    n = 257
    ip, ix, d = tridiag(n)
    dev = torch.device("cuda", 0)
    spare = 37
    ixs = np.concatenate([ix, np.full(spare, 1 << 30, np.int32)])   # garbage beyond nnz
    ds = np.concatenate([d, np.full(spare, np.nan)])
    s = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(s):
        td = torch.from_numpy(ds).to(dev, non_blocking=True).to(torch.float32).to(torch.float64)
        tix = torch.from_numpy(ixs.astype(np.int64)).to(dev)
        tip = torch.from_numpy(ip.astype(np.int64)).to(dev)
        A = vk.csr_matrix((td, tix, tip), shape=(n, n), ctx=gpu)
    x = twin.rhs(n, seed=0xC0FFEE)
    d32 = d.astype(np.float32).astype(np.float64)
    assert np.array_equal(A @ x, coracle.spmv(ip, ix, d32, x))
    with pytest.raises(TypeError):
        vk.csr_matrix((td, tix, tip.to("cpu")), shape=(n, n), ctx=gpu)


def test_retired_tuning_env_warns():
    """A VTK_<KEY> variable of a tuning switch removed in round 5 (vtk_api.cpp RETIRED_KEYS) is not
    silently ignored: context creation names every such variable on stderr once; the switch is
    gone from the key table (vtk_ctx_set_tuning -> VTK_ERR_ARG)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path[:0] = [%r, %r]\n"
            "import vtkrylov as vk\n"
            "c = vk.Context(0)\n"
            "print(vk._abi.lib().vtk_ctx_set_tuning(c._h, b'g4_pd', 2))\n") % (
        root, os.path.join(root, "vt-precondition_amd"))
    env = dict(os.environ, VTK_G4_PD="2", VTK_UPD_XB="8")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "VTK_G4_PD is set but no longer has an effect" in r.stderr
    assert "VTK_UPD_XB is set but no longer has an effect" in r.stderr
    import vtkrylov as vk
    assert int(r.stdout.strip().splitlines()[-1]) == vk._abi.ERR_ARG
