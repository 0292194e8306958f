"""Device operators from SciPy .npz archives.  A non-canonical archive
(unsorted columns, duplicates, empty rows) loads in stored order: SpMV bit-identical to
SciPy's csr_matvec on the same file, BJ inverse bit-identical to the oracle (duplicates summed,
as toarray()), GMRES within the parity bars of tests/test_gpu_parity.py."""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import coracle, twin
from test_npz import messy_csr

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("compressed", [True, False])
def test_messy_archive_spmv_bitexact(gpu, vk_lib, tmp_path, compressed):
    A = messy_csr(n=5000, seed=3)
    f = tmp_path / "m.npz"
    sp.save_npz(f, A, compressed=compressed)
    D = vk_lib.load_npz(f, ctx=gpu)
    x = twin.rhs(A.shape[0], seed=0xC0FFEE)
    assert np.array_equal(D @ x, A @ x)
    D.set_layout("sell" if D.layout == "csr" else "csr")   # the other layout, same bits
    assert np.array_equal(D @ x, A @ x)
    ip, ix, d = D.download()
    assert np.array_equal(ip, A.indptr) and np.array_equal(ix, A.indices) and np.array_equal(d, A.data)


@pytest.mark.parametrize("orth", ["mgs", "dcgs2"])
def test_messy_archive_bj_gmres(gpu, vk_lib, tmp_path, orth):
    A = messy_csr(n=5000, seed=4, empty_rows=False)
    f = tmp_path / "m.npz"
    sp.save_npz(f, A)
    D = vk_lib.load_npz(f, ctx=gpu)
    M = vk_lib.block_jacobi(D, 8)
    inv_ref = coracle.bj_setup(A.indptr, A.indices, A.data, 8)
    assert np.array_equal(M.inverse(), inv_ref)
    b = twin.rhs(A.shape[0])
    ref = coracle.gmres(A.indptr, A.indices, A.data, b, inv_ref, rtol=1e-8)
    x, info = vk_lib.gmres(D, b, rtol=1e-8, M=M, orth=orth)
    st = vk_lib.last_stats()
    assert info == ref.info == 0
    assert abs(st.inner_iters - ref.inner_iters) <= 1
    assert np.linalg.norm(x - ref.x) / np.linalg.norm(ref.x) <= 1e-9


def test_save_load_roundtrip_c1(gpu, vk_lib, tmp_path):
    p = twin.CONFIGS["C1"]
    A = vk_lib.vlasov_operator(vk_lib.vlasov_params(p.dim, p.shape, fp32=p.fp32), ctx=gpu)
    f = tmp_path / "c1.npz"
    vk_lib.save_npz(f, A)
    B = sp.load_npz(f)                          # SciPy reads what the device saved
    ip, ix, d = coracle.generate(p)
    assert np.array_equal(B.indptr, ip) and np.array_equal(B.indices, ix) and np.array_equal(B.data, d)
    A2 = vk_lib.load_npz(f, ctx=gpu)
    x = twin.rhs(p.n, seed=0xC0FFEE)
    assert np.array_equal(A2 @ x, A @ x)
