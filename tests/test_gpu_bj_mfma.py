"""Block-Jacobi setup on the matrix cores (vtk_bjacobi_create_ex(..., VTK_BJ_SETUP_MFMA); DESIGN.md
§3c): blocked Gauss-Jordan whose rank-4 panel updates run on v_mfma_f64_16x16x4f64, bs 16 / 32.

It is a tolerance mode: the pivots follow the scalar kernel's rule (first row of largest |a|)
but the rank-4 sums round differently from its rank-1 sequence, so the bar is the inverse within
1e-12 of the oracle's Gauss-Jordan inverse (coracle.bj_setup) and of numpy.linalg.inv, relative
to the block's largest inverse entry; GMRES with it keeps the solver bars (info, +-1 iteration,
x within 1e-9).  Singular blocks raise LinAlgError as in the exact setup.
"""
import time

import numpy as np
import pytest

from oracle import coracle, twin

pytestmark = pytest.mark.gpu


def _blocks_close(got, ref, bs, tol=1e-12):
    g = got.reshape(-1, bs, bs)
    r = ref.reshape(-1, bs, bs)
    scale = np.abs(r).max(axis=(1, 2), keepdims=True)
    err = np.abs(g - r) / scale
    assert err.max() <= tol, err.max()


def _np_inv_blocks(ip, ix, d, n, bs):
    import scipy.sparse as sp
    A = sp.csr_matrix((d, ix, ip), shape=(n, n)).toarray()
    nb = (n + bs - 1) // bs
    out = np.zeros((nb, bs, bs))
    for b in range(nb):
        r0, r1 = b * bs, min(n, b * bs + bs)
        blk = np.eye(bs)
        blk[:r1 - r0, :r1 - r0] = A[r0:r1, r0:r1]
        out[b] = np.linalg.inv(blk)
    return out


@pytest.mark.parametrize("bs", [16, 32])
@pytest.mark.parametrize("name", ["S2", "S4", "C0"])
def test_mfma_setup_vlasov(vk_lib, gpu, name, bs):
    p = twin.CONFIGS[name]
    A = vk_lib.vlasov_operator(vk_lib.vlasov_params(p.dim, p.shape, fp32=p.fp32), ctx=gpu)
    ip, ix, d = A.download()
    M = vk_lib.block_jacobi(A, bs, setup="mfma")
    inv = coracle.bj_setup(ip, ix, d, bs)
    _blocks_close(M.inverse(), inv, bs)
    if p.n <= 4096:
        _blocks_close(M.inverse(), _np_inv_blocks(ip, ix, d, p.n, bs), bs)
    M.close()
    A.close()


@pytest.mark.parametrize("bs", [16, 32])
def test_mfma_setup_ragged_random(vk_lib, gpu, golden, bs):
    ip, ix, d = golden["ragged/indptr"], golden["ragged/indices"], golden["ragged/data"]
    n = ip.shape[0] - 1
    A = vk_lib.csr_matrix((d, ix, ip), shape=(n, n), ctx=gpu)
    M = vk_lib.block_jacobi(A, bs, setup="mfma")
    assert M.mode == "inverse"
    _blocks_close(M.inverse(), coracle.bj_setup(ip, ix, d, bs), bs)
    M.close()
    A.close()


@pytest.mark.parametrize("bs", [16, 32])
def test_mfma_setup_pivoting(vk_lib, gpu, bs):
    """Dense random blocks with a zero diagonal (every column needs a row swap) and a padded
    last block: pivoting and padding against numpy.linalg.inv."""
    import scipy.sparse as sp
    rng = np.random.default_rng(7 + bs)
    n = 5 * bs + bs // 2
    dense = np.zeros((n, n))
    for b in range(0, n, bs):
        r1 = min(n, b + bs)
        blk = rng.standard_normal((r1 - b, r1 - b))
        np.fill_diagonal(blk, 0.0)
        dense[b:r1, b:r1] = blk
    dense[0, n - 1] = 3.0          # an off-block entry: ignored by the setup
    S = sp.csr_matrix(dense)
    A = vk_lib.csr_matrix(S, ctx=gpu)
    M = vk_lib.block_jacobi(A, bs, setup="mfma")
    ref = _np_inv_blocks(S.indptr, S.indices, S.data, n, bs)
    _blocks_close(M.inverse(), ref, bs, tol=1e-11)
    _blocks_close(M.inverse(), coracle.bj_setup(S.indptr.astype(np.int32), S.indices.astype(np.int32), S.data, bs),
                  bs, tol=1e-11)
    M.close()
    A.close()


def test_mfma_setup_singular_and_bad_bs(vk_lib, gpu):
    import scipy.sparse as sp
    n = 32
    dense = np.eye(n)
    dense[20, 20] = 0.0
    dense[20, 21] = 0.0
    A = vk_lib.csr_matrix(sp.csr_matrix(dense), ctx=gpu)
    with pytest.raises(np.linalg.LinAlgError):
        vk_lib.block_jacobi(A, 16, setup="mfma")
    with pytest.raises(ValueError):
        vk_lib.block_jacobi(A, 8, setup="mfma")
    A.close()


@pytest.mark.parametrize("bs", [16, 32])
def test_mfma_setup_gmres(vk_lib, gpu, bs):
    p = twin.CONFIGS["C1"]
    A = vk_lib.vlasov_operator(vk_lib.vlasov_params(p.dim, p.shape), ctx=gpu)
    ip, ix, d = A.download()
    b = coracle.rhs(p.n)
    M = vk_lib.block_jacobi(A, bs, setup="mfma")
    x, info = vk_lib.gmres(A, b, rtol=1e-8, M=M)
    st = vk_lib.last_stats()
    ref = coracle.gmres(ip, ix, d, b, coracle.bj_setup(ip, ix, d, bs), rtol=1e-8)
    assert info == ref.info == 0
    assert abs(st.inner_iters - ref.inner_iters) <= 1
    assert np.linalg.norm(x - ref.x) / np.linalg.norm(ref.x) < 1e-9
    M.close()
    A.close()


@pytest.mark.parametrize("bs", [16, 32])
def test_mfma_setup_time_c3(vk_lib, gpu, bs):
    """Setup kernel time of both paths on the 20M-row operator (HIP-event profile; printed)."""
    p = twin.CONFIGS["C3"]
    A = vk_lib.vlasov_operator(vk_lib.vlasov_params(p.dim, p.shape), ctx=gpu)
    gpu.profile(True)
    for setup in ("exact", "mfma", "exact", "mfma"):
        vk_lib.block_jacobi(A, bs, setup=setup).close()
    prof = gpu.profile_read()
    gpu.profile(False)
    ex, mf = prof["bj_setup"]["avg_us"], prof["bj_setup_mfma"]["avg_us"]
    print(f"\nC3 BJ({bs}) setup kernel: exact {ex / 1e3:.2f} ms, mfma {mf / 1e3:.2f} ms")
    A.close()
