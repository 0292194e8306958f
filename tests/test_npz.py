"""SciPy save_npz / load_npz CSR archives: vtkrylov.npz reads what SciPy
1.15.3 writes, entry for entry in stored order, and writes what SciPy reads.  Non-canonical
files (unsorted columns, duplicate entries, empty rows) stay as stored, because the device SpMV
sums each row in stored order like csr_matvec; the block-Jacobi blocks add duplicates up like
csr_matrix.toarray()."""
import io

import numpy as np
import pytest
import scipy.sparse as sp

from vtkrylov import npz  # pure Python: no HIP library needed
from oracle import coracle, twin


def messy_csr(n=300, seed=7, fp32=False, idx64=False, empty_rows=True):
    """Random CSR with unsorted columns, duplicates, empty rows and one long row."""
    rng = np.random.default_rng(seed)
    rows, cols, vals = [], [], []
    for r in range(n):
        if empty_rows and r % 17 == 5:
            continue                                   # empty row
        k = 40 if r == 11 else rng.integers(1, 7)
        c = rng.integers(max(0, r - 12), min(n, r + 12), size=k)
        c = np.concatenate([c, [r, r]])                # duplicate diagonal entries
        rng.shuffle(c)
        rows += [r] * len(c)
        cols += list(c)
        vals += list(rng.standard_normal(len(c)) + np.where(c == r, 4.0, 0.0))
    ip = np.zeros(n + 1, np.int64)
    np.add.at(ip, np.asarray(rows) + 1, 1)
    ip = np.cumsum(ip)
    dt = np.float32 if fp32 else np.float64
    A = sp.csr_matrix((np.asarray(vals, dt), np.asarray(cols, np.int64 if idx64 else np.int32),
                       ip.astype(np.int64 if idx64 else np.int32)), shape=(n, n))
    assert not A.has_canonical_format
    return A


@pytest.mark.parametrize("compressed", [True, False])
@pytest.mark.parametrize("fp32,idx64", [(False, False), (True, False), (False, True)])
def test_reads_scipy_archives(tmp_path, compressed, fp32, idx64):
    A = messy_csr(fp32=fp32, idx64=idx64)
    f = tmp_path / "a.npz"
    sp.save_npz(f, A, compressed=compressed)
    ip, ix, d, shape = npz.load_npz_arrays(f)
    assert shape == A.shape and ip.dtype == np.int32 and ix.dtype == np.int32
    assert d.dtype == (np.float32 if fp32 else np.float64)
    assert np.array_equal(ip, A.indptr) and np.array_equal(ix, A.indices)
    assert np.array_equal(d, A.data)
    # row blocks: rebased indptr, global columns, the stored slice
    for r0, r1 in [(0, 1), (5, 6), (11, 12), (37, 222), (299, 300), (300, 300)]:
        bp, bx, bd, _ = npz.load_npz_arrays(f, rows=(r0, r1))
        k0, k1 = A.indptr[r0], A.indptr[r1]
        assert np.array_equal(bp, A.indptr[r0:r1 + 1] - k0)
        assert np.array_equal(bx, A.indices[k0:k1]) and np.array_equal(bd, A.data[k0:k1])


def test_sparse_array_archive(tmp_path):
    A = sp.csr_array(messy_csr())            # writes the extra _is_array member
    f = tmp_path / "b.npz"
    sp.save_npz(f, A)
    ip, ix, d, _ = npz.load_npz_arrays(f)
    assert np.array_equal(d, A.data) and np.array_equal(ix, A.indices)


@pytest.mark.parametrize("compressed", [True, False])
def test_scipy_reads_our_archives(tmp_path, compressed, golden):
    ip, ix, d = golden["ragged/indptr"], golden["ragged/indices"], golden["ragged/data"]
    f = tmp_path / "ragged.npz"
    npz.save_npz_arrays(f, ip, ix, d, (ip.size - 1, ip.size - 1), compressed=compressed)
    B = sp.load_npz(f)
    assert B.format == "csr" and B.shape == (ip.size - 1, ip.size - 1)
    assert np.array_equal(B.indptr, ip) and np.array_equal(B.indices, ix) and np.array_equal(B.data, d)
    # same archive members as scipy.sparse.save_npz
    g = tmp_path / "ref.npz"
    sp.save_npz(g, sp.csr_matrix((d, ix, ip)), compressed=compressed)
    with np.load(f) as a, np.load(g) as b:
        assert sorted(a.files) == sorted(b.files)
        for k in a.files:
            assert np.array_equal(a[k], b[k]), k


def test_rejects(tmp_path):
    A = messy_csr()
    f = tmp_path / "csc.npz"
    sp.save_npz(f, A.tocsc())
    with pytest.raises(NotImplementedError):
        npz.load_npz_arrays(f)
    g = tmp_path / "obj.npz"
    np.savez(g, indices=np.array([object()], dtype=object), indptr=np.array([0, 1]),
             format=np.array(b"csr"), shape=np.array([1, 1]), data=np.array([1.0]))
    with pytest.raises(ValueError):
        npz.load_npz_arrays(g)
    h = tmp_path / "bad.npz"
    np.savez(h, indices=np.array([5], np.int32), indptr=np.array([0, 1], np.int32),
             format=np.array(b"csr"), shape=np.array([1, 1]), data=np.array([1.0]))
    with pytest.raises(ValueError):
        npz.load_npz_arrays(h)
    with pytest.raises(ValueError):
        npz.load_npz_arrays(io.BytesIO(b"not a zip"))


def test_bj_blocks_sum_duplicates_like_toarray():
    A = messy_csr(empty_rows=False)
    n, bs = A.shape[0], 8
    B = twin.bj_blocks(A.indptr, A.indices, A.data, n, bs)
    D = A.toarray()
    for b in range((n + bs - 1) // bs):
        r0, r1 = b * bs, min(n, b * bs + bs)
        assert np.array_equal(B[b, :r1 - r0, :r1 - r0], D[r0:r1, r0:r1])
    # C oracle Gauss-Jordan of the same blocks ~ LAPACK inverse
    inv = coracle.bj_setup(A.indptr, A.indices, A.data, bs)
    np.testing.assert_allclose(inv, np.linalg.inv(B).reshape(inv.shape), rtol=1e-10, atol=1e-12)


def test_c_spmv_of_loaded_archive_equals_scipy(tmp_path):
    A = messy_csr()
    f = tmp_path / "m.npz"
    sp.save_npz(f, A)
    ip, ix, d, _ = npz.load_npz_arrays(f)
    x = twin.rhs(A.shape[0], seed=0xC0FFEE)
    assert np.array_equal(coracle.spmv(ip, ix, d, x), A @ x)   # stored-order sums, bit for bit
