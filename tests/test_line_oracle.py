"""Line-Jacobi preconditioner — the oracle pinned before it is trusted:
the C restatement (oracle/vtk_oracle.c orc_line_setup/orc_line_apply/orc_gmres_line) against
the NumPy twin bit for bit, and against SciPy golden vectors (tests/golden/golden_line.npz:
splu solves with M, SciPy GMRES with that LinearOperator).  CPU only."""
import numpy as np
import pytest

from oracle import coracle, twin

SMALL = ["C0", "S2", "S4", "S4F"]
SEG = 25


def stride_of(p):
    return 1 if p.dim == 1 else (p.shape[1] if p.dim == 2 else p.n // p.shape[0])


def bits(a):
    return np.ascontiguousarray(a).view(np.uint64)


@pytest.mark.parametrize("name", SMALL + ["C1"])
@pytest.mark.parametrize("seg", [1, 3, SEG, 1 << 30])
def test_c_line_equals_twin(name, seg):
    p = twin.CONFIGS[name]
    ip, ix, d = coracle.generate(p)
    st = stride_of(p)
    lf = coracle.line_setup(ip, ix, d, st, seg)
    f = twin.line_factors_numpy(ip, ix, d, p.n, st, seg)
    assert np.array_equal(bits(lf.f), bits(f))
    r = twin.rhs(p.n)
    assert np.array_equal(bits(coracle.line_apply(lf, r)), bits(twin.line_apply_numpy(f, r, st, seg)))


@pytest.mark.parametrize("name", ["S2", "S4F", "C1"])
def test_c_line_row_blocks(name):
    """A rank's row block: lines are cut at the block edges (row0 aligned to whole x-columns,
    and also not aligned)."""
    p = twin.CONFIGS[name]
    st = stride_of(p)
    for r0, r1 in [((p.n // 4) // st * st, (3 * p.n // 4) // st * st), (st // 2 + 3, p.n - st - 5)]:
        ip, ix, d = coracle.generate(p, r0, r1)
        lf = coracle.line_setup(ip, ix, d, st, SEG, row0=r0)
        f = twin.line_factors_numpy(ip, ix, d, r1 - r0, st, SEG, row0=r0)
        assert np.array_equal(bits(lf.f), bits(f))
        r = twin.rhs(p.n, r0=r0, r1=r1)
        z = coracle.line_apply(lf, r)
        assert np.array_equal(bits(z), bits(twin.line_apply_numpy(f, r, st, SEG, row0=r0)))
        # the block's M (global columns shifted to the block) solved by SciPy
        from scipy.sparse.linalg import spsolve
        M = twin.line_matrix(ip, ix, d, r1 - r0, st, SEG, row0=r0)
        np.testing.assert_allclose(z, spsolve(M.tocsc(), r), rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("name", SMALL)
@pytest.mark.parametrize("seg", [3, SEG])
def test_c_line_apply_vs_scipy_splu(name, seg, golden_line):
    p = twin.CONFIGS[name]
    ip, ix, d = coracle.generate(p)
    z = coracle.line_apply(coracle.line_setup(ip, ix, d, stride_of(p), seg), twin.rhs(p.n))
    np.testing.assert_allclose(z, golden_line[f"{name}/line{seg}_z"], rtol=1e-12, atol=1e-14)


def test_c_line_ragged_vs_scipy(golden, golden_line):
    ip, ix, d = golden["ragged/indptr"], golden["ragged/indices"], golden["ragged/data"]
    n = ip.shape[0] - 1
    z = coracle.line_apply(coracle.line_setup(ip, ix, d, 37, 5), twin.rhs(n))
    np.testing.assert_allclose(z, golden_line["ragged/line37_5_z"], rtol=1e-12, atol=1e-14)


def test_c_line_duplicates_add_up():
    """Non-canonical rows (duplicate and unsorted entries): sums as toarray() does."""
    import scipy.sparse as sp
    p = twin.CONFIGS["S2"]
    ip, ix, d = coracle.generate(p)
    rows = np.repeat(np.arange(p.n), np.diff(ip))
    rng = np.random.default_rng(5)
    dup = rng.choice(rows.shape[0], 400, replace=False)
    R = np.concatenate([rows, rows[dup]])
    Cc = np.concatenate([ix, ix[dup]])
    V = np.concatenate([d * 0.75, d[dup] * 0.25])
    perm = np.lexsort((rng.random(R.shape[0]), R))        # row-major, columns shuffled
    R, Cc, V = R[perm], Cc[perm], V[perm]
    ip2 = np.concatenate([[0], np.cumsum(np.bincount(R, minlength=p.n))]).astype(np.int32)
    st = stride_of(p)
    z = coracle.line_apply(coracle.line_setup(ip2, Cc.astype(np.int32), V, st, SEG), twin.rhs(p.n))
    A = sp.csr_matrix((V, Cc, ip2), shape=(p.n, p.n))
    M = twin.line_matrix(A.indptr, A.indices, A.data, p.n, st, SEG)
    from scipy.sparse.linalg import spsolve
    np.testing.assert_allclose(z, spsolve(M.tocsc(), twin.rhs(p.n)), rtol=1e-12, atol=1e-14)


def test_c_line_zero_pivot_raises():
    ip = np.array([0, 1, 2], np.int32)
    ix = np.array([0, 1], np.int32)
    d = np.array([1.0, 0.0])
    with pytest.raises(np.linalg.LinAlgError):
        coracle.line_setup(ip, ix, d, 1, 2)


@pytest.mark.parametrize("name", SMALL)
def test_c_gmres_line_vs_scipy(name, golden_line):
    p = twin.CONFIGS[name]
    ip, ix, d = coracle.generate(p)
    b = twin.rhs(p.n)
    s = coracle.gmres(ip, ix, d, b, coracle.line_setup(ip, ix, d, stride_of(p), SEG), rtol=1e-8)
    info, iters, res, bn = golden_line[f"{name}/gmres_line_meta"]
    assert s.info == int(info)
    assert abs(s.inner_iters - int(iters)) <= 1
    gx = golden_line[f"{name}/gmres_line_x"]
    assert np.linalg.norm(s.x - gx) / np.linalg.norm(gx) < 1e-9


def test_c_gmres_line_c1_vs_scipy_summary(golden_large):
    p = twin.CONFIGS["C1"]
    ip, ix, d = coracle.generate(p)
    g = golden_large["C1"][f"gmres_line{SEG}"]
    s = coracle.gmres(ip, ix, d, twin.rhs(p.n), coracle.line_setup(ip, ix, d, g["stride"], g["seg"]), rtol=1e-8)
    assert s.info == g["info"] and abs(s.inner_iters - g["inner_iters"]) <= 1
    assert np.linalg.norm(s.x) == pytest.approx(g["x_norm2"], rel=1e-9)
    np.testing.assert_allclose(s.x[:8], g["x_first8"], rtol=1e-8)
