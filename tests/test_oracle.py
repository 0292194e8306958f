"""The oracle is pinned before it is trusted: the NumPy twin and the C restatement against each
other and against the SciPy golden vectors committed in tests/golden (make_golden.py).
CPU only."""
import numpy as np
import pytest

from oracle import coracle, twin

SMALL = ["C0", "S2", "S4", "S4F"]


@pytest.mark.parametrize("name", SMALL)
def test_twin_equals_c_generator(name):
    p = twin.CONFIGS[name]
    a = twin.generate(p)
    b = coracle.generate(p)
    for x, y in zip(a, b):
        assert x.dtype == y.dtype
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8))
    assert a[0][-1] == p.nnz


@pytest.mark.parametrize("name", SMALL)
def test_twin_is_canonical_scipy_csr(name):
    import scipy.sparse as sp
    p = twin.CONFIGS[name]
    ip, ix, d = twin.generate(p)
    rows = np.repeat(np.arange(p.n), np.diff(ip))
    A = sp.csr_matrix((d, (rows, ix)), shape=(p.n, p.n))
    A.sum_duplicates()
    A.sort_indices()
    assert np.array_equal(A.indptr, ip) and np.array_equal(A.indices, ix) and np.array_equal(A.data, d)


@pytest.mark.parametrize("name", ["C1", "C2"])
def test_twin_hash_matches_golden(name, golden_large):
    h = twin.csr_sha256(twin.CONFIGS[name])
    ref = golden_large[name]["sha256"]
    assert h["nnz"] == ref["nnz"]
    assert (h["indptr"], h["indices"], h["data"]) == (ref["indptr"], ref["indices"], ref["data"])


def test_rhs_twin_equals_c():
    assert np.array_equal(twin.rhs(100_000), coracle.rhs(100_000))
    assert np.array_equal(twin.rhs(1000, r0=500, r1=900), coracle.rhs(1000, r0=500, r1=900))
    b = twin.rhs(100_000)
    assert b.min() >= -1.0 and b.max() < 1.0


def test_lartg_matches_scipy_lapack():
    from scipy.linalg import get_lapack_funcs
    lartg = get_lapack_funcs("lartg", dtype=np.float64)
    rng = np.random.default_rng(0)
    cases = [(0.0, 0.0), (0.0, -2.0), (3.0, 0.0), (1e-310, 1e-300), (1e300, -1e300), (-4.0, 3.0)]
    for i in range(3000):
        f, g = rng.standard_normal(2) * 10.0 ** rng.integers(-300, 300, 2)
        cases.append((float(f), float(g)))
    for f, g in cases:
        assert tuple(lartg(f, g)) == coracle.lartg(f, g), (f, g)


@pytest.mark.parametrize("name", SMALL)
def test_c_spmv_bitexact_vs_scipy(name, golden):
    p = twin.CONFIGS[name]
    ip, ix, d = coracle.generate(p)
    x = twin.rhs(p.n, seed=0xC0FFEE)
    assert np.array_equal(coracle.spmv(ip, ix, d, x), golden[f"{name}/spmv_y"])
    assert np.array_equal(coracle.spmv(ip, ix, d, np.ones(p.n)), golden[f"{name}/ones_y"])


@pytest.mark.parametrize("name", SMALL)
def test_c_bj_vs_numpy_inv(name, golden):
    p = twin.CONFIGS[name]
    ip, ix, d = coracle.generate(p)
    inv = coracle.bj_setup(ip, ix, d, 8)
    if f"{name}/bj8_inv" in golden:
        np.testing.assert_allclose(inv, golden[f"{name}/bj8_inv"], rtol=1e-12, atol=1e-14)
    z = coracle.bj_apply(inv, twin.rhs(p.n))
    np.testing.assert_allclose(z, golden[f"{name}/bj8_z"], rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("name", SMALL)
def test_c_gmres_vs_scipy(name, golden):
    p = twin.CONFIGS[name]
    ip, ix, d = coracle.generate(p)
    b = twin.rhs(p.n)
    s = coracle.gmres(ip, ix, d, b, coracle.bj_setup(ip, ix, d, 8), rtol=1e-8)
    info, iters, res, bn = golden[f"{name}/gmres_meta"]
    assert s.info == int(info)
    assert s.inner_iters == int(iters)
    gx = golden[f"{name}/gmres_x"]
    assert np.linalg.norm(s.x - gx) / np.linalg.norm(gx) < 1e-10


@pytest.mark.parametrize("case", ["noprec", "x0", "restart5_maxiter3", "bzero", "atol", "restart40"])
def test_c_gmres_edge_cases_vs_scipy(case, golden):
    p = twin.CONFIGS["S2"]
    ip, ix, d = coracle.generate(p)
    b = np.zeros(p.n) if case == "bzero" else twin.rhs(p.n)
    inv = None if case == "noprec" else coracle.bj_setup(ip, ix, d, 8)
    kw = {"noprec": dict(rtol=1e-8), "x0": dict(x0=golden["edge/x0/x0"], rtol=1e-10),
          "restart5_maxiter3": dict(rtol=1e-12, restart=5, maxiter=3), "bzero": dict(rtol=1e-8),
          "atol": dict(rtol=0.0, atol=1e-3), "restart40": dict(rtol=1e-9, restart=40)}[case]
    s = coracle.gmres(ip, ix, d, b, inv, **kw)
    info, iters, res, bn = golden[f"edge/{case}/meta"]
    assert s.info == int(info)
    assert s.inner_iters == int(iters)
    gx = golden[f"edge/{case}/x"]
    if case == "bzero":
        assert np.all(s.x == 0)
    else:
        assert np.linalg.norm(s.x - gx) / np.linalg.norm(gx) < 1e-9


def test_c_ragged_csr_vs_scipy(golden):
    ip, ix, d = golden["ragged/indptr"], golden["ragged/indices"], golden["ragged/data"]
    n = ip.shape[0] - 1
    assert np.array_equal(coracle.spmv(ip, ix, d, twin.rhs(n, seed=0xC0FFEE)), golden["ragged/spmv_y"])
    for bs in (4, 7):
        z = coracle.bj_apply(coracle.bj_setup(ip, ix, d, bs), twin.rhs(n))
        np.testing.assert_allclose(z, golden[f"ragged/bj{bs}_z"], rtol=1e-12, atol=1e-14)
    s = coracle.gmres(ip, ix, d, twin.rhs(n), coracle.bj_setup(ip, ix, d, 4), rtol=1e-10)
    info, iters, res, bn = golden["ragged/gmres_meta"]
    assert s.info == int(info) and abs(s.inner_iters - int(iters)) <= 1
    gx = golden["ragged/gmres_x"]
    assert np.linalg.norm(s.x - gx) / np.linalg.norm(gx) < 1e-9


def test_c_gmres_c1_vs_scipy_summary(golden_large):
    p = twin.CONFIGS["C1"]
    ip, ix, d = coracle.generate(p)
    b = twin.rhs(p.n)
    s = coracle.gmres(ip, ix, d, b, coracle.bj_setup(ip, ix, d, 8), rtol=1e-8)
    g = golden_large["C1"]["gmres_bj8"]
    assert s.info == g["info"] and s.inner_iters == g["inner_iters"]
    assert np.linalg.norm(s.x) == pytest.approx(g["x_norm2"], rel=1e-12)
    np.testing.assert_allclose(s.x[:8], g["x_first8"], rtol=1e-10)
