"""GPU parity tests: the HIP path (through the C-ABI) against the CPU oracle and the committed
SciPy golden vectors.  Bars:
  * operator assembly, SpMV (stream tiles), BJ setup and BJ apply: bit-identical to the C
    oracle (same IEEE op sequence, -ffp-contract=off on both sides);
  * rows longer than TILE_NNZ (work-group reduction): relative 1e-13 per row;
  * GMRES: same info, inner iterations within +-1, ||x - x_ref|| / ||x_ref|| <= 1e-9 against
    the oracle / SciPy at small sizes; at full sizes the true residual ||b - A x|| <= atol
    (recomputed on the host by the oracle SpMV) and hash-level checks of the operator.
"""
import hashlib

import numpy as np
import pytest

from oracle import coracle, twin

pytestmark = pytest.mark.gpu

SMALL = ["C0", "S2", "S4", "S4F"]


def _vk_params(vk, p):
    return vk.vlasov_params(p.dim, p.shape, fp32=p.fp32)


@pytest.fixture(scope="module")
def ops(gpu, vk_lib):
    vk = vk_lib
    out = {}
    for name in SMALL + ["C1"]:
        p = twin.CONFIGS[name]
        out[name] = (p, vk.vlasov_operator(_vk_params(vk, p), ctx=gpu), coracle.generate(p))
    return out


@pytest.mark.parametrize("name", SMALL + ["C1"])
def test_device_generator_bitexact(ops, name):
    p, A, (ip, ix, d) = ops[name]
    gip, gix, gd = A.download()
    assert gd.dtype == d.dtype
    assert np.array_equal(gip, ip)
    assert np.array_equal(gix, ix)
    assert np.array_equal(gd.view(np.uint8), d.view(np.uint8))


@pytest.mark.parametrize("name", ["C1", "C2", "C3"])
def test_device_generator_hash(gpu, vk_lib, golden_large, name):
    vk = vk_lib
    p = twin.CONFIGS[name]
    A = vk.vlasov_operator(_vk_params(vk, p), ctx=gpu)
    ip, ix, d = A.download()
    A.close()
    ref = golden_large[name]["sha256"]
    assert int(ip[-1]) == ref["nnz"] == p.nnz
    assert hashlib.sha256(ip.tobytes()).hexdigest() == ref["indptr"]
    assert hashlib.sha256(ix.tobytes()).hexdigest() == ref["indices"]
    assert hashlib.sha256(d.tobytes()).hexdigest() == ref["data"]


@pytest.mark.slow
def test_device_generator_hash_c4(gpu, vk_lib, golden_large):
    if "C4" not in golden_large:
        pytest.skip("C4 hash not in golden_large.json")
    vk = vk_lib
    p = twin.CONFIGS["C4"]
    A = vk.vlasov_operator(_vk_params(vk, p), ctx=gpu)
    ip, ix, d = A.download()
    A.close()
    ref = golden_large["C4"]["sha256"]
    assert d.dtype == np.float32
    assert hashlib.sha256(ip.tobytes()).hexdigest() == ref["indptr"]
    assert hashlib.sha256(ix.tobytes()).hexdigest() == ref["indices"]
    assert hashlib.sha256(d.tobytes()).hexdigest() == ref["data"]


@pytest.mark.parametrize("layout", ["sell", "sell32", "csr"])
@pytest.mark.parametrize("name", SMALL + ["C1"])
def test_spmv_bitexact(ops, golden, name, layout):
    p, A, (ip, ix, d) = ops[name]
    assert A.layout == "sell"           # auto: the Vlasov operators pad < 25 %
    A.set_layout(layout)
    try:
        assert A.layout == layout
        x = twin.rhs(p.n, seed=0xC0FFEE)
        y = A @ x
        assert np.array_equal(y, coracle.spmv(ip, ix, d, x))
        if f"{name}/spmv_y" in golden:      # SciPy csr_matvec
            assert np.array_equal(y, golden[f"{name}/spmv_y"])
            assert np.array_equal(A @ np.ones(p.n), golden[f"{name}/ones_y"])
    finally:
        A.set_layout("auto")


def test_spmv_c1_golden_hash(ops, golden_large):
    p, A, _ = ops["C1"]
    y = A @ twin.rhs(p.n, seed=0xC0FFEE)
    assert hashlib.sha256(y.tobytes()).hexdigest() == golden_large["C1"]["spmv_y_sha256"]
    assert np.linalg.norm(A @ np.ones(p.n)) == pytest.approx(golden_large["C1"]["A_ones_norm2"], rel=1e-15)


def test_spmv_ragged_sell_forced_bitexact(gpu, vk_lib, golden):
    """SELL sums every row in one lane, long rows included: bit-identical everywhere."""
    vk = vk_lib
    ip, ix, d = golden["ragged/indptr"], golden["ragged/indices"], golden["ragged/data"]
    n = ip.shape[0] - 1
    A = vk.csr_matrix((d, ix, ip), shape=(n, n), ctx=gpu)
    assert A.layout == "csr"            # auto: padding too large for SELL
    x = twin.rhs(n, seed=0xC0FFEE)
    for lay in ("sell", "sell32"):
        A.set_layout(lay)
        assert A.layout == lay
        assert np.array_equal(A @ x, coracle.spmv(ip, ix, d, x))
        assert np.array_equal(A @ x, golden["ragged/spmv_y"])
    A.set_layout("sell")
    assert A.layout_info()["wide_chunks"] > 0     # random columns: int32 chunks


def _dict_edge_csr():
    """Chunk 0: exactly 15 distinct col-row offsets (coded); chunk 1: 16 (int32, "wide");
    chunk 2: ragged rows over 3 offsets incl. empty rows and unsorted duplicates; chunk 3:
    empty; chunk 4: 40-entry rows (5 code words per lane) over 2 offsets."""
    n = 320
    rows, cols = [], []
    for r in range(64):
        for o in range(15):
            rows.append(r); cols.append(r + 3 * o)
    for r in range(64, 128):
        for o in range(16):
            rows.append(r); cols.append(r + 2 * o - 10)
    rng = np.random.default_rng(7)
    for r in range(128, 192):
        for _ in range(int(rng.integers(0, 6))):
            rows.append(r); cols.append(r + int(rng.choice([-5, 0, 9])))
    for r in range(256, 320):
        for k in range(40):
            rows.append(r); cols.append(r - 1 if k % 2 else r - 200)
    rows, cols = np.array(rows), np.array(cols)
    vals = np.random.default_rng(8).standard_normal(rows.size)
    order = np.argsort(rows, kind="stable")
    rows, cols, vals = rows[order], cols[order], vals[order]
    ip = np.zeros(n + 1, np.int32)
    np.add.at(ip, rows + 1, 1)
    return n, np.cumsum(ip).astype(np.int32), cols.astype(np.int32), vals


def test_spmv_dictionary_chunks_bitexact(gpu, vk_lib):
    """SELL column dictionaries: the 15-offset limit, a wide chunk next to coded ones, ragged
    and empty rows, long rows spanning several code words -- bit-identical to csr_matvec."""
    vk = vk_lib
    n, ip, ix, d = _dict_edge_csr()
    A = vk.csr_matrix((d, ix, ip), shape=(n, n), ctx=gpu)
    x = twin.rhs(n, seed=0xC0FFEE)
    ref = coracle.spmv(ip, ix, d, x)
    for lay in ("sell", "sell32", "csr"):
        A.set_layout(lay)
        assert A.layout == lay
        assert np.array_equal(A @ x, ref), lay
    A.set_layout("sell")
    li = A.layout_info()
    assert li["sell_chunks"] == 5 and li["wide_chunks"] == 1


@pytest.mark.parametrize("layout", ["sell", "sell32", "csr"])
@pytest.mark.parametrize("bj_mode", ["tridiag", "inverse"])
def test_gmres_layouts_c1(ops, layout, bj_mode):
    p, A, (ip, ix, d) = ops["C1"]
    import vtkrylov as vk
    A.set_layout(layout)
    try:
        M = vk.block_jacobi(A, 8, mode=bj_mode)
        b = twin.rhs(p.n)
        inv = coracle.bj_setup(ip, ix, d, 8)
        ref = coracle.gmres(ip, ix, d, b, inv, rtol=1e-8)
        x, info = vk.gmres(A, b, rtol=1e-8, M=M)
        st = vk.last_stats()
        assert info == ref.info == 0
        assert abs(st.inner_iters - ref.inner_iters) <= 1
        assert np.linalg.norm(x - ref.x) / np.linalg.norm(ref.x) <= 1e-9
    finally:
        A.set_layout("auto")


def test_spmv_ragged_and_long_rows(gpu, vk_lib, golden):
    vk = vk_lib
    ip, ix, d = golden["ragged/indptr"], golden["ragged/indices"], golden["ragged/data"]
    n = ip.shape[0] - 1
    A = vk.csr_matrix((d, ix, ip), shape=(n, n), ctx=gpu)
    x = twin.rhs(n, seed=0xC0FFEE)
    y = A @ x
    assert np.array_equal(y, golden["ragged/spmv_y"])      # empty rows, 2500-nnz row
    # rows longer than TILE_NNZ (4096) take the work-group reduction path
    rng = np.random.default_rng(5)
    n2 = 20000
    lens = rng.integers(0, 6, n2)
    lens[[3, 9000, n2 - 1]] = [12000, 5000, 4097]
    rows = np.repeat(np.arange(n2), lens)
    cols = np.concatenate([np.sort(rng.choice(n2, l, replace=False)) for l in lens])
    vals = rng.standard_normal(rows.shape[0])
    ip2 = np.zeros(n2 + 1, np.int32)
    np.cumsum(lens, out=ip2[1:])
    B = vk.csr_matrix((vals, cols.astype(np.int32), ip2), shape=(n2, n2), ctx=gpu)
    x2 = rng.standard_normal(n2)
    y2 = B @ x2
    ref = coracle.spmv(ip2, cols.astype(np.int32), vals, x2)
    long_rows = lens > 4096
    assert np.array_equal(y2[~long_rows], ref[~long_rows])
    np.testing.assert_allclose(y2[long_rows], ref[long_rows], rtol=1e-13,
                               atol=1e-13 * np.abs(vals).max() * np.abs(x2).max())


@pytest.mark.parametrize("name", SMALL + ["C1"])
def test_bj_setup_and_apply_bitexact(ops, golden, name):
    p, A, (ip, ix, d) = ops[name]
    import vtkrylov as vk
    M = vk.block_jacobi(A, 8, mode="inverse")
    assert M.mode == "inverse"
    inv = coracle.bj_setup(ip, ix, d, 8)
    assert np.array_equal(M.inverse(), inv)
    b = twin.rhs(p.n)
    z = M @ b
    assert np.array_equal(z, coracle.bj_apply(inv, b))
    if f"{name}/bj8_z" in golden:     # numpy.linalg.inv + einsum
        np.testing.assert_allclose(z, golden[f"{name}/bj8_z"], rtol=1e-12, atol=1e-14)
    if f"{name}/bj8_inv" in golden:
        np.testing.assert_allclose(M.inverse(), golden[f"{name}/bj8_inv"], rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("name", SMALL + ["C1"])
@pytest.mark.parametrize("bs", [2, 4, 8])
def test_bj_tridiag_apply(ops, name, bs):
    """The Vlasov operators' diagonal blocks are tridiagonal (v-direction coupling): "auto"
    applies M^-1 with their LU factors; equal to the oracle's inverse apply to rounding."""
    p, A, (ip, ix, d) = ops[name]
    import vtkrylov as vk
    M = vk.block_jacobi(A, bs)
    assert M.tridiag_available and M.mode == "tridiag"
    inv = coracle.bj_setup(ip, ix, d, bs)
    assert np.array_equal(M.inverse(), inv)          # the inverse is still built (and exported)
    b = twin.rhs(p.n)
    ref = coracle.bj_apply(inv, b)
    z = M @ b
    np.testing.assert_allclose(z, ref, rtol=1e-12, atol=1e-14 * np.abs(ref).max())
    M.set_mode("inverse")
    assert M.mode == "inverse" and np.array_equal(M @ b, ref)


@pytest.mark.parametrize("bs", [4, 7, 16])
def test_bj_ragged_block_sizes(gpu, vk_lib, golden, bs):
    vk = vk_lib
    ip, ix, d = golden["ragged/indptr"], golden["ragged/indices"], golden["ragged/data"]
    n = ip.shape[0] - 1
    A = vk.csr_matrix((d, ix, ip), shape=(n, n), ctx=gpu)
    M = vk.block_jacobi(A, bs, setup="exact")        # the bit-exact setup (auto: MFMA at bs 16)
    assert M.mode == "inverse"                       # ragged blocks are not tridiagonal
    if bs in (2, 4, 8):
        with pytest.raises(ValueError):
            M.set_mode("tridiag")
    inv = coracle.bj_setup(ip, ix, d, bs)
    assert np.array_equal(M.inverse(), inv)
    b = twin.rhs(n)
    z = M @ b
    assert np.array_equal(z, coracle.bj_apply(inv, b))
    if f"ragged/bj{bs}_z" in golden:
        np.testing.assert_allclose(z, golden[f"ragged/bj{bs}_z"], rtol=1e-12, atol=1e-14)


def test_bj_singular_block_raises(gpu, vk_lib):
    vk = vk_lib
    n = 16
    ip = np.arange(n + 1, dtype=np.int32)
    ix = np.arange(n, dtype=np.int32)
    d = np.ones(n)
    d[5] = 0.0
    A = vk.csr_matrix((d, ix, ip), shape=(n, n), ctx=gpu)
    with pytest.raises(np.linalg.LinAlgError):
        vk.block_jacobi(A, 8)


@pytest.fixture(params=["mgs", "dcgs2"])
def orth(request, gpu, vk_lib):
    """Run a solver test with each orthogonalisation scheme; both must meet the same bars
    against SciPy's MGS (same info, inner iterations +-1, x within tolerance)."""
    gpu.set_orth({"mgs": vk_lib._abi.ORTH_MGS, "dcgs2": vk_lib._abi.ORTH_DCGS2}[request.param])
    yield request.param
    gpu.set_orth(vk_lib._abi.ORTH_AUTO)


def _check_solve(xg, info, st, ref_x, ref_info, ref_iters, tol=1e-9):
    assert info == ref_info
    assert abs(st.inner_iters - ref_iters) <= 1, (st.inner_iters, ref_iters)
    rel = np.linalg.norm(xg - ref_x) / max(np.linalg.norm(ref_x), 1e-300)
    assert rel <= tol, rel


@pytest.mark.parametrize("name", SMALL)
def test_gmres_vs_oracle_and_scipy(ops, golden, name, orth):
    import vtkrylov as vk
    p, A, (ip, ix, d) = ops[name]
    M = vk.block_jacobi(A, 8)
    b = twin.rhs(p.n)
    xg, info = vk.gmres(A, b, rtol=1e-8, M=M)
    st = vk.last_stats()
    ref = coracle.gmres(ip, ix, d, b, coracle.bj_setup(ip, ix, d, 8), rtol=1e-8)
    _check_solve(xg, info, st, ref.x, ref.info, ref.inner_iters)
    meta = golden[f"{name}/gmres_meta"]
    _check_solve(xg, info, st, golden[f"{name}/gmres_x"], int(meta[0]), int(meta[1]))
    res = np.linalg.norm(b - coracle.spmv(ip, ix, d, xg))
    assert res <= 1e-8 * np.linalg.norm(b)


@pytest.mark.parametrize("case", ["noprec", "x0", "restart5_maxiter3", "bzero", "atol", "restart40"])
def test_gmres_edge_cases(ops, golden, case, orth):
    import vtkrylov as vk
    p, A, (ip, ix, d) = ops["S2"]
    b = twin.rhs(p.n)
    M = vk.block_jacobi(A, 8)
    kw = {"noprec": dict(rtol=1e-8, M=None),
          "x0": dict(M=M, x0=golden["edge/x0/x0"], rtol=1e-10),
          "restart5_maxiter3": dict(M=M, rtol=1e-12, restart=5, maxiter=3),
          "bzero": dict(M=M, rtol=1e-8),
          "atol": dict(M=M, rtol=0.0, atol=1e-3),
          "restart40": dict(M=M, rtol=1e-9, restart=40)}[case]
    if case == "bzero":
        b = np.zeros(p.n)
    if orth == "dcgs2" and case == "restart40":   # DCGS2 is limited to restart <= 32: explicit
        with pytest.raises(ValueError):
            vk.gmres(A, b, **kw)
        return
    xg, info = vk.gmres(A, b, **kw)
    st = vk.last_stats()
    meta = golden[f"edge/{case}/meta"]
    gx = golden[f"edge/{case}/x"]
    if case == "bzero":
        assert info == 0 and np.all(xg == 0.0)
        return
    # info > 0 (not converged) solutions are compared at the same tolerance: same iterations
    _check_solve(xg, info, st, gx, int(meta[0]), int(meta[1]), tol=1e-8)


def test_gmres_ragged_generic_bs(gpu, vk_lib, golden, orth):
    vk = vk_lib
    ip, ix, d = golden["ragged/indptr"], golden["ragged/indices"], golden["ragged/data"]
    n = ip.shape[0] - 1
    A = vk.csr_matrix((d, ix, ip), shape=(n, n), ctx=gpu)
    M = vk.block_jacobi(A, 4)
    b = twin.rhs(n)
    xg, info = vk.gmres(A, b, rtol=1e-10, M=M)
    st = vk.last_stats()
    meta = golden["ragged/gmres_meta"]
    _check_solve(xg, info, st, golden["ragged/gmres_x"], int(meta[0]), int(meta[1]), tol=1e-8)


def test_gmres_c1_vs_scipy_summary(ops, golden_large, orth):
    import vtkrylov as vk
    p, A, (ip, ix, d) = ops["C1"]
    M = vk.block_jacobi(A, 8)
    b = twin.rhs(p.n)
    xg, info = vk.gmres(A, b, rtol=1e-8, M=M)
    st = vk.last_stats()
    g = golden_large["C1"]["gmres_bj8"]
    assert info == g["info"] == 0
    assert abs(st.inner_iters - g["inner_iters"]) <= 1
    assert np.linalg.norm(xg) == pytest.approx(g["x_norm2"], rel=1e-9)
    assert st.orth == (0 if orth == "mgs" else 1)
    np.testing.assert_allclose(xg[:8], g["x_first8"], rtol=1e-8)
    res = np.linalg.norm(b - coracle.spmv(ip, ix, d, xg))
    assert res <= 1e-8 * g["b_norm2"]


def test_orth_auto_default(ops):
    import vtkrylov as vk
    p, A, _ = ops["S2"]
    M = vk.block_jacobi(A, 8)
    b = twin.rhs(p.n)
    vk.gmres(A, b, rtol=1e-8, M=M)
    assert vk.last_stats().orth == 1                     # restart 20 -> DCGS2
    vk.gmres(A, b, rtol=1e-8, M=M, restart=40)
    assert vk.last_stats().orth == 0                     # restart 40 -> MGS
    x1, _ = vk.gmres(A, b, rtol=1e-8, M=M, orth="mgs")
    assert vk.last_stats().orth == 0
    x2, _ = vk.gmres(A, b, rtol=1e-8, M=M)
    assert vk.last_stats().orth == 1                     # per-call choice does not stick
    assert np.linalg.norm(x1 - x2) / np.linalg.norm(x1) < 1e-10


def test_gmres_device_tensors(ops, orth):
    import torch

    import vtkrylov as vk
    p, A, (ip, ix, d) = ops["S2"]
    M = vk.block_jacobi(A, 8)
    b = twin.rhs(p.n)
    xh, infoh = vk.gmres(A, b, rtol=1e-8, M=M)
    bt = torch.from_numpy(b).to("cuda:0")
    xt, infot = vk.gmres(A, bt, rtol=1e-8, M=M)
    assert infot == infoh == 0
    assert np.array_equal(xt.cpu().numpy(), xh)      # same kernels, same order: bitwise
    yt = A @ bt
    assert np.array_equal(yt.cpu().numpy(), A @ b)


@pytest.mark.slow
def test_gmres_c3_full_size(gpu, vk_lib, orth):
    """C3 (20M rows): the bench workload.  Size-independent properties: convergence to
    rtol, the true residual recomputed on the host by the oracle SpMV, and repeatability."""
    vk = vk_lib
    p = twin.CONFIGS["C3"]
    A = vk.vlasov_operator(_vk_params(vk, p), ctx=gpu)
    M = vk.block_jacobi(A, 8)
    b = vk.rhs_splitmix(p.n)
    x1, info = vk.gmres(A, b, rtol=1e-8, M=M)
    st = vk.last_stats()
    assert info == 0
    ip, ix, d = A.download()
    res = np.linalg.norm(b - coracle.spmv(ip, ix, d, x1))
    assert res <= 1e-8 * np.linalg.norm(b)
    assert st.rnorm == pytest.approx(res, rel=1e-6)
    x2, _ = vk.gmres(A, b, rtol=1e-8, M=M)
    assert np.array_equal(x1, x2)      # deterministic reductions
