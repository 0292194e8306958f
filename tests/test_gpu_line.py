"""GPU parity of the line-Jacobi preconditioner through the C-ABI.
Bars: factors and apply bit-identical to the C oracle (orc_line_setup / orc_line_apply: same
IEEE operations, -ffp-contract=off on both sides); apply within 1e-12 of SciPy's splu solve
(golden_line.npz); GMRES with M = line Jacobi: same info, inner iterations +-1,
||x - x_ref|| / ||x_ref|| <= 1e-9 against the oracle and SciPy; multi-rank: per-rank factors
bit-identical to the oracle's row-block factors, and with seg dividing every rank's x-range the
distributed solve matches the single-rank oracle."""
import os
import socket

import numpy as np
import pytest

from oracle import coracle, twin

pytestmark = pytest.mark.gpu

SMALL = ["C0", "S2", "S4", "S4F"]
SEG = 25


def stride_of(p):
    return 1 if p.dim == 1 else (p.shape[1] if p.dim == 2 else p.n // p.shape[0])


def bits(a):
    return np.ascontiguousarray(a).view(np.uint64)


@pytest.fixture(scope="module")
def ops(gpu, vk_lib):
    vk = vk_lib
    out = {}
    for name in SMALL + ["C1"]:
        p = twin.CONFIGS[name]
        out[name] = (p, vk.vlasov_operator(vk.vlasov_params(p.dim, p.shape, fp32=p.fp32), ctx=gpu),
                     coracle.generate(p))
    return out


@pytest.mark.parametrize("name", SMALL + ["C1"])
@pytest.mark.parametrize("seg", [1, 3, 8, 16, SEG, 32, 40, 1 << 30])
def test_line_factors_and_apply_bitexact(ops, vk_lib, name, seg):
    """Every apply variant: register sweeps (seg <= 8/16/25/32) and the generic one (> 32)."""
    p, A, (ip, ix, d) = ops[name]
    if name == "C1" and seg == 1 << 30:
        seg = 625               # whole-ish lines of C1 without a 1250-step serial lane
    st = stride_of(p)
    assert vk_lib.vlasov_line_stride(vk_lib.vlasov_params(p.dim, p.shape)) == st
    M = vk_lib.line_jacobi(A, st, seg)
    lf = coracle.line_setup(ip, ix, d, st, seg)
    assert np.array_equal(bits(M.factors()), bits(lf.f))
    r = twin.rhs(p.n)
    assert np.array_equal(bits(M @ r), bits(coracle.line_apply(lf, r)))


@pytest.mark.parametrize("name", SMALL)
@pytest.mark.parametrize("seg", [3, SEG])
def test_line_apply_vs_scipy(ops, vk_lib, golden_line, name, seg):
    p, A, _ = ops[name]
    z = vk_lib.line_jacobi(A, stride_of(p), seg) @ twin.rhs(p.n)
    np.testing.assert_allclose(z, golden_line[f"{name}/line{seg}_z"], rtol=1e-12, atol=1e-14)


def test_line_ragged_csr(gpu, vk_lib, golden, golden_line):
    vk = vk_lib
    ip, ix, d = golden["ragged/indptr"], golden["ragged/indices"], golden["ragged/data"]
    n = ip.shape[0] - 1
    A = vk.csr_matrix((d, ix, ip), shape=(n, n), ctx=gpu)
    M = vk.line_jacobi(A, 37, 5)
    lf = coracle.line_setup(ip, ix, d, 37, 5)
    assert np.array_equal(bits(M.factors()), bits(lf.f))
    r = twin.rhs(n)
    z = M @ r
    assert np.array_equal(bits(z), bits(coracle.line_apply(lf, r)))
    np.testing.assert_allclose(z, golden_line["ragged/line37_5_z"], rtol=1e-12, atol=1e-14)


def test_line_device_tensor_apply(ops, vk_lib):
    import torch
    p, A, _ = ops["S2"]
    M = vk_lib.line_jacobi(A, stride_of(p), SEG)
    r = twin.rhs(p.n)
    zt = M @ torch.from_numpy(r).to("cuda:0")
    assert np.array_equal(zt.cpu().numpy(), M @ r)


def test_line_singular_and_bad_args(gpu, vk_lib):
    vk = vk_lib
    n = 16
    ip = np.arange(n + 1, dtype=np.int32)
    ix = np.arange(n, dtype=np.int32)
    d = np.ones(n)
    d[5] = 0.0
    A = vk.csr_matrix((d, ix, ip), shape=(n, n), ctx=gpu)
    with pytest.raises(np.linalg.LinAlgError):
        vk.line_jacobi(A, 2, 4)
    with pytest.raises(ValueError):
        vk.line_jacobi(A, 0, 4)
    d[5] = 1.0
    B = vk.csr_matrix((d, ix, ip), shape=(n, n), ctx=gpu)
    M = vk.line_jacobi(B, 2, 4)
    with pytest.raises(vk._abi.VtkError):     # a line M is not a block-Jacobi M
        vk._abi.check(vk._abi.lib().vtk_bjacobi_set_mode(M.handle, 1), B.ctx.handle)
    np.testing.assert_array_equal(M @ np.arange(n, dtype=np.float64), np.arange(n, dtype=np.float64))


def test_line_tiny_systems(gpu, vk_lib):
    """1x1, a block shorter than one line, n not a multiple of the stride."""
    vk = vk_lib
    for n, st, seg in [(1, 1, 1), (5, 1, 25), (37, 8, 3), (100, 7, 25)]:
        rng = np.random.default_rng(n)
        rows, cols = [], []
        for r in range(n):
            for c in {r, r - st, r + st, (r * 7 + 3) % n}:
                if 0 <= c < n:
                    rows.append(r)
                    cols.append(c)
        import scipy.sparse as sp
        Asp = sp.csr_matrix((rng.standard_normal(len(rows)), (rows, cols)), shape=(n, n))
        Asp = sp.csr_matrix(Asp + sp.diags(np.abs(Asp).sum(axis=1).A1 + 1.0))
        ip, ix, d = Asp.indptr.astype(np.int32), Asp.indices.astype(np.int32), Asp.data
        A = vk.csr_matrix((d, ix, ip), shape=(n, n), ctx=gpu)
        M = vk.line_jacobi(A, st, seg)
        lf = coracle.line_setup(ip, ix, d, st, seg)
        assert np.array_equal(bits(M.factors()), bits(lf.f))
        r = twin.rhs(n)
        assert np.array_equal(bits(M @ r), bits(coracle.line_apply(lf, r)))


@pytest.fixture(params=["mgs", "dcgs2"])
def orth(request, gpu, vk_lib):
    gpu.set_orth({"mgs": vk_lib._abi.ORTH_MGS, "dcgs2": vk_lib._abi.ORTH_DCGS2}[request.param])
    yield request.param
    gpu.set_orth(vk_lib._abi.ORTH_AUTO)


def _check(xg, info, iters, ref_x, ref_info, ref_iters, tol=1e-9):
    assert info == ref_info
    assert abs(iters - ref_iters) <= 1, (iters, ref_iters)
    rel = np.linalg.norm(xg - ref_x) / max(np.linalg.norm(ref_x), 1e-300)
    assert rel <= tol, rel


@pytest.mark.parametrize("name", SMALL)
@pytest.mark.parametrize("layout", ["csr", "sell"])
def test_gmres_line_vs_oracle_and_scipy(ops, vk_lib, golden_line, name, layout, orth):
    vk = vk_lib
    p, A, (ip, ix, d) = ops[name]
    A.set_layout(layout)
    try:
        M = vk.line_jacobi(A, stride_of(p), SEG)
        b = twin.rhs(p.n)
        xg, info = vk.gmres(A, b, rtol=1e-8, M=M)
        st = vk.last_stats()
    finally:
        A.set_layout("auto")
    ref = coracle.gmres(ip, ix, d, b, coracle.line_setup(ip, ix, d, stride_of(p), SEG), rtol=1e-8)
    _check(xg, info, st.inner_iters, ref.x, ref.info, ref.inner_iters)
    meta = golden_line[f"{name}/gmres_line_meta"]
    _check(xg, info, st.inner_iters, golden_line[f"{name}/gmres_line_x"], int(meta[0]), int(meta[1]))
    assert np.linalg.norm(b - coracle.spmv(ip, ix, d, xg)) <= 1e-8 * np.linalg.norm(b)


def test_gmres_line_c1_vs_scipy_summary(ops, vk_lib, golden_large, orth):
    vk = vk_lib
    p, A, (ip, ix, d) = ops["C1"]
    g = golden_large["C1"][f"gmres_line{SEG}"]
    M = vk.line_jacobi(A, g["stride"], g["seg"])
    b = twin.rhs(p.n)
    xg, info = vk.gmres(A, b, rtol=1e-8, M=M)
    st = vk.last_stats()
    assert info == g["info"] == 0
    assert abs(st.inner_iters - g["inner_iters"]) <= 1
    assert np.linalg.norm(xg) == pytest.approx(g["x_norm2"], rel=1e-9)
    np.testing.assert_allclose(xg[:8], g["x_first8"], rtol=1e-8)
    assert np.linalg.norm(b - coracle.spmv(ip, ix, d, xg)) <= 1e-8 * g["b_norm2"]


# ---- several ranks sharing the GPU (host-staged communicator, as test_gpu_multirank) -------

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, case, outdir, orth):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import vtkrylov as vk
    ctx = vk.Context(0)
    hc = ctx.comm_init_host(rank, world)
    p = twin.CONFIGS[case]
    st = stride_of(p)
    offs = vk.partition_rows(p.n, world, st)
    rb, re_ = int(offs[rank]), int(offs[rank + 1])
    A = vk.vlasov_operator(vk.vlasov_params(p.dim, p.shape, fp32=p.fp32), ctx=ctx, offsets=offs)
    M = vk.line_jacobi(A, st, SEG)
    f = M.factors()
    b = twin.rhs(p.n)
    z = M @ b[rb:re_]
    xs, info = vk.gmres(A, b[rb:re_], rtol=1e-8, M=M, orth=orth)
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), f=f, z=z, x=xs, info=info,
             iters=vk.last_stats().inner_iters, rb=rb, re=re_,
             errors=np.array(hc.errors, dtype=object).astype(str))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("case,world,orth", [("C1", 2, "dcgs2"), ("S2", 3, "mgs"), ("S4", 2, "dcgs2")])
def test_line_ranks_sharing_one_gpu(tmp_path, case, world, orth):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(world, _free_port(), case, str(tmp_path), orth), nprocs=world, join=True)
    p = twin.CONFIGS[case]
    st = stride_of(p)
    ip, ix, d = coracle.generate(p)
    b = twin.rhs(p.n)
    xs = np.zeros(p.n)
    aligned = True
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz", allow_pickle=False)
        assert z["errors"].size == 0, z["errors"]
        rb, re_ = int(z["rb"]), int(z["re"])
        aligned &= (rb // st) % SEG == 0
        bip, bix, bd = coracle.generate(p, rb, re_)
        lf = coracle.line_setup(bip, bix, bd, st, SEG, row0=rb)
        assert np.array_equal(bits(z["f"]), bits(lf.f))                  # rank-local factors
        assert np.array_equal(bits(z["z"]), bits(coracle.line_apply(lf, b[rb:re_])))
        assert int(z["info"]) == 0
        xs[rb:re_] = z["x"]
    assert np.linalg.norm(b - coracle.spmv(ip, ix, d, xs)) <= 1e-8 * np.linalg.norm(b)
    if aligned:   # M does not depend on the rank count: the single-rank oracle solve
        ref = coracle.gmres(ip, ix, d, b, coracle.line_setup(ip, ix, d, st, SEG), rtol=1e-8)
        z0 = np.load(tmp_path / "rank0.npz", allow_pickle=False)
        assert abs(int(z0["iters"]) - ref.inner_iters) <= 1
        assert np.linalg.norm(xs - ref.x) / np.linalg.norm(ref.x) <= 1e-9



@pytest.mark.parametrize("name", SMALL + ["C1"])
def test_compact_apply_bitexact_vs_stored_factors(ops, gpu, vk_lib, name):
    """The Vlasov operators' x-couplings are constant along each line: the compact apply (l, g
    formed from a_j, c_j and m) must give the stored-factor apply's bits, in GMRES too (both
    through the two-kernel line step, line_fuse 0: the fused one needs the compact factors)."""
    vk = vk_lib
    p, A, _ = ops[name]
    M = vk.line_jacobi(A, stride_of(p), SEG)
    assert M.compact_available and M.compact
    r = twin.rhs(p.n)
    zc = M @ r
    b = twin.rhs(p.n)
    with gpu.tuning(line_fuse=0):
        xc, ic = vk.gmres(A, b, rtol=1e-8, M=M)
    M.set_compact(False)
    assert not M.compact
    assert np.array_equal(bits(zc), bits(M @ r))
    with gpu.tuning(line_fuse=0):
        xg, ig = vk.gmres(A, b, rtol=1e-8, M=M)
    assert ic == ig == 0 and np.array_equal(bits(xc), bits(xg))


def test_compact_unavailable_on_general_csr(gpu, vk_lib, golden):
    vk = vk_lib
    ip, ix, d = golden["ragged/indptr"], golden["ragged/indices"], golden["ragged/data"]
    n = ip.shape[0] - 1
    M = vk.line_jacobi(vk.csr_matrix((d, ix, ip), shape=(n, n), ctx=gpu), 37, 5)
    assert not M.compact_available and not M.compact
    with pytest.raises(ValueError):
        M.set_compact(True)


@pytest.mark.slow
@pytest.mark.parametrize("name", ["C3", "C4"])
def test_gmres_line_full_size(gpu, vk_lib, name):
    """BASELINE sizes (C3 20M rows, C4 50M rows fp32): size-independent properties - the true
    residual recomputed on the host by the oracle SpMV meets rtol, the factors' compact mode is
    taken, two solves are bit-identical, and the line preconditioner needs far fewer iterations
    than BJ(8) on the same system."""
    vk = vk_lib
    p = twin.CONFIGS[name]
    A = vk.vlasov_operator(vk.vlasov_params(p.dim, p.shape, fp32=p.fp32), ctx=gpu)
    M = vk.line_jacobi(A, stride_of(p), SEG)
    assert M.compact
    b = vk.rhs_splitmix(p.n)
    x1, info = vk.gmres(A, b, rtol=1e-8, M=M)
    it_line = vk.last_stats().inner_iters
    assert info == 0
    ip, ix, d = A.download()
    res = np.linalg.norm(b - coracle.spmv(ip, ix, d, x1))
    assert res <= 1e-8 * np.linalg.norm(b)
    x2, _ = vk.gmres(A, b, rtol=1e-8, M=M)
    assert np.array_equal(bits(x1), bits(x2))
    M.close()
    vk.gmres(A, b, rtol=1e-8, M=vk.block_jacobi(A, 8))
    assert it_line * 1.5 < vk.last_stats().inner_iters


def test_line_path_separable_spmv_bit_identical(vk_lib, gpu):
    """On a line-separable operator the line path's SpMV reads the values from the tables
    (k_lsv_spmv): k_sell's plain sum in the same order, so the solve is
    bit-identical with band_lsv off (the SELL values)."""
    import os
    import numpy as np
    from oracle import twin
    p = twin.CONFIGS["C1"]
    A = vk_lib.vlasov_operator(vk_lib.vlasov_params(p.dim, p.shape, fp32=p.fp32), ctx=gpu)
    assert A.line_separable
    M = vk_lib.line_jacobi(A, vk_lib.vlasov_line_stride(vk_lib.vlasov_params(p.dim, p.shape)), 25)
    b = twin.rhs(p.n)
    # (line_fuse 0: the SpMV as its own kernel, whose output the sweep kernel reads)
    with gpu.tuning(line_fuse=0):
        x1, i1 = vk_lib.gmres(A, b, rtol=1e-8, M=M)
        it1 = vk_lib.last_stats().inner_iters
    with gpu.tuning(band_lsv=0, line_fuse=0):
        x0, i0 = vk_lib.gmres(A, b, rtol=1e-8, M=M)
    assert i1 == i0 == 0 and it1 == vk_lib.last_stats().inner_iters
    assert np.array_equal(x1, x0)
    with gpu.tuning(sell_canon=0, line_fuse=0):   # the SELL codes instead of canon_row's columns
        x2, i2 = vk_lib.gmres(A, b, rtol=1e-8, M=M)
    assert i2 == 0 and it1 == vk_lib.last_stats().inner_iters
    assert np.array_equal(x1, x2)
    for wgs in (64, 2048):   # x staged through LDS (k_lsv_ring): the same products, the same order
        with gpu.tuning(lsv_ring=wgs, line_fuse=0):
            x3, i3 = vk_lib.gmres(A, b, rtol=1e-8, M=M)
        assert i3 == 0 and it1 == vk_lib.last_stats().inner_iters
        assert np.array_equal(x1, x3), wgs
    M.close()
    A.close()


@pytest.mark.parametrize("name,seg", [("C1", 25), ("S2", 8), ("S2", 3), ("C1", 32)])
def test_line_spmv_fused_into_sweep(vk_lib, gpu, name, seg):
    """The default one-rank line path forms the SpMV inside the sweep kernel (k_line_spmv_dc,
    DESIGN.md §3f): the same products, order and sweeps, the dots grouped by 62-lane blocks --
    within the DCGS2 bars of the two-kernel form, deterministic, and against the C oracle's
    line-Jacobi GMRES; x0 != 0 and restart 5 (several cycles) too."""
    import numpy as np
    from oracle import twin
    p = twin.CONFIGS[name]
    A = vk_lib.vlasov_operator(vk_lib.vlasov_params(p.dim, p.shape, fp32=p.fp32), ctx=gpu)
    M = vk_lib.line_jacobi(A, vk_lib.vlasov_line_stride(vk_lib.vlasov_params(p.dim, p.shape)), seg)
    b = twin.rhs(p.n)
    x0 = twin.rhs(p.n, seed=0xB0B) * 1e-3
    # the kernel-level pin: w = M^-1 A p from the fused kernel (k_line_spmv_dc) is the
    # two-kernel form's (table SpMV, then the sweeps), bit for bit
    pv = twin.rhs(p.n, seed=0xC0FFEE)
    gpu.profile(True)
    wf = A.precond_matvec(M, pv)
    assert gpu.profile_read().get("line_dc", {}).get("launches", 0) == 1   # the fused kernel ran
    gpu.profile(False)
    with gpu.tuning(line_fuse=0):
        wu = A.precond_matvec(M, pv)
    assert np.array_equal(wf, wu)
    assert np.array_equal(wu, M.matvec(A @ pv))
    for kw in ({}, {"x0": x0}, {"restart": 5}):
        gpu.profile(True)
        xf, i_f = vk_lib.gmres(A, b, rtol=1e-8, M=M, orth="dcgs2", **kw)
        st_f = vk_lib.last_stats()
        prof = gpu.profile_read()
        gpu.profile(False)
        assert "spmv_lsv" not in prof or prof["spmv_lsv"]["launches"] == 0, sorted(prof)   # the fused kernel ran
        xg, _ = vk_lib.gmres(A, b, rtol=1e-8, M=M, orth="dcgs2", **kw)
        assert np.array_equal(xf, xg) and vk_lib.last_stats().inner_iters == st_f.inner_iters
        with gpu.tuning(line_fuse=0):
            xu, i_u = vk_lib.gmres(A, b, rtol=1e-8, M=M, orth="dcgs2", **kw)
            st_u = vk_lib.last_stats()
        assert i_f == i_u == 0, kw
        assert abs(st_f.inner_iters - st_u.inner_iters) <= 1, kw
        assert np.linalg.norm(xf - xu) / np.linalg.norm(xu) < 1e-9, kw
    M.close()
    A.close()
