"""The drop-in path gets the fast solver: a CSR handed over the way the
reference's scipy.sparse path would hand it -- ``vtkrylov.csr_matrix`` of a SciPy matrix, of
host arrays or of device tensors, ``vtkrylov.load_npz`` of a ``save_npz`` archive -- is checked
for the 2D Vlasov x-line structure inside ``vtk_csr_create`` (candidate line length from the
first and last rows' columns, then the same device checks as ``vtk_csr_set_line_band``).  When
it holds, the operator gets the line band, the line-separable tables and canonical rows, and
GMRES runs the band step exactly as on the generated operator: the same bits.
"""
import numpy as np
import pytest

from oracle import coracle, twin

pytestmark = pytest.mark.gpu


def _solve(vk, A, M, b, **kw):
    x, info = vk.gmres(A, b, rtol=kw.pop("rtol", 1e-8), M=M, **kw)
    return x, info, vk.last_stats()


@pytest.mark.parametrize("name", ["S2", "C1"])
@pytest.mark.parametrize("how", ["scipy", "arrays", "device", "npz"])
def test_uploaded_csr_runs_the_band_step_bit_identical(vk_lib, gpu, tmp_path, name, how):
    import scipy.sparse as sp
    p = twin.CONFIGS[name]
    G = vk_lib.vlasov_operator(vk_lib.vlasov_params(p.dim, p.shape), ctx=gpu)
    ip, ix, d = G.download()
    if how == "scipy":
        A = vk_lib.csr_matrix(sp.csr_matrix((d, ix, ip), shape=(p.n, p.n)), ctx=gpu)
    elif how == "arrays":
        A = vk_lib.csr_matrix((d, ix, ip), shape=(p.n, p.n), ctx=gpu)
    elif how == "device":
        import torch
        dev = torch.device("cuda", gpu.device)
        A = vk_lib.csr_matrix((torch.from_numpy(d).to(dev), torch.from_numpy(ix).to(dev),
                               torch.from_numpy(ip).to(dev)), shape=(p.n, p.n), ctx=gpu)
    else:
        f = tmp_path / "A.npz"
        sp.save_npz(f, sp.csr_matrix((d, ix, ip), shape=(p.n, p.n)))
        A = vk_lib.load_npz(f, ctx=gpu)
    assert A.line_band == G.line_band == p.shape[1]
    assert A.line_values == G.line_values == 2     # separable values, canonical rows
    b = twin.rhs(p.n)
    MG, MA = vk_lib.block_jacobi(G, 8), vk_lib.block_jacobi(A, 8)
    xg, ig, sg = _solve(vk_lib, G, MG, b)
    xa, ia, sa = _solve(vk_lib, A, MA, b)
    assert sg.band == sa.band == 1 and ig == ia == 0
    assert sa.inner_iters == sg.inner_iters
    assert np.array_equal(xa, xg), "uploaded operator's solve differs from the generated one's"
    for o in (MG, MA, A, G):
        o.close()


def test_line_len_argument(vk_lib, gpu):
    """line_len=0 keeps the plain path; an explicit line length is required to hold."""
    import scipy.sparse as sp
    p = twin.CONFIGS["S2"]
    ip, ix, d = coracle.generate(p)
    S = sp.csr_matrix((d, ix, ip), shape=(p.n, p.n))
    A0 = vk_lib.csr_matrix(S, ctx=gpu, line_len=0)
    assert A0.line_band == 0 and A0.line_values == 0
    M0 = vk_lib.block_jacobi(A0, 8)
    x0, i0, s0 = _solve(vk_lib, A0, M0, coracle.rhs(p.n))
    assert s0.band == 0 and i0 == 0
    A1 = vk_lib.csr_matrix(S, ctx=gpu, line_len=p.shape[1])
    assert A1.line_band == p.shape[1]
    with pytest.raises(ValueError):   # x couplings two half-lines away: no such structure
        vk_lib.csr_matrix(S, ctx=gpu, line_len=p.shape[1] // 2)
    for o in (M0, A0, A1):
        o.close()


def test_detection_can_be_switched_off(vk_lib, gpu):
    import scipy.sparse as sp
    p = twin.CONFIGS["S2"]
    ip, ix, d = coracle.generate(p)
    with gpu.tuning(auto_band=0):
        A = vk_lib.csr_matrix(sp.csr_matrix((d, ix, ip), shape=(p.n, p.n)), ctx=gpu)
    assert A.line_band == 0
    A.close()


@pytest.mark.parametrize("name", ["C0", "S4"])
def test_no_band_where_there_is_none(vk_lib, gpu, name):
    """1D (every coupling within one row) and 4D (x couplings Ny*Nvx*Nvy rows away): the
    candidate fails the device check, the operator keeps the plain path, nothing raises."""
    p = twin.CONFIGS[name]
    ip, ix, d = coracle.generate(p)
    A = vk_lib.csr_matrix((d, ix, ip), shape=(p.n, p.n), ctx=gpu)
    assert A.line_band == 0
    M = vk_lib.block_jacobi(A, 8)
    b = coracle.rhs(p.n)
    x, info, st = _solve(vk_lib, A, M, b)
    ref = coracle.gmres(ip, ix, d, b, coracle.bj_setup(ip, ix, d, 8), rtol=1e-8)
    assert st.band == 0 and info == ref.info == 0
    assert abs(st.inner_iters - ref.inner_iters) <= 1
    assert np.linalg.norm(x - ref.x) / np.linalg.norm(ref.x) < 1e-9
    M.close()
    A.close()


def test_ragged_and_random_csr_unaffected(vk_lib, gpu):
    """Ragged random CSR (empty rows, a long row): no line band, SpMV still bit-identical to SciPy."""
    import scipy.sparse as sp
    rng = np.random.default_rng(7)
    n = 2000
    R = sp.random(n, n, density=0.003, random_state=11, format="csr") + sp.identity(n, format="csr")
    R = R.tolil()
    R[5, :] = 0
    R[17, rng.choice(n, 600, replace=False)] = 1.5
    R = R.tocsr()
    A = vk_lib.csr_matrix(R, ctx=gpu)
    assert A.line_band == 0
    x = rng.standard_normal(n)
    assert np.array_equal(A @ x, R @ x)
    A.close()


def test_device_csr_overlong_indptr_rejected(vk_lib, gpu):
    """indptr[-1] beyond the index / value tensors is refused before any copy."""
    import torch
    p = twin.CONFIGS["S2"]
    ip, ix, d = coracle.generate(p)
    dev = torch.device("cuda", gpu.device)
    ipt = torch.from_numpy(ip.copy()).to(dev)
    ipt[-1] = ix.shape[0] + 1000
    with pytest.raises(ValueError):
        vk_lib.csr_matrix((torch.from_numpy(d).to(dev), torch.from_numpy(ix).to(dev), ipt), shape=(p.n, p.n), ctx=gpu)
    with pytest.raises(ValueError):   # wrong indptr length
        vk_lib.csr_matrix((torch.from_numpy(d).to(dev), torch.from_numpy(ix).to(dev),
                           torch.from_numpy(ip[:-1].copy()).to(dev)), shape=(p.n, p.n), ctx=gpu)
    with pytest.raises(ValueError):   # host arrays, too
        ip2 = ip.copy()
        ip2[-1] += 5
        vk_lib.csr_matrix((d, ix, ip2), shape=(p.n, p.n), ctx=gpu)


def test_destroy_in_any_order(vk_lib):
    """Finalisers of a reference cycle run in any order: a preconditioner destroyed after its
    operator, and an operator after its context, must not touch the freed parent."""
    import scipy.sparse as sp
    p = twin.CONFIGS["S2"]
    ip, ix, d = coracle.generate(p)
    ctx = vk_lib.Context(0)
    A = vk_lib.csr_matrix(sp.csr_matrix((d, ix, ip), shape=(p.n, p.n)), ctx=ctx)
    M = vk_lib.block_jacobi(A, 8)
    L = vk_lib.line_jacobi(A, p.shape[1], 8)
    A.close()
    M.close()
    L.close()
    B = vk_lib.csr_matrix(sp.csr_matrix((d, ix, ip), shape=(p.n, p.n)), ctx=ctx)
    ctx.close()
    B.close()


@pytest.mark.parametrize("name", ["S4", "S4F"])
def test_grid4_rows_bit_identical(vk_lib, gpu, name):
    """4D grid rows (vtk_csr_set_grid4): the solver's SELL launches take the columns
    from the row's coordinates and the values from D and the per-coordinate tables -- the same
    entries in the same order as the SELL copy, so x is bit-identical with the grid4 switch off;
    the uploaded CSR is detected as a grid too."""
    p = twin.CONFIGS[name]
    G = vk_lib.vlasov_operator(vk_lib.vlasov_params(p.dim, p.shape, fp32=p.fp32), ctx=gpu)
    assert G.grid4 == tuple(p.shape[1:])
    ip, ix, d = G.download()
    U = vk_lib.csr_matrix((d, ix, ip), shape=(p.n, p.n), ctx=gpu)
    assert U.grid4 == tuple(p.shape[1:])
    b = twin.rhs(p.n)
    out = []
    for A in (G, U):
        M = vk_lib.block_jacobi(A, 8)
        # the kernel-level pin: w = M^-1 A x from the ring kernel (k_g4_ring, 512- and
        # 256-row groups, 1 .. 4096 workgroups, the inner-wave sum on and off) is the SELL
        # grid-row kernel's (k_sell<EPI_PREC>) and the SELL-value kernel's, bit for bit
        xr = twin.rhs(p.n, seed=0xC0FFEE)
        with gpu.tuning(g4_ring=0):
            w_sell = A.precond_matvec(M, xr)
        with gpu.tuning(g4_ring=0, grid4=0):
            w_vals = A.precond_matvec(M, xr)
        assert np.array_equal(w_sell, w_vals)
        for wgs, gr, fast in ((2048, 512, 1), (2048, 512, 0), (1, 256, 1), (7, 256, 0), (4096, 256, 1), (5, 512, 1)):
            with gpu.tuning(g4_ring=wgs, g4_gr=gr, g4_fast=fast):
                assert np.array_equal(A.precond_matvec(M, xr), w_sell), (wgs, gr, fast)
        for orth in ("dcgs2", "mgs"):
            with gpu.tuning(c4_fused=0, g4_ring=0):   # the split step (SELL SpMV + BJ, then the dots)
                x1, i1, s1 = _solve(vk_lib, A, M, b, orth=orth)
            with gpu.tuning(grid4=0):      # ... reading the SELL values and codes
                x0, i0, s0 = _solve(vk_lib, A, M, b, orth=orth)
            with gpu.tuning(g4_ring=0):    # grid rows, dots fused into the SELL kernel
                x2, i2, s2 = _solve(vk_lib, A, M, b, orth=orth)
            assert i1 == i0 == i2 == 0 and s1.inner_iters == s0.inner_iters
            assert np.array_equal(x1, x0), "grid rows change the bits"
            # the split step's SpMV + BJ with x staged through LDS (k_g4_ring), in 256- and 512-row
            # groups over 1 .. 4096 workgroups, step 0's dots and the cycle-start residual in the
            # ring kernel: its partials follow the workgroups (reductions in another fixed order:
            # the solver bars; deterministic per setting)
            for wgs, gr in ((1, 256), (3, 256), (4096, 256), (7, 256), (1, 512), (5, 512)):
                with gpu.tuning(c4_fused=0, g4_ring=wgs, g4_gr=gr):
                    x3, i3, s3 = _solve(vk_lib, A, M, b, orth=orth)
                    x3b, _, s3b = _solve(vk_lib, A, M, b, orth=orth)
                assert i3 == 0 and np.array_equal(x3, x3b) and s3.inner_iters == s3b.inner_iters, (wgs, gr)
                assert abs(s3.inner_iters - s1.inner_iters) <= 1, (wgs, gr)
                assert np.linalg.norm(x3 - x1) / np.linalg.norm(x1) < 1e-9, (wgs, gr)
            # default: the ring split step (2048 workgroups of 512 rows)
            xd, _, sd = _solve(vk_lib, A, M, b, orth=orth)
            with gpu.tuning(g4_fast=0):   # every wave through the general select chains
                xg, _, sg = _solve(vk_lib, A, M, b, orth=orth)
            assert np.array_equal(xd, xg) and sd.inner_iters == sg.inner_iters, "the inner-row sum changes the bits"
            xe, _, se = _solve(vk_lib, A, M, b, orth=orth, x0=b * 1e-3)
            xf, _, sf = _solve(vk_lib, A, M, b, orth=orth, x0=b * 1e-3)
            assert np.array_equal(xe, xf) and se.inner_iters == sf.inner_iters
            assert abs(sd.inner_iters - s1.inner_iters) <= 1
            assert np.linalg.norm(xd - x1) / np.linalg.norm(x1) < 1e-9
            if orth == "mgs":
                assert np.array_equal(x1, x2)
            else:   # the fused dots sum in another fixed order: the DCGS2 bars
                assert abs(s2.inner_iters - s1.inner_iters) <= 1
                assert np.linalg.norm(x2 - x1) / np.linalg.norm(x1) < 1e-9
            out.append(x1)
        M.close()
    assert np.array_equal(out[0], out[2]) and np.array_equal(out[1], out[3])
    ref = coracle.gmres(ip, ix, d, b, coracle.bj_setup(ip, ix, d, 8), rtol=1e-8)
    assert np.linalg.norm(out[1] - ref.x) / np.linalg.norm(ref.x) < 1e-9
    for o in (U, G):
        o.close()


def test_grid4_rejects_other_structures(vk_lib, gpu):
    import scipy.sparse as sp
    p = twin.CONFIGS["S4"]
    ip, ix, d = coracle.generate(p)
    A = vk_lib.csr_matrix(sp.csr_matrix((d, ix, ip), shape=(p.n, p.n)), ctx=gpu)
    with pytest.raises(ValueError):   # another split of the plane into (vx, vy)
        A.set_grid4(p.shape[1], p.shape[2] * 2, p.shape[3] // 2)
    assert A.grid4 == tuple(p.shape[1:])                   # the detected structure is kept
    A.set_grid4(0, 0, 0)
    assert A.grid4 == (0, 0, 0)
    d2 = d.copy()
    d2[ip[7]] *= 1.0 + 1e-6                                 # row 7's vy-1 coupling: no longer by iy alone
    B = vk_lib.csr_matrix(sp.csr_matrix((d2, ix, ip), shape=(p.n, p.n)), ctx=gpu)
    assert B.grid4 == (0, 0, 0)
    S2 = twin.CONFIGS["S2"]
    q = coracle.generate(S2)
    C2 = vk_lib.csr_matrix((q[2], q[1], q[0]), shape=(S2.n, S2.n), ctx=gpu)
    assert C2.grid4 == (0, 0, 0) and C2.line_band == S2.shape[1]
    for o in (A, B, C2):
        o.close()


@pytest.mark.parametrize("shape", [(520, 3, 4, 4), (3, 3, 64, 64)])
def test_grid4_past_ring_limits(vk_lib, gpu, shape):
    """4D grids past k_g4_ring's LDS limits -- the coordinate tables over 1024 doubles
    (520 x planes on one rank) or the y-line window over the ring (Nvx Nvy = 4096) -- solve
    through the SELL grid-row kernels instead of failing in the ring launch."""
    p = twin.Vlasov(4, shape)
    G = vk_lib.vlasov_operator(vk_lib.vlasov_params(4, shape), ctx=gpu)
    assert G.grid4 == tuple(shape[1:])
    ip, ix, d = G.download()
    M = vk_lib.block_jacobi(G, 8)
    b = twin.rhs(p.n)
    x, info, st = _solve(vk_lib, G, M, b)
    ref = coracle.gmres(ip, ix, d, b, coracle.bj_setup(ip, ix, d, 8), rtol=1e-8)
    assert info == ref.info == 0
    assert abs(st.inner_iters - ref.inner_iters) <= 1
    assert np.linalg.norm(x - ref.x) / np.linalg.norm(ref.x) < 1e-9
    M.close()
    G.close()
