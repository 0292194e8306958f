"""Line-band DCGS2 step (vtk_kernels.hip k_band_step): the update pass of step j
fused with step j+1's SpMV + tridiagonal BJ(8) + dots in one sweep over x-lines.

The band step performs the same update arithmetic as k_dc_update and the same SpMV / BJ
arithmetic as k_sell (v_j, p_{j+1} and w bit-identical for the same inputs); only the dot
products are summed in another fixed order.  So the solve follows the DCGS2 bars of
tests/test_gpu_parity.py against the band-off path, the C oracle (SciPy's sequence) and SciPy's
own summaries: same info, inner iterations +-1, ||x - x_ref|| / ||x_ref|| <= 1e-9, plus a
bit-identical repeat (deterministic reductions).  Full size (C2, C3): tests/test_gpu_large.py
runs the default path, which is this one (asserted there via stats.band).
"""
import numpy as np
import pytest

from oracle import coracle, twin

pytestmark = pytest.mark.gpu


def _op(vk, gpu, name):
    p = twin.CONFIGS[name]
    return p, vk.vlasov_operator(vk.vlasov_params(p.dim, p.shape, fp32=p.fp32), ctx=gpu)


def _solve(vk, gpu, A, M, b, band, **kw):
    gpu.set_band(band)
    try:
        x, info = vk.gmres(A, b, rtol=kw.pop("rtol", 1e-8), M=M, **kw)
    finally:
        gpu.set_band(True)
    return x, info, vk.last_stats()


@pytest.mark.parametrize("name", ["S2", "C1"])
def test_band_detected_on_2d_vlasov(vk_lib, gpu, name):
    p, A = _op(vk_lib, gpu, name)
    assert A.line_band == p.shape[1]
    A.close()


def test_band_not_set_on_4d_and_rejected_on_random(vk_lib, gpu):
    p, A = _op(vk_lib, gpu, "S4")
    assert A.line_band == 0
    # the 4D operator's x-couplings are Ny*Nvx*Nvy rows away: not within lines of Nvy rows
    with pytest.raises(ValueError):
        A.set_line_band(p.shape[3])
    A.close()
    import scipy.sparse as sp
    R = sp.random(640, 640, density=0.02, random_state=3, format="csr") + sp.identity(640, format="csr")
    B = vk_lib.csr_matrix(R.tocsr(), ctx=gpu)
    with pytest.raises(ValueError):
        B.set_line_band(64)
    B.set_line_band(0)
    assert B.line_band == 0
    B.close()


def test_band_explicit_on_uploaded_csr(vk_lib, gpu):
    """A SciPy CSR of the 2D operator uploaded as plain CSR with the detection off (line_len=0):
    set_line_band enables the path (the default detection: tests/test_gpu_dropin.py)."""
    p = twin.CONFIGS["S2"]
    ip, ix, d = coracle.generate(p)
    import scipy.sparse as sp
    A = vk_lib.csr_matrix(sp.csr_matrix((d, ix, ip), shape=(p.n, p.n)), ctx=gpu, line_len=0)
    assert A.line_band == 0
    A.set_line_band(p.shape[1])
    assert A.line_band == p.shape[1]
    M = vk_lib.block_jacobi(A, 8)
    b = coracle.rhs(p.n)
    x, info, st = _solve(vk_lib, gpu, A, M, b, True)
    assert st.band == 1 and info == 0
    ref = coracle.gmres(ip, ix, d, b, coracle.bj_setup(ip, ix, d, 8), rtol=1e-8)
    assert abs(st.inner_iters - ref.inner_iters) <= 1
    assert np.linalg.norm(x - ref.x) / np.linalg.norm(ref.x) < 1e-9
    M.close()
    A.close()


@pytest.mark.parametrize("restart", [2, 5, 20])
@pytest.mark.parametrize("name", ["S2", "C1"])
def test_band_vs_unfused_and_oracle(vk_lib, gpu, name, restart):
    p, A = _op(vk_lib, gpu, name)
    M = vk_lib.block_jacobi(A, 8)
    assert M.mode == "tridiag"
    ip, ix, d = A.download()
    b = coracle.rhs(p.n)
    xb, ib, sb = _solve(vk_lib, gpu, A, M, b, True, restart=restart, maxiter=400)
    xu, iu, su = _solve(vk_lib, gpu, A, M, b, False, restart=restart, maxiter=400)
    assert sb.band == 1 and su.band == 0
    assert ib == iu == 0
    assert abs(sb.inner_iters - su.inner_iters) <= 1
    assert np.linalg.norm(xb - xu) / np.linalg.norm(xu) < 1e-9
    ref = coracle.gmres(ip, ix, d, b, coracle.bj_setup(ip, ix, d, 8), rtol=1e-8, restart=restart, maxiter=400)
    assert ref.info == 0 and abs(sb.inner_iters - ref.inner_iters) <= 1, (sb.inner_iters, ref.inner_iters)
    assert np.linalg.norm(xb - ref.x) / np.linalg.norm(ref.x) < 1e-9
    # the true residual, recomputed on the host
    assert np.linalg.norm(b - coracle.spmv(ip, ix, d, xb)) <= 1e-8 * np.linalg.norm(b) * 1.0001
    M.close()
    A.close()


def test_band_nonzero_x0_and_repeat(vk_lib, gpu):
    p, A = _op(vk_lib, gpu, "C1")
    M = vk_lib.block_jacobi(A, 8)
    ip, ix, d = A.download()
    b = coracle.rhs(p.n)
    x0 = twin.rhs(p.n, seed=0xB00) * 1e-3
    x1, i1, s1 = _solve(vk_lib, gpu, A, M, b, True, x0=x0.copy())
    x2, i2, s2 = _solve(vk_lib, gpu, A, M, b, True, x0=x0.copy())
    assert s1.band == 1 and i1 == i2 == 0
    assert np.array_equal(x1, x2), "band solve not bit-identical on repeat"
    ref = coracle.gmres(ip, ix, d, b, coracle.bj_setup(ip, ix, d, 8), x0=x0.copy(), rtol=1e-8)
    assert abs(s1.inner_iters - ref.inner_iters) <= 1
    assert np.linalg.norm(x1 - ref.x) / np.linalg.norm(ref.x) < 1e-9
    M.close()
    A.close()


def test_band_off_for_inverse_mode_and_long_restart(vk_lib, gpu):
    p, A = _op(vk_lib, gpu, "S2")
    M = vk_lib.block_jacobi(A, 8, mode="inverse")
    b = coracle.rhs(p.n)
    _, info, st = _solve(vk_lib, gpu, A, M, b, True)
    assert info == 0 and st.band == 0
    M.set_mode("auto")
    _, info, st = _solve(vk_lib, gpu, A, M, b, True, restart=25)
    assert info == 0 and st.band == 0
    M.close()
    A.close()


def test_band_c1_vs_scipy_summary(vk_lib, gpu, golden_large):
    """C1 against SciPy 1.15.3's own GMRES(20) + BJ(8) summary (golden_large.json)."""
    g = golden_large["C1"]["gmres_bj8"]
    p, A = _op(vk_lib, gpu, "C1")
    M = vk_lib.block_jacobi(A, 8)
    b = vk_lib.rhs_splitmix(p.n)
    x, info, st = _solve(vk_lib, gpu, A, M, b, True)
    assert st.band == 1
    assert info == g["info"] == 0
    assert abs(st.inner_iters - g["inner_iters"]) <= 1
    assert np.linalg.norm(x) == pytest.approx(g["x_norm2"], rel=1e-9)
    M.close()
    A.close()


@pytest.mark.parametrize("shape", [(48, 8), (40, 816), (24, 1000)])
def test_band_other_line_lengths(vk_lib, gpu, shape):
    """Line lengths giving one part (L = 8), three parts of 272 rows (L = 816) and five parts of
    200 rows (L = 1000): the v-halo rows between parts and the per-line boundary copies."""
    p = twin.Vlasov(2, shape)
    A = vk_lib.vlasov_operator(vk_lib.vlasov_params(2, shape), ctx=gpu)
    assert A.line_band == shape[1]
    M = vk_lib.block_jacobi(A, 8)
    ip, ix, d = A.download()
    b = coracle.rhs(p.n)
    xb, ib, sb = _solve(vk_lib, gpu, A, M, b, True, maxiter=400)
    xu, iu, su = _solve(vk_lib, gpu, A, M, b, False, maxiter=400)
    assert sb.band == 1 and su.band == 0 and ib == iu == 0
    assert abs(sb.inner_iters - su.inner_iters) <= 1
    assert np.linalg.norm(xb - xu) / np.linalg.norm(xu) < 1e-9
    ref = coracle.gmres(ip, ix, d, b, coracle.bj_setup(ip, ix, d, 8), rtol=1e-8, maxiter=400)
    assert abs(sb.inner_iters - ref.inner_iters) <= 1
    assert np.linalg.norm(xb - ref.x) / np.linalg.norm(ref.x) < 1e-9
    M.close()
    A.close()


@pytest.mark.parametrize("name", ["S2", "C1"])
def test_band_line_separable_values_bit_identical(vk_lib, gpu, name):
    """The 2D Vlasov operators' values are line-separable (x couplings per position v, v couplings
    per line x; vtk_csr_get_line_values): the band step reads them from the tables -- the same
    values summed in the same order as from the SELL copy, so x is bit-identical with
    the context's band_lsv switch off."""
    import os
    p, A = _op(vk_lib, gpu, name)
    assert A.line_separable and A.line_values == 2   # the Vlasov rows are canonical too
    M = vk_lib.block_jacobi(A, 8)
    b = twin.rhs(p.n)
    # (cyc_ring 0: the cycle-start launches through k_sell, which sums its reductions in the same
    # order with and without the tables; the ring form is pinned by test_cycle_ring_epilogues.
    # band_opt 0: the one-rank variants' grid exists only with the tables and canonical rows, and
    # the dots' partials follow the grid -- test_band_step_variants pins the variants)
    with gpu.tuning(cyc_ring=0, band_opt=0):
        x1, i1, s1 = _solve(vk_lib, gpu, A, M, b, True, restart=20)
    with gpu.tuning(band_lsv=0, cyc_ring=0, band_opt=0):
        x0, i0, s0 = _solve(vk_lib, gpu, A, M, b, True, restart=20)
    # canonical rows (the kinds' order from the row's line instead of the SELL codes) vs the codes
    with gpu.tuning(band_canon=0, cyc_ring=0, band_opt=0):
        x2, i2, s2 = _solve(vk_lib, gpu, A, M, b, True, restart=20)
    # the cycle-start SELL launches (residual + BJ, step 0's SpMV + BJ + dots) with their columns
    # from canon_row vs the codes
    with gpu.tuning(sell_canon=0, cyc_ring=0, band_opt=0):
        x3, i3, s3 = _solve(vk_lib, gpu, A, M, b, True, restart=20)
    assert s1.band == s0.band == s2.band == s3.band == 1 and i1 == i0 == i2 == i3 == 0
    assert s1.inner_iters == s0.inner_iters == s2.inner_iters == s3.inner_iters
    assert np.array_equal(x1, x0), "line-separable values change the band step's bits"
    assert np.array_equal(x1, x2), "canonical rows change the band step's bits"
    assert np.array_equal(x1, x3), "canonical rows change the SELL launches' bits"
    M.close()
    A.close()


def test_band_not_separable_falls_back(vk_lib, gpu):
    """One x coupling perturbed: still a line-band operator, no longer line-separable -- the band
    step reads the SELL values and the solve still meets the oracle on the perturbed matrix."""
    p = twin.CONFIGS["S2"]
    ip, ix, d = coracle.generate(p)
    import scipy.sparse as sp
    d = d.copy()
    L = p.shape[1]
    r = 5 * L + 7   # an interior row; its x+1 coupling (column r + L)
    k = ip[r] + int(np.nonzero(ix[ip[r]:ip[r + 1]] == r + L)[0][0])
    d[k] *= 1.0 + 1e-6
    A = vk_lib.csr_matrix(sp.csr_matrix((d, ix, ip), shape=(p.n, p.n)), ctx=gpu)
    A.set_line_band(L)
    assert A.line_band == L and not A.line_separable
    M = vk_lib.block_jacobi(A, 8)
    b = coracle.rhs(p.n)
    x, info, st = _solve(vk_lib, gpu, A, M, b, True)
    assert st.band == 1 and info == 0
    ref = coracle.gmres(ip, ix, d, b, coracle.bj_setup(ip, ix, d, 8), rtol=1e-8)
    assert abs(st.inner_iters - ref.inner_iters) <= 1
    assert np.linalg.norm(x - ref.x) / np.linalg.norm(ref.x) < 1e-9
    M.close()
    A.close()


@pytest.mark.parametrize("orth", ["dcgs2", "mgs"])
def test_separable_values_in_unfused_paths_bit_identical(vk_lib, gpu, orth):
    """The solver's other SELL launches (fused SpMV + BJ + dots, residual, MGS matvec) also read
    the line-separable tables on such operators: with the band step off, x is bit-identical with
    band_lsv off for both orthogonalisations."""
    import os
    p, A = _op(vk_lib, gpu, "C1")
    assert A.line_separable
    M = vk_lib.block_jacobi(A, 8)
    b = twin.rhs(p.n)
    with gpu.tuning(cyc_ring=0):
        x1, i1, s1 = _solve(vk_lib, gpu, A, M, b, False, orth=orth)
    with gpu.tuning(band_lsv=0, cyc_ring=0):
        x0, i0, s0 = _solve(vk_lib, gpu, A, M, b, False, orth=orth)
    with gpu.tuning(sell_canon=0, cyc_ring=0):   # the SELL codes instead of canon_row's columns
        x2, i2, s2 = _solve(vk_lib, gpu, A, M, b, False, orth=orth)
    assert s1.band == s0.band == s2.band == 0 and i1 == i0 == i2 == 0
    assert s1.inner_iters == s0.inner_iters == s2.inner_iters
    assert np.array_equal(x1, x0)
    assert np.array_equal(x1, x2)
    M.close()
    A.close()


@pytest.mark.parametrize("name,band,orth", [("S2", True, "dcgs2"), ("C1", True, "dcgs2"), ("C1", False, "mgs")])
def test_cycle_ring_epilogues(vk_lib, gpu, name, band, orth):
    """The cycle-start residual + BJ and the band cycle's step 0 through the x-line ring
    (k_lsv_ring_epi, tuning cyc_ring): the same row sums and BJ solves as k_sell's
    canonical rows, the norms and dots reduced in another fixed order -- within the solver bars
    of the k_sell form, bit-identical from run to run, for any workgroup count; several cycles
    (restart 5) and x0 != 0 so that every cycle starts with the ring residual."""
    p, A = _op(vk_lib, gpu, name)
    M = vk_lib.block_jacobi(A, 8)
    b = twin.rhs(p.n)
    x0 = twin.rhs(p.n, seed=0xB0B) * 1e-3
    with gpu.tuning(cyc_ring=0):
        xr, ir, sr = _solve(vk_lib, gpu, A, M, b, band, restart=5, orth=orth, x0=x0)
    for wgs in (1, 64, 1024):
        with gpu.tuning(cyc_ring=wgs):
            xa, ia, sa = _solve(vk_lib, gpu, A, M, b, band, restart=5, orth=orth, x0=x0)
            xb, ib, sb = _solve(vk_lib, gpu, A, M, b, band, restart=5, orth=orth, x0=x0)
        assert ia == ib == ir == 0 and sa.band == sr.band == int(band)
        assert np.array_equal(xa, xb) and sa.inner_iters == sb.inner_iters, wgs
        assert abs(sa.inner_iters - sr.inner_iters) <= 1, wgs
        assert np.linalg.norm(xa - xr) / np.linalg.norm(xr) < 1e-9, wgs
    M.close()
    A.close()


@pytest.mark.parametrize("name", ["S2", "C1"])
def test_band_step_variants(vk_lib, gpu, name):
    """The band step's launch variants (tunings band_opt: bit 0 the SpMV operands in the next-line
    prefetch, bit 1 three workgroups per CU for j <= 2 with their own grid): the same update,
    SpMV and BJ arithmetic; the dots' partials follow the grid, so the solves agree within the
    DCGS2 bars and each variant is bit-identical from run to run.  Bit 2 (a line range's two parts
    on one XCD: the partial slots follow the logical index) and bit 3 (the LDS-DMA L2 prefetch for
    J > 12) change no sum: bit-identical to the variant without them."""
    p, A = _op(vk_lib, gpu, name)
    M = vk_lib.block_jacobi(A, 8)
    b = twin.rhs(p.n)
    xr, ir, sr = _solve(vk_lib, gpu, A, M, b, True, restart=20)
    assert ir == 0
    with gpu.tuning(band_long_rows=0):   # bits 3, 4 at these sizes too (by default only >= 16M rows)
        _band_variants(vk_lib, gpu, A, M, b, xr, sr)
    M.close()
    A.close()


def _band_variants(vk_lib, gpu, A, M, b, xr, sr):
    for opt in (0, 1, 2, 3):
        with gpu.tuning(band_opt=opt):
            xa, ia, sa = _solve(vk_lib, gpu, A, M, b, True, restart=20)
            xb, ib, sb = _solve(vk_lib, gpu, A, M, b, True, restart=20)
        assert ia == ib == 0 and sa.band == 1
        assert np.array_equal(xa, xb) and sa.inner_iters == sb.inner_iters, opt
        assert abs(sa.inner_iters - sr.inner_iters) <= 1, opt
        assert np.linalg.norm(xa - xr) / np.linalg.norm(xr) < 1e-9, opt
        for extra in (4, 8, 12):
            with gpu.tuning(band_opt=opt | extra):
                xc, ic, sc = _solve(vk_lib, gpu, A, M, b, True, restart=20)
            assert ic == 0 and np.array_equal(xc, xa) and sc.inner_iters == sa.inner_iters, (opt, extra)
        # bit 4: odd line ranges walk backwards (their dots sum the lines in reverse order): the
        # DCGS2 bars against the reference, bit-identical from run to run
        with gpu.tuning(band_opt=opt | 28):
            xd, idd, sd = _solve(vk_lib, gpu, A, M, b, True, restart=20)
            xe, _, se = _solve(vk_lib, gpu, A, M, b, True, restart=20)
        assert idd == 0 and sd.band == 1 and np.array_equal(xd, xe) and sd.inner_iters == se.inner_iters, opt
        assert abs(sd.inner_iters - sr.inner_iters) <= 1, opt
        assert np.linalg.norm(xd - xr) / np.linalg.norm(xr) < 1e-9, opt
