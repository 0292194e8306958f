"""x0 handling (iterative.py:737 `r = b - matvec(x) if x.any() else b.copy()`): a zero x0 skips
the first residual SpMV (r = b, psolve(r) = the M b already formed for ||M b||); any nonzero
entry - even one subnormal - takes the SpMV.  Both preconditioner paths (fused BJ residual,
unfused line apply) and both orthogonalisations."""
import numpy as np
import pytest

from oracle import coracle, twin

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("prec", ["bj", "line", "none"])
@pytest.mark.parametrize("orth", ["mgs", "dcgs2"])
def test_zero_and_tiny_x0(gpu, vk_lib, prec, orth):
    vk = vk_lib
    p = twin.CONFIGS["S2"]
    A = vk.vlasov_operator(vk.vlasov_params(p.dim, p.shape), ctx=gpu)
    M = {"bj": lambda: vk.block_jacobi(A, 8), "line": lambda: vk.line_jacobi(A, p.shape[1], 25),
         "none": lambda: None}[prec]()
    b = twin.rhs(p.n)
    x_none, i0 = vk.gmres(A, b, rtol=1e-8, M=M, orth=orth)
    x_zero, i1 = vk.gmres(A, b, x0=np.zeros(p.n), rtol=1e-8, M=M, orth=orth)
    assert i0 == i1 == 0
    assert np.array_equal(x_none, x_zero)
    x0 = np.zeros(p.n)
    x0[123] = 5e-324                      # nonzero: x.any() is True, the SpMV path
    x_tiny, i2 = vk.gmres(A, b, x0=x0, rtol=1e-8, M=M, orth=orth)
    assert i2 == 0
    ip, ix, d = coracle.generate(p)
    assert np.linalg.norm(b - coracle.spmv(ip, ix, d, x_tiny)) <= 1e-8 * np.linalg.norm(b)
    assert np.linalg.norm(x_tiny - x_none) <= 1e-9 * np.linalg.norm(x_none)
