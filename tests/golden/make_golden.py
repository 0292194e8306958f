"""Generate the committed golden fixtures from SciPy 1.15.3 / NumPy 2.2.6 (the north_star's
"reference scipy.sparse path"; /root/reference itself has no numerical code).

    python tests/golden/make_golden.py            # small fixtures + C1/C2/C3 summaries
    python tests/golden/make_golden.py --c4       # also hash the 445.5M-nnz C4 operator

Outputs (all data, no code):
  golden_small.npz  — vectors for C0, S2, S4, S4F, a ragged random CSR, GMRES edge cases
  golden_large.json — SHA-256 of the C1..C4 CSR byte streams, ||A·1||, SciPy GMRES summary
  golden_line.npz   — line-Jacobi solves (SciPy splu of M) and SciPy GMRES with it (--line-only,
                      which also adds the C1 line-GMRES summary to golden_large.json)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))

from oracle import twin  # noqa: E402

X_SEED = 0xC0FFEE


def ragged_csr(seed=1234, n=3000):
    """Random CSR with empty rows, one very long row and one dense-ish band; canonical."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 12, size=n)
    lens[rng.choice(n, 50, replace=False)] = 0          # empty rows
    lens[7] = 2500                                       # one wave-per-row candidate
    lens[1500] = 700
    rows = np.repeat(np.arange(n), lens)
    cols = np.concatenate([rng.choice(n, size=l, replace=False) for l in lens])
    vals = rng.standard_normal(rows.shape[0])
    A = sp.csr_matrix((vals, (rows, cols)), shape=(n, n))
    A.sum_duplicates()
    A.sort_indices()
    # make it comfortably non-singular (diagonal dominance) for BJ/GMRES on it
    A = A + sp.diags(np.abs(A).sum(axis=1).A1 + 1.0)
    A = sp.csr_matrix(A)
    A.sort_indices()
    return A


def small(out):
    import scipy.sparse as sp  # noqa: F401
    g = {}
    for name in ["C0", "S2", "S4", "S4F"]:
        p = twin.CONFIGS[name]
        ip, ix, d = twin.generate(p)
        A = twin.scipy_csr(ip, ix, d, p.n)
        x = twin.rhs(p.n, seed=X_SEED)
        b = twin.rhs(p.n)
        g[f"{name}/spmv_y"] = A @ x
        g[f"{name}/ones_y"] = A @ np.ones(p.n)
        inv = twin.bj_inverse_numpy(ip, ix, d, p.n, 8)
        g[f"{name}/bj8_z"] = twin.bj_apply_numpy(inv, b, p.n)
        if name != "C0":
            g[f"{name}/bj8_inv"] = inv
        s = twin.scipy_gmres(A, b, inv, rtol=1e-8)
        g[f"{name}/gmres_x"] = s.x
        g[f"{name}/gmres_meta"] = np.array([s.info, s.inner_iters, s.true_resid, s.b_norm])
        print(name, "info", s.info, "inner", s.inner_iters, "res", s.true_resid / s.b_norm)
    # GMRES edge cases on S2 / C0
    p = twin.CONFIGS["S2"]
    ip, ix, d = twin.generate(p)
    A = twin.scipy_csr(ip, ix, d, p.n)
    b = twin.rhs(p.n)
    inv = twin.bj_inverse_numpy(ip, ix, d, p.n, 8)
    from scipy.sparse.linalg import gmres

    def case(key, **kw):
        M = kw.pop("M", None)
        bb = kw.pop("b", b)
        AA = kw.pop("A", A)
        count = [0]
        x, info = gmres(AA, bb, M=M, callback=lambda _: count.__setitem__(0, count[0] + 1),
                        callback_type="pr_norm", **kw)
        g[f"edge/{key}/x"] = x
        g[f"edge/{key}/meta"] = np.array([info, count[0], np.linalg.norm(bb - AA @ x),
                                          np.linalg.norm(bb)])
        print("edge", key, info, count[0])

    Mbj = twin.bj_operator(inv, p.n)
    case("noprec", rtol=1e-8)
    x0 = 0.1 * twin.rhs(p.n, seed=7)
    g["edge/x0/x0"] = x0
    case("x0", M=Mbj, x0=x0, rtol=1e-10)
    case("restart5_maxiter3", M=Mbj, rtol=1e-12, restart=5, maxiter=3)
    case("bzero", M=Mbj, b=np.zeros(p.n), rtol=1e-8)
    case("atol", M=Mbj, rtol=0.0, atol=1e-3)
    case("restart40", M=Mbj, rtol=1e-9, restart=40)
    # ragged random CSR: SpMV and BJ(4) only (general-CSR path: empty rows, long rows)
    R = ragged_csr()
    g["ragged/indptr"] = R.indptr.astype(np.int32)
    g["ragged/indices"] = R.indices.astype(np.int32)
    g["ragged/data"] = R.data
    xr = twin.rhs(R.shape[0], seed=X_SEED)
    g["ragged/spmv_y"] = R @ xr
    invr = twin.bj_inverse_numpy(R.indptr, R.indices, R.data, R.shape[0], 4)
    g["ragged/bj4_z"] = twin.bj_apply_numpy(invr, twin.rhs(R.shape[0]), R.shape[0])
    # partial last block: n not divisible by bs (n = 3000, bs = 7)
    invr7 = twin.bj_inverse_numpy(R.indptr, R.indices, R.data, R.shape[0], 7)
    g["ragged/bj7_z"] = twin.bj_apply_numpy(invr7, twin.rhs(R.shape[0]), R.shape[0])
    Mr = twin.bj_operator(invr, R.shape[0])
    case_b = twin.rhs(R.shape[0])
    count = [0]
    xr_s, info = gmres(R, case_b, M=Mr, rtol=1e-10, callback=lambda _: count.__setitem__(0, count[0] + 1),
                       callback_type="pr_norm")
    g["ragged/gmres_x"] = xr_s
    g["ragged/gmres_meta"] = np.array([info, count[0], np.linalg.norm(case_b - R @ xr_s),
                                       np.linalg.norm(case_b)])
    np.savez_compressed(out, **g)
    print("wrote", out, os.path.getsize(out), "bytes")


LINE_SEG = 25   # x-points per line segment (divides Nx / 8 of C1..C4)


def line_stride(p) -> int:
    """Rows between x-neighbours: 1 (1D), Nv (2D), Ny*Nvx*Nvy (4D)."""
    return 1 if p.dim == 1 else (p.shape[1] if p.dim == 2 else p.n // p.shape[0])


def line(out, out_json):
    """Line-Jacobi fixtures: SciPy splu solves with M and SciPy GMRES with
    that LinearOperator, on the small configs, a ragged random CSR and C1 (summary)."""
    g = {}
    cases = [(name, twin.CONFIGS[name]) for name in ["C0", "S2", "S4", "S4F"]]
    for name, p in cases:
        ip, ix, d = twin.generate(p)
        A = twin.scipy_csr(ip, ix, d, p.n)
        b = twin.rhs(p.n)
        st = line_stride(p)
        for seg in (3, LINE_SEG):
            M = twin.line_operator(ip, ix, d, p.n, st, seg)
            g[f"{name}/line{seg}_z"] = M.matvec(b)
        s = twin.scipy_gmres(A, b, twin.line_operator(ip, ix, d, p.n, st, LINE_SEG), rtol=1e-8)
        g[f"{name}/gmres_line_x"] = s.x
        g[f"{name}/gmres_line_meta"] = np.array([s.info, s.inner_iters, s.true_resid, s.b_norm])
        print(name, "line gmres info", s.info, "inner", s.inner_iters)
    R = ragged_csr()
    n = R.shape[0]
    M = twin.line_operator(R.indptr, R.indices, R.data, n, 37, 5)
    g["ragged/line37_5_z"] = M.matvec(twin.rhs(n))
    # non-canonical rows: duplicates and unsorted columns add up as toarray() does
    np.savez_compressed(out, **g)
    print("wrote", out, os.path.getsize(out), "bytes")
    with open(out_json) as f:
        res = json.load(f)
    p = twin.CONFIGS["C1"]
    ip, ix, d = twin.generate(p)
    A = twin.scipy_csr(ip, ix, d, p.n)
    b = twin.rhs(p.n)
    s = twin.scipy_gmres(A, b, twin.line_operator(ip, ix, d, p.n, line_stride(p), LINE_SEG), rtol=1e-8)
    print("C1 line gmres", s.info, s.inner_iters)
    res["C1"][f"gmres_line{LINE_SEG}"] = {
        "rtol": 1e-8, "restart": 20, "stride": line_stride(p), "seg": LINE_SEG, "info": s.info,
        "inner_iters": s.inner_iters, "x_norm2": float(np.linalg.norm(s.x)),
        "true_resid": s.true_resid, "b_norm2": s.b_norm, "x_first8": s.x[:8].tolist()}
    with open(out_json, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print("wrote", out_json)


def large(out, with_c4):
    res = {}
    if os.path.exists(out):
        with open(out) as f:
            res = json.load(f)
    res["_provenance"] = ("SciPy 1.15.3 / NumPy 2.2.6 in the build container; operator = "
                          "oracle/twin.py (SURVEY.md Appendix A); script tests/golden/make_golden.py")
    names = ["C1", "C2", "C3"] + (["C4"] if with_c4 else [])
    for name in names:
        p = twin.CONFIGS[name]
        t = time.time()
        h = twin.csr_sha256(p)
        h["n"] = p.n
        assert h["nnz"] == p.nnz
        print(name, "hash", time.time() - t, "s")
        res.setdefault(name, {}).update({"sha256": h})
    # C1: ||A 1||, SpMV of the x-seed vector (norm + checksum), SciPy GMRES+BJ(8) summary
    p = twin.CONFIGS["C1"]
    ip, ix, d = twin.generate(p)
    A = twin.scipy_csr(ip, ix, d, p.n)
    b = twin.rhs(p.n)
    x = twin.rhs(p.n, seed=X_SEED)
    y = A @ x
    inv = twin.bj_inverse_numpy(ip, ix, d, p.n, 8)
    t = time.time()
    s = twin.scipy_gmres(A, b, inv, rtol=1e-8)
    print("C1 gmres", time.time() - t, s.info, s.inner_iters)
    res["C1"].update({
        "A_ones_norm2": float(np.linalg.norm(A @ np.ones(p.n))),
        "spmv_y_norm2": float(np.linalg.norm(y)),
        "spmv_y_sha256": __import__("hashlib").sha256(y.tobytes()).hexdigest(),
        "gmres_bj8": {"rtol": 1e-8, "restart": 20, "info": s.info, "inner_iters": s.inner_iters,
                      "x_norm2": float(np.linalg.norm(s.x)), "true_resid": s.true_resid,
                      "b_norm2": s.b_norm, "x_first8": s.x[:8].tolist()},
    })
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print("wrote", out)


def solve_summary(s_x, info, inner, true_resid, b_norm, **extra):
    """What a full-size GPU parity test compares (tests/test_gpu_large.py): info, inner
    iterations, ||x||, the first/last 8 entries and 64 entries sampled at a fixed stride."""
    n = s_x.shape[0]
    stride = max(1, n // 64)
    return {"rtol": 1e-8, "restart": 20, "info": int(info), "inner_iters": int(inner),
            "x_norm2": float(np.linalg.norm(s_x)), "true_resid": float(true_resid), "b_norm2": float(b_norm),
            "x_first8": s_x[:8].tolist(), "x_last8": s_x[-8:].tolist(),
            "x_sample_stride": stride, "x_sample": s_x[::stride][:64].tolist(), **extra}


def bj_inverse_numpy_chunked(ip, ix, d, n, bs, rows_per_chunk=1 << 22):
    """twin.bj_inverse_numpy over row chunks (the 50M-row C4 operator: bounded memory).  Same
    blocks, same numpy.linalg.inv per block: identical bits to the one-shot form."""
    nb = (n + bs - 1) // bs
    out = np.empty((nb, bs, bs))
    step = max(bs, rows_per_chunk // bs * bs)
    for r0 in range(0, n, step):
        r1 = min(n, r0 + step)
        k0, k1 = int(ip[r0]), int(ip[r1])
        sub_ip = (np.asarray(ip[r0:r1 + 1], np.int64) - k0)
        sub_ix = np.asarray(ix[k0:k1], np.int64) - r0   # columns relative to the chunk
        # entries outside the chunk's rows are never in a diagonal block (chunks align to bs)
        keep = (sub_ix >= 0) & (sub_ix < r1 - r0)
        cols = np.where(keep, sub_ix, -(10 ** 9))
        B = twin.bj_blocks(sub_ip, cols, d[k0:k1], r1 - r0, bs)
        out[r0 // bs:(r1 + bs - 1) // bs] = np.linalg.inv(B)
    return out


def gmres_large(out, names):
    """SciPy GMRES(20) + BJ(8) to rtol 1e-8 at the headline sizes (C2, C3: the bench workload;
    C4: 50M rows, fp32 values).  For C4 the fp32 values are widened to f64 once: SciPy's
    csr_matvec on fp32 data and an f64 vector upcasts the values (checked bit-equal), so this
    is the same product without a 3.6 GB copy per SpMV; the operator comes from the C
    generator, which is pinned to twin.py by the SHA-256 in this file."""
    from oracle import coracle
    with open(out) as f:
        res = json.load(f)
    for name in names:
        p = twin.CONFIGS[name]
        t = time.time()
        if name == "C4":
            ip, ix, d32 = coracle.generate(p)
            h = res.get("C4", {}).get("sha256", {})
            if h:
                import hashlib
                assert hashlib.sha256(ix.tobytes()).hexdigest() == h["indices"], "C4 indices differ from the pinned hash"
                assert hashlib.sha256(d32.tobytes()).hexdigest() == h["data"], "C4 data differ from the pinned hash"
            b = twin.rhs(p.n)
            inv = bj_inverse_numpy_chunked(ip, ix, d32, p.n, 8)
            d = d32.astype(np.float64)
            del d32
            A = twin.scipy_csr(ip, ix, d, p.n)
            print("C4 setup", round(time.time() - t, 1), "s", flush=True)
            s = twin.scipy_gmres(A, b, inv, rtol=1e-8)
            summ = solve_summary(s.x, s.info, s.inner_iters, s.true_resid, s.b_norm,
                                 source="scipy.sparse.linalg.gmres, M = BJ(8) LinearOperator (numpy inverses); "
                                        "fp32 values widened to f64 as SciPy's csr_matvec does",
                                 seconds=round(s.seconds, 1))
        else:
            ip, ix, d = twin.generate(p)
            A = twin.scipy_csr(ip, ix, d, p.n)
            b = twin.rhs(p.n)
            inv = twin.bj_inverse_numpy(ip, ix, d, p.n, 8)
            s = twin.scipy_gmres(A, b, inv, rtol=1e-8)
            summ = solve_summary(s.x, s.info, s.inner_iters, s.true_resid, s.b_norm,
                                 source="scipy.sparse.linalg.gmres, M = BJ(8) LinearOperator (numpy inverses)",
                                 seconds=round(s.seconds, 1))
        print(name, "gmres", round(time.time() - t, 1), "s", summ["info"], summ["inner_iters"], flush=True)
        res.setdefault(name, {})["gmres_bj8"] = summ
        with open(out, "w") as f:
            json.dump(res, f, indent=1, sort_keys=True)
    print("wrote", out)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--gmres-large", nargs="+", default=None, metavar="CFG",
                    help="only the full-size GMRES summaries of these configs (C2 C3 C4)")
    ap.add_argument("--c4", action="store_true")
    ap.add_argument("--skip-small", action="store_true")
    ap.add_argument("--line-only", action="store_true", help="only the line-Jacobi fixtures")
    a = ap.parse_args()
    if a.gmres_large:
        gmres_large(os.path.join(HERE, "golden_large.json"), a.gmres_large)
        sys.exit(0)
    if a.line_only:
        line(os.path.join(HERE, "golden_line.npz"), os.path.join(HERE, "golden_large.json"))
        sys.exit(0)
    if not a.skip_small:
        small(os.path.join(HERE, "golden_small.npz"))
    large(os.path.join(HERE, "golden_large.json"), a.c4)
