"""vtsetup entry for the preconditioned-Krylov path.

Mirrors the reference's step-object convention — a class whose ``main()`` runs a fixed
sequence (hypervisor.py:589-594: deploy -> network -> tools -> vms -> env) — with the
solver's sequence: generate operator -> set up preconditioner -> solve -> report.  Errors
surface as exceptions that ``test_main`` turns into a return code, as in
vt_precondition.py:66-79.

    python -m vtsetup.krylov_precondition [--config C1] [--xml path] [--report out.json]
                                          [--operator-file matrix.npz]
"""
from __future__ import annotations

import argparse
import json
import sys
import time


class KrylovPrecondition:
    def __init__(self, cfg, ctx=None):
        self.cfg = cfg
        self.ctx = ctx
        self.A = self.M = self.b = self.x = None
        self.result = {}

    def generate_operator(self):
        """The config's Vlasov operator assembled on the device, or the SciPy archive named by
        operator/file (vtkrylov.load_npz)."""
        import vtkrylov as vk
        c = self.cfg
        self.ctx = self.ctx or vk.Context(c.device)
        t = time.perf_counter()
        if c.operator_file:
            # the x-line structure of a 2D Vlasov archive is found by the library (line_len None)
            # and runs the fused band step, as a generated operator does; operator/line_len
            # requires (L) or refuses (0) it
            self.A = vk.load_npz(c.operator_file, ctx=self.ctx, line_len=c.line_len)
        else:
            p = vk.vlasov_params(c.dim, c.shape, fp32=c.fp32, **c.physics)
            self.A = vk.vlasov_operator(p, ctx=self.ctx)
            if c.line_len is not None and c.line_len != self.A.line_band:
                self.A.set_line_band(c.line_len)
        self.result["operator"] = {"n": self.A.n_global, "nnz": self.A.nnz,
                                   "source": c.operator_file or f"vlasov {c.config}",
                                   "line_band": self.A.line_band, "line_values": self.A.line_values,
                                   "t_assemble_s": time.perf_counter() - t}

    def setup_preconditioner(self):
        import vtkrylov as vk
        t = time.perf_counter()
        c = self.cfg
        info = {"type": c.preconditioner}
        if c.preconditioner == "block_jacobi":
            self.M = vk.block_jacobi(self.A, c.block_size)
            info["block_size"] = c.block_size
        elif c.preconditioner == "line_jacobi":
            stride = c.line_stride
            if stride <= 0:
                if c.operator_file:
                    # the detected x-line length is the line stride of a 2D operator
                    stride = self.A.line_band
                    if stride <= 0:
                        raise ValueError("line_jacobi on an operator file without a detected x-line "
                                         "structure needs preconditioner/line_stride")
                else:
                    stride = vk.vlasov_line_stride(vk.vlasov_params(c.dim, c.shape))
            self.M = vk.line_jacobi(self.A, stride, c.line_segment)
            info.update(line_stride=stride, line_segment=c.line_segment)
        info["t_setup_s"] = time.perf_counter() - t
        self.result["preconditioner"] = info

    def solve(self):
        import vtkrylov as vk
        c = self.cfg
        self.b = vk.rhs_splitmix(self.A.n_global, seed=c.seed)
        self.x, info = vk.gmres(self.A, self.b, rtol=c.rtol, atol=c.atol, restart=c.restart,
                                maxiter=c.maxiter or None, M=self.M, orth=c.orth)
        st = vk.last_stats()
        self.result["solve"] = {"info": info, "inner_iters": st.inner_iters,
                                "restarts": st.restarts, "rnorm": st.rnorm, "bnorm": st.bnorm,
                                "t_solve_s": st.t_solve, "band_step": bool(st.band),
                                "iters_per_s": st.inner_iters / st.t_solve if st.t_solve else None}

    def report(self):
        self.result["config"] = self.cfg.config
        if self.cfg.report:
            with open(self.cfg.report, "w") as f:
                json.dump(self.result, f, indent=1)
        return self.result

    def main(self):
        self.generate_operator()
        self.setup_preconditioner()
        self.solve()
        return self.report()


def test_main(argv=None) -> int:
    from .config import DEFAULT_XML, SolverConfig
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--xml", default=DEFAULT_XML)
    ap.add_argument("--config")
    ap.add_argument("--report")
    ap.add_argument("--operator-file", help="SciPy save_npz CSR archive to solve")
    ap.add_argument("--preconditioner", choices=["block_jacobi", "line_jacobi", "none"])
    a = ap.parse_args(argv)
    try:
        cfg = SolverConfig.load(a.xml, config=a.config, report=a.report, operator_file=a.operator_file,
                                 preconditioner=a.preconditioner)
        res = KrylovPrecondition(cfg).main()
        print(json.dumps(res))
        return 0 if res["solve"]["info"] == 0 else 1
    except Exception as e:   # vt_precondition.py:70-71 style: report and fail
        print(f"vtsetup.krylov_precondition failed: {type(e).__name__}: {e}", file=sys.stderr)
        return 2


if __name__ == "__main__":
    sys.exit(test_main())
