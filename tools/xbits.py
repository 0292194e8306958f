"""Bit-identity probe for A/B builds (GPU): solves a few systems and prints, per case, the
inner-iteration count, info and the SHA-256 of x's bytes.  Run it once per library
(VTK_LIB=<other build>) and diff the outputs: a change meant to keep the arithmetic must print
the same lines.

    python tools/xbits.py > a.txt; VTK_LIB=tools/bin/lib_x/libvtkrylov.so python tools/xbits.py > b.txt
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vt-precondition_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import vtkrylov as vk  # noqa: E402
from oracle import twin  # noqa: E402


def main():
    for shape in ((64, 32), (1250, 800)):
        n = shape[0] * shape[1]
        A = vk.vlasov_operator(vk.vlasov_params(2, shape))
        b = twin.rhs(n)
        M = vk.block_jacobi(A, 8)
        for restart in (2, 5, 20):
            for orth in ("dcgs2", "mgs"):
                for rtol in (1e-8, 1e-12):
                    x, info = vk.gmres(A, b, rtol=rtol, M=M, restart=restart, orth=orth, maxiter=400)
                    st = vk.last_stats()
                    h = hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()[:16]
                    print(f"{shape} restart={restart} {orth} rtol={rtol:g}: info={info} "
                          f"inner={st.inner_iters} x={h}", flush=True)
        Lj = vk.line_jacobi(A, shape[1], 25)
        x, info = vk.gmres(A, b, rtol=1e-8, M=Lj)
        h = hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()[:16]
        print(f"{shape} line: info={info} inner={vk.last_stats().inner_iters} x={h}", flush=True)


if __name__ == "__main__":
    main()
