import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
PKG = os.path.join(ROOT, "vt-precondition_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libvtkrylov.so")
    config.addinivalue_line("markers", "slow: long-running (large configs)")


def pytest_sessionstart(session):
    # the CPU oracle is test infrastructure: (re)build it when missing or older than its
    # sources (make, gcc: seconds)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


@pytest.fixture(scope="session")
def golden():
    with np.load(os.path.join(GOLDEN, "golden_small.npz"), allow_pickle=False) as g:
        return {k: g[k] for k in g.files}


@pytest.fixture(scope="session")
def golden_line():
    with np.load(os.path.join(GOLDEN, "golden_line.npz"), allow_pickle=False) as g:
        return {k: g[k] for k in g.files}


@pytest.fixture(scope="session")
def golden_large():
    with open(os.path.join(GOLDEN, "golden_large.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def vk_lib():
    lib = os.path.join(PKG, "vtkrylov", "lib", "libvtkrylov.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(PKG, "csrc")], check=True)
    import vtkrylov
    vtkrylov._abi.lib()
    # the GPU box runs the prebuilt library pushed with the tree: it must be built from these
    # sources (vtk_build_id), else every result below would describe other code
    vtkrylov._abi.check_build_id()
    return vtkrylov


@pytest.fixture(scope="session")
def gpu(vk_lib):
    if vk_lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return vk_lib.default_context(0)
