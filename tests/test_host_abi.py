"""libvtkrylov.so on the CPU: it loads, exports every symbol include/vtkrylov.h declares, its
host-only entry points (operator assembly, RHS, partition, halo plan) agree with the oracle,
and the device entry points fail loudly (no CPU fallback) when no GPU is visible."""
import hashlib
import os
import re

import numpy as np
import pytest

from oracle import coracle, twin

HEADER = os.path.join(os.path.dirname(__file__), "..", "include", "vtkrylov.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vtk_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol(vk_lib):
    import ctypes
    names = declared_functions()
    assert len(names) >= 25
    L = ctypes.CDLL(vk_lib._abi.LIB_PATH)
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(vk_lib._abi.PROTOTYPES), set(names) ^ set(vk_lib._abi.PROTOTYPES)
    assert vk_lib._abi.lib().vtk_abi_version() == vk_lib._abi.ABI_VERSION == 6


def test_status_strings(vk_lib):
    L = vk_lib._abi.lib()
    for s in range(0, -9, -1):
        assert L.vtk_status_string(s).decode() != "unknown status"


def test_no_cpu_fallback_without_gpu(vk_lib):
    if vk_lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(vk_lib._abi.VtkError) as e:
        vk_lib.Context(0)
    assert e.value.status == vk_lib._abi.ERR_NODEVICE
    # the SciPy-compatible entry rejects what it cannot run on the GPU before touching it
    from scipy.sparse.linalg import LinearOperator
    with pytest.raises(TypeError):
        vk_lib.gmres(None, np.ones(4), M=LinearOperator((4, 4), matvec=lambda v: v))
    with pytest.raises(NotImplementedError):
        vk_lib.gmres(None, np.ones(4), callback=lambda r: None)


@pytest.mark.parametrize("name", ["C0", "S2", "S4", "S4F"])
def test_host_generator_equals_oracle(vk_lib, name):
    p = twin.CONFIGS[name]
    params = vk_lib.vlasov_params(p.dim, p.shape, fp32=p.fp32)
    a = vk_lib.vlasov_generate_host(params)
    b = coracle.generate(p)
    for x, y in zip(a, b):
        assert x.dtype == y.dtype and np.array_equal(x.view(np.uint8), y.view(np.uint8))
    # row blocks (what each rank assembles) concatenate to the whole operator
    n = p.n
    cut = n // 3
    ip1, ix1, d1 = vk_lib.vlasov_generate_host(params, 0, cut)
    ip2, ix2, d2 = vk_lib.vlasov_generate_host(params, cut, n)
    assert np.array_equal(np.concatenate([ix1, ix2]), b[1])
    assert np.array_equal(np.concatenate([ip1[:-1], ip2 + ip1[-1]]), b[0])


@pytest.mark.parametrize("name", ["C1", "C2", "C3", pytest.param("C4", marks=pytest.mark.slow)])
def test_host_generator_hash_matches_golden(vk_lib, golden_large, name):
    if name not in golden_large:
        pytest.skip(f"{name} hash not generated")
    p = twin.CONFIGS[name]
    ip, ix, d = vk_lib.vlasov_generate_host(vk_lib.vlasov_params(p.dim, p.shape, fp32=p.fp32))
    ref = golden_large[name]["sha256"]
    assert int(ip[-1]) == ref["nnz"]
    assert hashlib.sha256(ip.tobytes()).hexdigest() == ref["indptr"]
    assert hashlib.sha256(ix.tobytes()).hexdigest() == ref["indices"]
    assert hashlib.sha256(d.tobytes()).hexdigest() == ref["data"]


def test_rhs_equals_oracle(vk_lib):
    assert np.array_equal(vk_lib.rhs_splitmix(50_000), coracle.rhs(50_000))
    assert np.array_equal(vk_lib.rhs_splitmix(50_000, r0=1234, r1=5678), coracle.rhs(50_000, r0=1234, r1=5678))


def test_invalid_parameters_raise(vk_lib):
    with pytest.raises(ValueError):
        vk_lib.vlasov_generate_host(vk_lib.vlasov_params(2, (2, 8)))   # Nx < 3: duplicate columns
    with pytest.raises(ValueError):
        vk_lib.vlasov_generate_host(vk_lib.vlasov_params(3, (4, 4, 4)))


@pytest.mark.parametrize("world,align", [(1, 1), (2, 8), (3, 800), (8, 800), (7, 8)])
def test_partition_rows(vk_lib, world, align):
    n = twin.CONFIGS["C1"].n
    offs = vk_lib.partition_rows(n, world, align)
    assert offs[0] == 0 and offs[-1] == n and np.all(np.diff(offs) >= 0)
    assert np.all(offs[1:-1] % align == 0)
    sizes = np.diff(offs)
    assert sizes.max() - sizes.min() <= 2 * align
    # nnz-balanced variant
    ip2, _, _ = coracle.generate(twin.CONFIGS["S2"])
    offs2 = vk_lib.partition_rows(ip2.shape[0] - 1, world, min(align, 32), indptr=ip2)
    assert offs2[0] == 0 and offs2[-1] == ip2.shape[0] - 1 and np.all(np.diff(offs2) >= 0)


def _halo_ref(n, offs, rank, ix):
    rb, re_ = offs[rank], offs[rank + 1]
    ext = np.unique(ix[(ix < rb) | (ix >= re_)].astype(np.int64))
    loc = np.where((ix >= rb) & (ix < re_), ix - rb, (re_ - rb) + np.searchsorted(ext, ix))
    cnt = np.array([np.count_nonzero((ext >= offs[q]) & (ext < offs[q + 1])) for q in range(len(offs) - 1)])
    return loc, ext, cnt


@pytest.mark.parametrize("name,world", [("S2", 2), ("S2", 4), ("S4", 3), ("C0", 5)])
def test_halo_plan_matches_reference(vk_lib, name, world):
    p = twin.CONFIGS[name]
    ip, ix, d = coracle.generate(p)
    offs = vk_lib.partition_rows(p.n, world, p.shape[-1] if p.dim == 2 else 8)
    x = twin.rhs(p.n, seed=3)
    y = coracle.spmv(ip, ix, d, x)
    for rank in range(world):
        rb, re_ = offs[rank], offs[rank + 1]
        lip = ip[rb:re_ + 1] - ip[rb]
        lix = ix[ip[rb]:ip[re_]]
        loc, cols, cnt = vk_lib.halo_plan(p.n, offs, rank, lix)
        rloc, rcols, rcnt = _halo_ref(p.n, offs, rank, lix)
        assert np.array_equal(loc, rloc) and np.array_equal(cols, rcols) and np.array_equal(cnt, rcnt)
        assert cnt[rank] == 0
        # local SpMV on [x_local | halo] reproduces the global rows bit for bit
        xe = np.concatenate([x[rb:re_], x[cols]])
        yl = coracle.spmv(lip.astype(np.int32), loc.astype(np.int32), d[ip[rb]:ip[re_]], xe)
        assert np.array_equal(yl, y[rb:re_])


def test_library_is_current():
    """The in-tree libvtkrylov.so travels to the GPU box as built here: it must not be older
    than any of its sources (rebuild with `make -C vt-precondition_amd/csrc`)."""
    import glob
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = os.path.join(root, "vt-precondition_amd", "vtkrylov", "lib", "libvtkrylov.so")
    if not os.path.exists(so):
        import pytest
        pytest.skip("library not built yet")
    srcs = glob.glob(os.path.join(root, "vt-precondition_amd", "csrc", "*.[hc]*")) + \
        [os.path.join(root, "include", "vtkrylov.h")]
    stale = [s for s in srcs if os.path.getmtime(s) > os.path.getmtime(so)]
    assert not stale, f"libvtkrylov.so is older than {stale}"


def test_build_id_matches_sources(vk_lib):
    """vtk_build_id() is the SHA-256 of the sources the library was built from (csrc/Makefile);
    _abi.source_build_id() recomputes it over the checked-out tree: equal for a current build."""
    bid = vk_lib._abi.build_id()
    assert re.fullmatch(r"[0-9a-f]{16}", bid)
    assert bid == vk_lib._abi.source_build_id()
    assert vk_lib._abi.check_build_id() == bid


def test_build_id_mismatch_is_refused(vk_lib, tmp_path, monkeypatch):
    """A library built from other sources (the GPU box runs the binary pushed with the tree) is
    refused: one changed byte in any source changes the id, and check_build_id raises."""
    import shutil
    src = os.path.join(os.path.dirname(vk_lib._abi.CSRC), "csrc")
    d = tmp_path / "csrc"
    shutil.copytree(src, d, ignore=shutil.ignore_patterns("build"))
    hdr = tmp_path / "vtkrylov.h"
    shutil.copy(vk_lib._abi.HEADER, hdr)
    same = vk_lib._abi.source_build_id(str(d), str(hdr))
    assert same == vk_lib._abi.build_id()
    with open(d / "vtk_band.hip", "ab") as f:
        f.write(b"\n// edited\n")
    other = vk_lib._abi.source_build_id(str(d), str(hdr))
    assert other != same
    monkeypatch.delenv("VTK_LIB", raising=False)
    with pytest.raises(vk_lib._abi.StaleBuildError):
        vk_lib._abi.check_build_id(sources=other)
    # EXTRA build flags are part of the id too
    assert vk_lib._abi.source_build_id(str(d), str(hdr), extra="-DX=1") != other


def test_tuning_keys_without_gpu(vk_lib):
    """vtk_ctx_set_tuning / get_tuning need a context (no GPU here): NULL context -> VTK_ERR_ARG."""
    import ctypes
    L = vk_lib._abi.lib()
    v = ctypes.c_int()
    assert L.vtk_ctx_set_tuning(None, b"band", 0) == vk_lib._abi.ERR_ARG
    assert L.vtk_ctx_get_tuning(None, b"band", ctypes.byref(v)) == vk_lib._abi.ERR_ARG


@pytest.mark.slow
def test_host_code_under_asan_ubsan():
    """tools/asan_host.sh: the host routines under AddressSanitizer + UBSan (CPU only)."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["bash", os.path.join(root, "tools", "asan_host.sh")], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0 and "asan_host: ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


def _band_plan(vk_lib, n, L, ncu=256):
    import ctypes
    g = vk_lib._abi.BandGeometry()
    st = vk_lib._abi.lib().vtk_line_band_plan(n, L, ncu, ctypes.byref(g))
    return st, g


def test_line_band_plan_geometry(vk_lib):
    """The band step's geometry (vtk_line_band_plan, ABI 3): C3 = 25 000 lines of 800 rows ->
    two 400-row parts per line, one 7-wave workgroup per part, two workgroups per CU."""
    st, g = _band_plan(vk_lib, 20_000_000, 800)
    assert st == vk_lib._abi.OK
    assert (g.parts, g.wg_per_range, g.waves_per_wg, g.ranges, g.lines) == (2, 2, 7, 256, 25_000)
    st, g = _band_plan(vk_lib, 64 * 32, 32)   # S2: one part per line; 32 ranges of 2 lines
    assert st == vk_lib._abi.OK and (g.parts, g.ranges) == (1, 32)
    st, g = _band_plan(vk_lib, 24 * 1000, 1000)   # five 200-row parts; X / 2 = 12 ranges
    assert st == vk_lib._abi.OK and (g.parts, g.ranges) == (5, 12)


@pytest.mark.parametrize("n,L", [(2**31, 1024), (2**30 + 2**20, 1024), (800 * 7 + 8, 800), (800, 800), (1000, 100),
                                 (0, 8), (24 * 404, 404)])
def test_line_band_plan_rejects(vk_lib, n, L):
    """32-bit index guard (slabs whose rows + halo reach 2^30), partial lines, one line, line
    lengths not a multiple of 8, no equal split into 8-row-multiple parts of <= 400 rows:
    VTK_ERR_ARG with a message, no GPU needed."""
    st, _ = _band_plan(vk_lib, n, L)
    assert st == vk_lib._abi.ERR_ARG
    assert vk_lib._abi.last_error()


def test_header_lists_every_tuning_key():
    """include/vtkrylov.h documents the tuning keys vtk_ctx_set_tuning accepts: the list there is
    the library's table (vtk_api.cpp TUNE_KEYS), no more and no fewer."""
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hdr = open(os.path.join(root, "include", "vtkrylov.h")).read()
    m = re.search(r"Keys:(.*?)\.\s*\n\s*\* VTK_ERR_ARG for an unknown key", hdr, re.S)
    assert m, "key list not found in the header"
    listed = {k.strip() for k in m.group(1).replace("*", " ").replace("\n", " ").split(",")}
    src = open(os.path.join(root, "vt-precondition_amd", "csrc", "vtk_api.cpp")).read()
    table = set(re.findall(r'\{"([a-z0-9_]+)", &Tuning::', src))
    assert listed == table, (sorted(listed - table), sorted(table - listed))
