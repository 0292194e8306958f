"""bench.py's roofline.traffic gate (CPU): PMC HBM bytes are reported only from a committed
profiles/rNN[_tag]_pmc_traffic.json of the same config AND the same device sources (bench.KERNEL_SOURCES)
(a summary of other kernels must never be reported as this run's traffic)."""
import hashlib
import json
import os

import bench


def _tree(tmp_path, src=b"// kernels v1\n"):
    d = tmp_path / "vt-precondition_amd" / "csrc"
    d.mkdir(parents=True)
    h = hashlib.sha256()
    for i, name in enumerate(bench.KERNEL_SOURCES):   # every device source is hashed, in order
        body = src + bytes(f"// {i}\n", "ascii")
        (d / name).write_bytes(body)
        h.update(body)
    (tmp_path / "profiles").mkdir()
    return h.hexdigest()[:16]


def _summary(tmp_path, name, config, sha, bytes_per_launch):
    rec = {"config": config, "kernels_sha16": sha,
           "kernels": {"band_step": {"hbm_bytes_per_launch": bytes_per_launch}}}
    (tmp_path / "profiles" / name).write_text(json.dumps(rec))


def test_traffic_from_matching_summary(tmp_path, monkeypatch):
    sha = _tree(tmp_path)
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.kernels_sha16() == sha
    _summary(tmp_path, "r02_c3_pmc_traffic.json", "C3", sha, 3.1e9)
    _summary(tmp_path, "r02_c4_pmc_traffic.json", "C4", sha, 7.0e9)
    t, src = bench.pmc_traffic("band_step", "C3", 1)
    assert t == 3.1e9 and src.startswith("r02_c3_pmc_traffic.json")
    t, _ = bench.pmc_traffic("band_step", "C4", 1)
    assert t == 7.0e9


def test_traffic_stale_source_is_null(tmp_path, monkeypatch):
    _tree(tmp_path)
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    _summary(tmp_path, "r02_c3_pmc_traffic.json", "C3", "0123456789abcdef", 3.1e9)
    t, why = bench.pmc_traffic("band_step", "C3", 1)
    assert t is None and "other kernel sources" in why


def test_traffic_newest_matching_wins_and_missing_class(tmp_path, monkeypatch):
    sha = _tree(tmp_path)
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    _summary(tmp_path, "r01_c3_pmc_traffic.json", "C3", sha, 1.0e9)
    _summary(tmp_path, "r02_c3_pmc_traffic.json", "C3", sha, 2.0e9)
    assert bench.pmc_traffic("band_step", "C3", 1)[0] == 2.0e9
    t, why = bench.pmc_traffic("spmv", "C3", 1)
    assert t is None and "no C3 PMC summary" in why


def test_traffic_multi_gpu_and_other_config(tmp_path, monkeypatch):
    sha = _tree(tmp_path)
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    _summary(tmp_path, "r02_c3_pmc_traffic.json", "C3", sha, 3.1e9)
    assert bench.pmc_traffic("band_step", "C3", 2)[0] is None
    t, why = bench.pmc_traffic("band_step", "C2", 1)
    assert t is None and "no C2" in why
    assert os.path.exists(tmp_path / "profiles" / "r02_c3_pmc_traffic.json")
