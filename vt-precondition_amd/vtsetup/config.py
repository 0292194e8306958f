"""vtconfig reader for the Krylov path.

Keeps the reference's two lookup conventions (ini_info.py:72-118) so configuration reads the
same way as the rest of VT-precondition:
    Etree.get_node_value("solver/rtol")      -> stripped text of the first matching node
    Etree.dict_walkData("operator/physics")  -> {child tag: stripped text}
but the file is a parameter (not a hard-coded path) and is parsed once per Etree instance.
``SolverConfig.load(path)`` turns it into typed values.
"""
from __future__ import annotations

import os
import xml.etree.ElementTree as ET
from dataclasses import dataclass

DEFAULT_XML = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                           "vtconfig", "vt_krylov_configuration.xml")


class Etree:
    def __init__(self, path: str = DEFAULT_XML):
        self.path = path
        self.root = ET.parse(path).getroot()

    def _find(self, attrib: str):
        node = self.root.find(f".//{attrib}")
        if node is None:
            raise KeyError(f"{attrib!r} not found in {self.path}")
        return node

    def get_node_value(self, attrib: str) -> str:
        return (self._find(attrib).text or "").strip()

    def dict_walkData(self, attrib: str) -> dict:
        return {n.tag: (n.text or "").strip() for n in self._find(attrib)}

    def get_optional(self, attrib: str, default=None):
        """get_node_value for nodes a configuration may leave out (None / default when absent)."""
        node = self.root.find(f".//{attrib}")
        return default if node is None else (node.text or "").strip()


def parse_config_spec(spec: str):
    """'2:1250x800:f64' -> (dim, shape, fp32)"""
    dim, shape, prec = spec.split(":")
    shape = tuple(int(v) for v in shape.split("x"))
    dim = int(dim)
    if {1: 1, 2: 2, 4: 4}.get(dim) != len(shape):
        raise ValueError(f"config {spec!r}: dim {dim} needs {dim} extents")
    if prec not in ("f64", "f32"):
        raise ValueError(f"config {spec!r}: precision must be f64 or f32")
    return dim, shape, prec == "f32"


@dataclass
class SolverConfig:
    config: str
    dim: int
    shape: tuple
    fp32: bool
    physics: dict
    rtol: float
    atol: float
    restart: int
    maxiter: int
    orth: str
    operator_file: str
    preconditioner: str
    block_size: int
    line_stride: int
    line_segment: int
    seed: int
    device: int
    report: str
    line_len: int | None = None   # operator/line_len: None (absent / "auto") = detected by vtk_csr_create
    gpus: int = 1                 # run/gpus: ranks, one process per GPU (absent: 1)
    comm: str = "rccl"            # run/comm: rccl, or host (host-staged, ranks may share a GPU)

    @classmethod
    def load(cls, path: str = DEFAULT_XML, **overrides) -> "SolverConfig":
        t = Etree(path)
        name = overrides.pop("config", None) or t.get_node_value("solver/config")
        specs = t.dict_walkData("operator/configs")
        if name not in specs:
            raise KeyError(f"config {name!r} not in operator/configs ({sorted(specs)})")
        dim, shape, fp32 = parse_config_spec(specs[name])
        phys = {k: float(v) for k, v in t.dict_walkData("operator/physics").items()}
        cfg = cls(config=name, dim=dim, shape=shape, fp32=fp32, physics=phys,
                  rtol=float(t.get_node_value("solver/rtol")),
                  atol=float(t.get_node_value("solver/atol")),
                  restart=int(t.get_node_value("solver/restart")),
                  maxiter=int(t.get_node_value("solver/maxiter")),
                  orth=t.get_node_value("solver/orth").lower(),
                  operator_file=t.get_node_value("operator/file"),
                  preconditioner=t.get_node_value("preconditioner/type").lower(),
                  block_size=int(t.get_node_value("preconditioner/block_size")),
                  line_stride=int(t.get_node_value("preconditioner/line_stride")),
                  line_segment=int(t.get_node_value("preconditioner/line_segment")),
                  seed=int(t.get_node_value("rhs/seed"), 0),
                  device=int(t.get_node_value("run/device")),
                  report=t.get_node_value("run/report"))
        ll = t.get_optional("operator/line_len", "auto").lower()
        cfg.line_len = None if ll in ("", "auto") else int(ll)
        cfg.gpus = int(t.get_optional("run/gpus", "1") or 1)
        cfg.comm = (t.get_optional("run/comm", "rccl") or "rccl").lower()
        for k, v in overrides.items():
            if v is not None:
                setattr(cfg, k, v)
        if cfg.preconditioner not in ("block_jacobi", "line_jacobi", "none"):
            raise ValueError(f"unknown preconditioner {cfg.preconditioner!r}")
        if cfg.orth not in ("auto", "mgs", "dcgs2"):
            raise ValueError(f"unknown orthogonalisation {cfg.orth!r}")
        if cfg.gpus < 1:
            raise ValueError(f"run/gpus must be >= 1, got {cfg.gpus}")
        if cfg.comm not in ("rccl", "host"):
            raise ValueError(f"unknown run/comm {cfg.comm!r} (rccl, host)")
        return cfg

    def slab_align(self) -> int:
        """Row-partition granule: whole x-slabs (a 2D x-line of Nv rows, a 4D x-plane of
        Ny Nvx Nvy rows), so that the band step and the 4D grid rows run across ranks; 1 for an
        operator file unless operator/line_len names its line length."""
        if self.operator_file:
            return self.line_len or 1
        if self.dim == 2:
            return self.shape[1]
        if self.dim == 4:
            return self.shape[1] * self.shape[2] * self.shape[3]
        return 1
