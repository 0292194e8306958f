"""tools/pmc_summary.py's kernel classes match the demangled names rocprofv3 reports for the
current kernels (a template change left the C4 ring kernel out of the PMC summary).
CPU only: the names are the instantiations the solver launches on the bench configurations."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import pmc_summary  # noqa: E402

NAMES = {   # rocprofv3 Kernel_Name (argument lists shortened) -> class
    "void vtk::k_band_step<5, 3, 2, false, 3>(vtk::BandK)": "band_step",
    "void vtk::k_band_step<5, 14, 2, false, 1>(vtk::BandK)": "band_step",
    "void vtk::k_g4_ring<float, false, 5120, 0, 512>(vtk::Grid4, double const*)": "spmv_bj",
    "void vtk::k_g4_ring<double, true, 8192, 0, 256>(vtk::Grid4, double const*)": "spmv_bj",
    "void vtk::k_g4_ring<float, false, 5120, 2, 512>(vtk::Grid4, double const*)": "spmv_bj_dc",
    "void vtk::k_g4_ring<float, true, 5120, 3, 512>(vtk::Grid4, double const*)": "spmv_resid_bj",
    "void vtk::k_lsv_ring_epi<3>(vtk::LsvEpiK)": "spmv_resid_bj",
    "void vtk::k_lsv_ring_epi<4>(vtk::LsvEpiK)": "spmv_bj_dc",
    "void vtk::k_sell<float, false, 0, 1, false, 0, 9, 0>(vtk::SpmvK<float, false>)": "spmv",
    "void vtk::k_dc_update<true>(double*, long, int)": "dc_update",
    "void vtk::k_dc_dots_rows<16>(double const*, long, int)": "dc_dots",
    "vtk::k_dc_scalar(double const*, int, double const*, int)": "dc_scalar",
    "vtk::k_xupdate(double const*, double const*, double const*, long)": "xupdate",
    "void vtk::k_line_apply<25, true, true>(vtk::LineOp, double const*)": "line_dc",
    "void vtk::k_line_spmv_dc<25>(vtk::LineOp, double const*, double const*, double*, int, int const*, int, vtk::LineDc)": "line_dc",
    "void vtk::k_line_spmv_dc<8>(vtk::LineOp, double const*)": "line_dc",
    "void vtk::k_line_apply<25, true, false>(vtk::LineOp, double const*, double*)": "line_apply",
}


def _classes(name):
    out = []
    for cls, p in pmc_summary.CLASSES.items():
        rx = re.compile(p if p.startswith("void") else re.escape(p))
        if rx.match(name):
            out.append(cls)
    return out


def test_every_kernel_lands_in_its_class():
    for name, cls in NAMES.items():
        assert _classes(name) == [cls], (name, _classes(name))
