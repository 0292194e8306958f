"""SciPy ``save_npz`` / ``load_npz`` CSR archives, without SciPy.

File format (scipy/sparse/_matrix_io.py, SciPy 1.15): a NumPy ``.npz`` (zip of ``.npy``
members, deflated by default) holding ``indices``, ``indptr``, ``format`` (b"csr"), ``shape``,
``data`` and, for sparse arrays, ``_is_array``.  ``load_npz`` here reads the same members with
``allow_pickle=False`` semantics (only plain dtypes are accepted) and can read one rank's row
block: the member streams are read piecewise (a stored member seeks directly, a deflated one
is inflated up to the slice), so a rank never holds more than its rows.

Entries keep their stored order: the device SpMV sums each row in that order, exactly as
SciPy's ``csr_matvec`` does, so a non-canonical file (unsorted columns, duplicates) gives the
same y as ``scipy.sparse.load_npz(f) @ x``.
"""
from __future__ import annotations

import zipfile

import numpy as np
from numpy.lib import format as npf

__all__ = ["load_npz_arrays", "save_npz_arrays", "npz_shape"]


class _Member:
    """One ``.npy`` member of an open zip: dtype, shape and piecewise reads."""

    def __init__(self, zf: zipfile.ZipFile, key: str):
        name = key + ".npy"
        if name not in zf.namelist():
            raise ValueError(f"npz archive has no '{key}' member")
        self.f = zf.open(name)
        version = npf.read_magic(self.f)
        if version == (1, 0):
            shape, fortran, dtype = npf.read_array_header_1_0(self.f)
        elif version in ((2, 0), (3, 0)):
            shape, fortran, dtype = npf.read_array_header_2_0(self.f)
        else:
            raise ValueError(f"unsupported .npy version {version} in member '{key}'")
        if dtype.hasobject:
            raise ValueError(f"member '{key}' holds Python objects (pickles are not loaded)")
        if fortran and len(shape) > 1:
            raise ValueError(f"member '{key}' is Fortran-ordered")
        self.shape, self.dtype = tuple(shape), dtype
        self.data_start = self.f.tell()

    def read(self, start: int = 0, stop: int | None = None) -> np.ndarray:
        n = int(np.prod(self.shape)) if self.shape else 1
        stop = n if stop is None else stop
        if not 0 <= start <= stop <= n:
            raise ValueError("slice outside the member")
        isz = self.dtype.itemsize
        self.f.seek(self.data_start + start * isz)
        buf = self.f.read((stop - start) * isz)
        if len(buf) != (stop - start) * isz:
            raise ValueError("truncated npz member")
        a = np.frombuffer(buf, dtype=self.dtype)
        return a if stop - start != n or not self.shape else a.reshape(self.shape)

    def close(self):
        self.f.close()


def _format(zf) -> str:
    m = _Member(zf, "format")
    v = m.read()
    m.close()
    v = v.item() if v.shape == () else v[0]
    return v.decode("ascii") if isinstance(v, bytes) else str(v)


def _open(file) -> zipfile.ZipFile:
    try:
        return zipfile.ZipFile(file)
    except zipfile.BadZipFile as e:
        raise ValueError(f"not an npz archive: {e}") from e


def npz_shape(file) -> tuple[int, int]:
    with _open(file) as zf:
        m = _Member(zf, "shape")
        s = m.read()
        m.close()
    return int(s[0]), int(s[1])


def load_npz_arrays(file, rows: tuple[int, int] | None = None):
    """``(indptr, indices, data, shape)`` of a SciPy CSR archive; with ``rows=(r0, r1)`` only
    that row block (``indptr`` rebased to 0, column indices global).  Indices are returned as
    int32 (ValueError when they do not fit), data as float64, or float32 when stored so."""
    with _open(file) as zf:
        fmt = _format(zf)
        if fmt != "csr":
            raise NotImplementedError(f"sparse format '{fmt}': only CSR archives are supported "
                                      "(convert with scipy.sparse's .tocsr() before saving)")
        ms = _Member(zf, "shape")
        shape = tuple(int(v) for v in ms.read())
        ms.close()
        if len(shape) != 2:
            raise ValueError("CSR archive shape must be 2-D")
        r0, r1 = (0, shape[0]) if rows is None else (int(rows[0]), int(rows[1]))
        if not 0 <= r0 <= r1 <= shape[0]:
            raise ValueError("row block outside the matrix")
        mp = _Member(zf, "indptr")
        if mp.shape != (shape[0] + 1,):
            raise ValueError("indptr length does not match shape")
        ip = mp.read(r0, r1 + 1).astype(np.int64)
        mp.close()
        k0, k1 = int(ip[0]), int(ip[-1])
        if np.any(np.diff(ip) < 0):
            raise ValueError("indptr must be non-decreasing")
        mi, md = _Member(zf, "indices"), _Member(zf, "data")
        if mi.shape != md.shape or (mi.shape and k1 > mi.shape[0]):
            raise ValueError("indices/data lengths do not match indptr")
        ix, d = mi.read(k0, k1), md.read(k0, k1)
        mi.close()
        md.close()
    if ix.dtype.kind not in "iu":
        raise ValueError("indices must be integers")
    if ix.size and (int(ix.min()) < 0 or int(ix.max()) >= shape[1]):
        raise ValueError("column index out of range")
    if k1 - k0 > np.iinfo(np.int32).max or shape[1] > np.iinfo(np.int32).max:
        raise ValueError("row block too large for int32 CSR indices")
    if d.dtype.kind == "c":
        raise ValueError("complex matrices are not supported")
    d = np.ascontiguousarray(d, dtype=np.float32 if d.dtype == np.float32 else np.float64)
    return ((ip - k0).astype(np.int32), np.ascontiguousarray(ix, dtype=np.int32), d, shape)


def save_npz_arrays(file, indptr, indices, data, shape, compressed: bool = True) -> None:
    """Write a CSR archive that ``scipy.sparse.load_npz`` reads back as a ``csr_matrix``
    (same members and member order as ``scipy.sparse.save_npz``)."""
    arrays = {"indices": np.asarray(indices), "indptr": np.asarray(indptr),
              "format": np.array(b"csr"), "shape": np.asarray(shape, dtype=np.int64),
              "data": np.asarray(data)}
    (np.savez_compressed if compressed else np.savez)(file, **arrays)
