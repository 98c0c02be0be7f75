"""Classic netCDF files (CDF-1, CDF-2 "64-bit offset", CDF-5 "64-bit data") in numpy.

MPAS reads and writes its meshes, initial conditions and restarts through PIO
(`framework/mpas_io.F`), whose serial and parallel-netCDF back ends produce
exactly these three formats (`io_type="pnetcdf"` -> CDF-2, `"pnetcdf,cdf5"` ->
CDF-5).  This module is a from-scratch reader/writer of the published classic
format (the netCDF "File Format Specification"): big-endian header of
dimensions, attributes and variables; fixed-size variables stored contiguously
at their `begin` offsets; record variables interleaved record by record along
the unlimited dimension (MPAS's `Time`).  netCDF-4/HDF5 files are recognised and
refused with a clear message (there is no HDF5 library in this image).

    ds = read("x1.40962.init.nc")          # Dataset: .dims, .vars, .attrs, .unlimited
    u = ds["u"]                             # numpy array, (Time, nEdges, nVertLevels)
    write("out.nc", ds, version=2)          # or version=5

Arrays come back in the file's C order, which for MPAS is the transpose of the
Fortran dimension list -- e.g. `u(nVertLevels, nEdges, Time)` in Registry.xml
is `u[Time, nEdges, nVertLevels]` here, the element-major layout of
`mpas_dycore` (fields.py).
"""
from __future__ import annotations

import mmap
import os
import struct
from dataclasses import dataclass, field

import numpy as np

NC_DIMENSION, NC_VARIABLE, NC_ATTRIBUTE = 0x0A, 0x0B, 0x0C
# nc_type -> numpy big-endian dtype
NC_TYPES = {1: ">i1", 2: "S1", 3: ">i2", 4: ">i4", 5: ">f4", 6: ">f8",
            7: ">u1", 8: ">u2", 9: ">u4", 10: ">i8", 11: ">u8"}
CDF5_ONLY = {7, 8, 9, 10, 11}


def _nc_type_of(dt: np.dtype) -> int:
    dt = np.dtype(dt)
    if dt.kind == "S":
        return 2
    key = {("i", 1): 1, ("i", 2): 3, ("i", 4): 4, ("f", 4): 5, ("f", 8): 6, ("u", 1): 7, ("u", 2): 8,
           ("u", 4): 9, ("i", 8): 10, ("u", 8): 11}.get((dt.kind, dt.itemsize))
    if key is None:
        raise TypeError(f"no netCDF type for numpy dtype {dt}")
    return key


@dataclass
class Variable:
    name: str
    dims: tuple
    data: np.ndarray
    attrs: dict = field(default_factory=dict)


@dataclass
class Dataset:
    dims: dict = field(default_factory=dict)       # name -> length (the unlimited one: current record count)
    vars: dict = field(default_factory=dict)       # name -> Variable
    attrs: dict = field(default_factory=dict)
    unlimited: str | None = None
    version: int = 2

    def __getitem__(self, name):
        return self.vars[name].data

    def __contains__(self, name):
        return name in self.vars

    def add(self, name, dims, data, **attrs):
        data = np.asarray(data)
        dims = tuple(dims)
        if data.ndim != len(dims):
            raise ValueError(f"{name}: {data.ndim}-d data for dims {dims}")
        for d, n in zip(dims, data.shape):
            if d == self.unlimited:
                self.dims[d] = max(self.dims.get(d, 0), n)
            elif self.dims.setdefault(d, n) != n:
                raise ValueError(f"{name}: dimension {d} is {self.dims[d]}, data has {n}")
        self.vars[name] = Variable(name, dims, data, dict(attrs))
        return self


class FormatError(ValueError):
    pass


# ---------------------------------------------------------------------------------------------
# reading
class _Reader:
    def __init__(self, buf, version):
        self.b = buf
        self.p = 4
        self.v = version

    def i4(self):
        (x,) = struct.unpack_from(">i", self.b, self.p)
        self.p += 4
        return x

    def i8(self):
        (x,) = struct.unpack_from(">q", self.b, self.p)
        self.p += 8
        return x

    def nonneg(self):  # NON_NEG: INT (CDF-1/2) or INT64 (CDF-5)
        return self.i8() if self.v == 5 else self.i4()

    def offset(self):  # OFFSET: INT (CDF-1) or INT64 (CDF-2/5)
        return self.i4() if self.v == 1 else self.i8()

    def name(self):
        n = self.nonneg()
        s = bytes(self.b[self.p:self.p + n]).decode("utf-8")
        self.p += (n + 3) & ~3
        return s

    def values(self, nc_type, n):
        dt = np.dtype(NC_TYPES[nc_type])
        nb = n * dt.itemsize
        a = np.frombuffer(self.b, dtype=dt, count=n, offset=self.p).copy()
        self.p += (nb + 3) & ~3
        if nc_type == 2:
            return a.tobytes().rstrip(b"\0").decode("utf-8", "replace")
        return a.astype(dt.newbyteorder("="))

    def header_list(self, tag_expected):
        tag = self.i4()
        n = self.nonneg()
        if tag == 0:
            if n != 0:
                raise FormatError("malformed ABSENT list")
            return 0
        if tag != tag_expected:
            raise FormatError(f"expected list tag {tag_expected:#x}, found {tag:#x}")
        return n

    def attrs(self):
        out = {}
        for _ in range(self.header_list(NC_ATTRIBUTE)):
            nm = self.name()
            t = self.i4()
            n = self.nonneg()
            out[nm] = self.values(t, n)
        return out


def read(path: str, variables=None, mmap_data: bool = False) -> Dataset:
    """Read a classic netCDF file.  ``variables`` restricts which variables are loaded
    (the header is always parsed); ``mmap_data`` returns read-only memory-mapped views
    in file byte order instead of native-order copies (large meshes)."""
    with open(path, "rb") as f:
        head = f.read(8)
        if head.startswith(b"\x89HDF"):
            raise FormatError(f"{path}: netCDF-4/HDF5 file; convert it to a classic format first "
                              f"(e.g. nccopy -k cdf5 or -k 64-bit-offset)")
        if head[:3] != b"CDF" or head[3] not in (1, 2, 5):
            raise FormatError(f"{path}: not a classic netCDF file")
        mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
    version = mm[3]
    r = _Reader(mm, version)
    numrecs = r.nonneg()
    ds = Dataset(version=version)
    dimlist = []
    for _ in range(r.header_list(NC_DIMENSION)):
        nm = r.name()
        ln = r.nonneg()
        if ln == 0:
            ds.unlimited = nm
            ln = max(numrecs, 0)
        dimlist.append((nm, ln))
        ds.dims[nm] = ln
    ds.attrs = r.attrs()
    specs = []
    for _ in range(r.header_list(NC_VARIABLE)):
        nm = r.name()
        nd = r.nonneg()
        dimids = [r.nonneg() for _ in range(nd)]
        va = r.attrs()
        t = r.i4()
        vsize = r.nonneg()
        begin = r.offset()
        specs.append((nm, dimids, va, t, vsize, begin))
    def rec_bytes(sp):  # one record of a record variable (vsize recomputed: it saturates in CDF-2)
        return int(np.prod([dimlist[d][1] for d in sp[1][1:]], dtype=np.int64)) * np.dtype(NC_TYPES[sp[3]]).itemsize

    rec_specs = [sp for sp in specs if sp[1] and dimlist[sp[1][0]][0] == ds.unlimited]
    if len(rec_specs) == 1:  # a single record variable is not padded (format spec, "vsize")
        recsize = rec_bytes(rec_specs[0])
    else:
        recsize = sum((rec_bytes(sp) + 3) & ~3 for sp in rec_specs)
    if ds.unlimited and numrecs < 0:  # STREAMING: count the records the file holds
        first = min(sp[5] for sp in rec_specs) if rec_specs else len(mm)
        numrecs = (len(mm) - first) // recsize if recsize else 0
        ds.dims[ds.unlimited] = numrecs
        dimlist = [(nm, numrecs if nm == ds.unlimited else ln) for nm, ln in dimlist]
    for nm, dimids, va, t, vsize, begin in specs:
        dims = tuple(dimlist[d][0] for d in dimids)
        if variables is not None and nm not in variables:
            ds.vars[nm] = Variable(nm, dims, None, va)
            continue
        dt = np.dtype(NC_TYPES[t])
        is_rec = bool(dimids) and dims[0] == ds.unlimited
        shape = tuple(dimlist[d][1] for d in dimids)
        if is_rec:
            inner = shape[1:]
            nin = int(np.prod(inner, dtype=np.int64))
            nrec = ds.dims[ds.unlimited]
            if nrec and recsize == nin * dt.itemsize:
                a = np.frombuffer(mm, dtype=dt, count=nrec * nin, offset=begin).reshape((nrec,) + inner)
            else:
                a = np.empty((nrec,) + inner, dtype=dt)
                for i in range(nrec):
                    a[i] = np.frombuffer(mm, dtype=dt, count=nin, offset=begin + i * recsize).reshape(inner)
        else:
            n = int(np.prod(shape, dtype=np.int64))
            a = np.frombuffer(mm, dtype=dt, count=n, offset=begin).reshape(shape)
        if t == 2:
            a = a.view("S1")
        elif not mmap_data:
            a = a.astype(dt.newbyteorder("="))
        ds.vars[nm] = Variable(nm, dims, a, va)
    return ds


# ---------------------------------------------------------------------------------------------
# writing
def _pad4(b: bytes) -> bytes:
    return b + b"\0" * ((-len(b)) % 4)


class _Writer:
    def __init__(self, version):
        self.v = version
        self.out = bytearray()

    def i4(self, x):
        self.out += struct.pack(">i", x)

    def nonneg(self, x):
        self.out += struct.pack(">q" if self.v == 5 else ">i", x)

    def offset(self, x):
        self.out += struct.pack(">i" if self.v == 1 else ">q", x)

    def name(self, s):
        b = s.encode("utf-8")
        self.nonneg(len(b))
        self.out += _pad4(b)

    def attrs(self, attrs):
        if not attrs:
            self.i4(0)
            self.nonneg(0)
            return
        self.i4(NC_ATTRIBUTE)
        self.nonneg(len(attrs))
        for k, val in attrs.items():
            self.name(k)
            if isinstance(val, (str, bytes)):
                b = val.encode("utf-8") if isinstance(val, str) else val
                self.i4(2)
                self.nonneg(len(b))
                self.out += _pad4(b)
            else:
                a = np.atleast_1d(np.asarray(val))
                if a.dtype == np.int64 and self.v != 5:
                    a = a.astype(np.int32)
                t = _nc_type_of(a.dtype)
                self.i4(t)
                self.nonneg(a.size)
                self.out += _pad4(a.astype(NC_TYPES[t]).tobytes())


def write(path: str, ds: Dataset, version: int | None = None) -> None:
    """Write ``ds`` as CDF-1, CDF-2 (default, what MPAS's pnetcdf output uses) or CDF-5."""
    v = version or ds.version or 2
    if v not in (1, 2, 5):
        raise ValueError("version must be 1, 2 or 5")
    dimnames = list(ds.dims)
    if ds.unlimited and ds.unlimited in dimnames:  # the record dimension goes first, by convention
        dimnames.remove(ds.unlimited)
        dimnames.insert(0, ds.unlimited)
    dimid = {d: i for i, d in enumerate(dimnames)}
    nrec = ds.dims.get(ds.unlimited, 0) if ds.unlimited else 0

    def enc(var):
        a = np.asarray(var.data)
        if a.dtype.kind in "SU":
            if a.dtype.itemsize != 1 or a.dtype.kind == "U":
                raise TypeError(f"{var.name}: char variables are 'S1' arrays (last axis = string length)")
            return 2, a
        if a.dtype == np.int64 and v != 5:
            if a.size and (a.min() < -2 ** 31 or a.max() >= 2 ** 31):
                raise ValueError(f"{var.name}: int64 values need CDF-5")
            a = a.astype(np.int32)
        t = _nc_type_of(a.dtype)
        if t in CDF5_ONLY and v != 5:
            raise ValueError(f"{var.name}: type {a.dtype} needs CDF-5")
        return t, a.astype(NC_TYPES[t])

    encoded = {n: enc(var) for n, var in ds.vars.items()}
    fixed = [n for n, var in ds.vars.items() if not (var.dims and var.dims[0] == ds.unlimited)]
    recs = [n for n in ds.vars if n not in fixed]

    def vsize(n):
        var = ds.vars[n]
        t, a = encoded[n]
        shape = [ds.dims[d] for d in var.dims]
        if n in recs:
            shape = shape[1:]
        nb = int(np.prod(shape, dtype=np.int64)) * np.dtype(NC_TYPES[t]).itemsize
        if n in recs and len(recs) == 1:
            return nb
        return (nb + 3) & ~3

    def header(begins):
        w = _Writer(v)
        w.out += b"CDF" + bytes([v])
        w.nonneg(nrec)
        if dimnames:
            w.i4(NC_DIMENSION)
            w.nonneg(len(dimnames))
            for d in dimnames:
                w.name(d)
                w.nonneg(0 if d == ds.unlimited else ds.dims[d])
        else:
            w.i4(0)
            w.nonneg(0)
        w.attrs(ds.attrs)
        names = fixed + recs
        if names:
            w.i4(NC_VARIABLE)
            w.nonneg(len(names))
            for n in names:
                var = ds.vars[n]
                w.name(n)
                w.nonneg(len(var.dims))
                for d in var.dims:
                    w.nonneg(dimid[d])
                w.attrs(var.attrs)
                w.i4(encoded[n][0])
                vs = vsize(n)
                w.nonneg(vs if v == 5 or vs < 2 ** 32 - 4 else 2 ** 32 - 1)
                w.offset(begins.get(n, 0))
        else:
            w.i4(0)
            w.nonneg(0)
        return bytes(w.out)

    hlen = len(header({}))
    begins = {}
    pos = hlen
    for n in fixed:
        begins[n] = pos
        pos += vsize(n)
    recstart = pos
    for n in recs:
        begins[n] = pos
        pos += vsize(n)
    recsize = pos - recstart
    if v == 1 and pos > 2 ** 31 - 1:
        raise ValueError("file too large for CDF-1; use version 2 or 5")
    hdr = header(begins)
    assert len(hdr) == hlen
    tmp = path + f".{os.getpid()}.tmp"
    with open(tmp, "wb") as f:
        f.write(hdr)
        for n in fixed:
            b = encoded[n][1].tobytes()
            f.write(b + b"\0" * (vsize(n) - len(b)))
        for i in range(nrec):
            for n in recs:
                a = encoded[n][1]
                b = a[i].tobytes() if i < a.shape[0] else b"\0" * (vsize(n))
                f.write(b + b"\0" * (vsize(n) - len(b)))
        assert f.tell() == recstart + nrec * recsize
    os.replace(tmp, path)
