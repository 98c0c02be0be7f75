"""MPAS netCDF mesh / init files: the classic-format reader/writer
(mpas_dycore.ncio) against scipy's independent netCDF-3 implementation, and init-file round
trips into dycore cases (mpas_dycore.mpas_files).  CPU only."""
import os

import numpy as np
import pytest
import scipy.io

from mpas_dycore import mpas_files, ncio
from mpas_dycore.cases import jw_case


def _demo_dataset():
    rng = np.random.default_rng(7)
    ds = ncio.Dataset(unlimited="Time")
    ds.add("latCell", ("nCells",), rng.random(7))
    ds.add("cellsOnEdge", ("nEdges", "TWO"), rng.integers(0, 7, (9, 2)).astype(np.int32))
    ds.add("u", ("Time", "nEdges", "nVertLevels"), rng.random((3, 9, 5)))
    ds.add("w", ("Time", "nCells", "nVertLevelsP1"), rng.random((3, 7, 6)))
    ds.add("flag", ("nCells",), np.arange(7, dtype=np.int8))
    ds.add("xtime", ("Time", "StrLen"),
           np.frombuffer(b"2000-01-01_00:00:00".ljust(64) * 3, dtype="S1").reshape(3, 64))
    ds.add("cf1", (), np.float64(2.0))
    ds.attrs = dict(on_a_sphere="YES", sphere_radius=6371229.0)
    return ds


@pytest.mark.parametrize("version", [1, 2, 5])
def test_classic_roundtrip(tmp_path, version):
    ds = _demo_dataset()
    p = str(tmp_path / f"t{version}.nc")
    ncio.write(p, ds, version=version)
    r = ncio.read(p)
    assert r.version == version and r.unlimited == "Time" and r.dims["Time"] == 3
    for n in ds.vars:
        assert np.array_equal(np.asarray(r[n]), np.asarray(ds[n])), n
    assert r.attrs["on_a_sphere"] == "YES" and float(r.attrs["sphere_radius"][0]) == 6371229.0


@pytest.mark.parametrize("version", [1, 2])
def test_scipy_reads_our_files_and_we_read_scipys(tmp_path, version):
    ds = _demo_dataset()
    p = str(tmp_path / "ours.nc")
    ncio.write(p, ds, version=version)
    f = scipy.io.netcdf_file(p, "r", mmap=False)
    for n in ds.vars:
        assert np.array_equal(np.asarray(f.variables[n].data), np.asarray(ds[n])), n
    f.close()
    q = str(tmp_path / "scipy.nc")
    rng = np.random.default_rng(3)
    th, ne = rng.random((2, 7, 5)), np.arange(7, dtype=np.int32)
    f = scipy.io.netcdf_file(q, "w", version=version)
    f.createDimension("Time", None)
    f.createDimension("nCells", 7)
    f.createDimension("nVertLevels", 5)
    f.createVariable("theta", "d", ("Time", "nCells", "nVertLevels"))[:] = th
    f.createVariable("nEdgesOnCell", "i", ("nCells",))[:] = ne
    f.close()
    r = ncio.read(q)
    assert np.array_equal(r["theta"], th) and np.array_equal(r["nEdgesOnCell"], ne)


def test_hdf5_is_refused(tmp_path):
    p = str(tmp_path / "h.nc")
    with open(p, "wb") as f:
        f.write(b"\x89HDF\r\n\x1a\n" + b"\0" * 64)
    with pytest.raises(ncio.FormatError, match="HDF5"):
        ncio.read(p)


def test_mesh_file_roundtrip(tmp_path):
    case = jw_case(642, K=8, cache=False)
    p = str(tmp_path / "x1.642.grid.nc")
    mpas_files.write_mesh(p, case)
    raw = ncio.read(p)
    assert raw["cellsOnEdge"].min() >= 1                       # 1-based on disk
    assert raw["edgesOnEdge"].min() == 0                       # 0 = none (pentagon-adjacent edges)
    m = mpas_files.read_mesh(p)
    for n in list(mpas_files.MESH_INDEX) + ["nEdgesOnCell", "nEdgesOnEdge", "dvEdge", "dcEdge", "areaCell",
                                            "weightsOnEdge", "kiteAreasOnVertex", "angleEdge", "fVertex"]:
        assert np.array_equal(np.asarray(m[n]), np.asarray(case[n])), n


@pytest.mark.parametrize("version", [2, 5])
def test_init_file_gives_the_same_case(tmp_path, version):
    """write_init -> read_init reproduces every array the dycore uploads, bit for bit
    (the model-init precompute runs again on the file's fields)."""
    case = jw_case(642, K=8, ns=3, moist=True, cache=False)
    p = str(tmp_path / "x1.642.init.nc")
    mpas_files.write_init(p, case, version=version)
    got = mpas_files.read_init(p, config=case["config"])
    assert got["num_scalars"] == 3 and got["scalar_names"] == ["qv", "qc", "qr"]
    from mpas_dycore import fields as F
    names = [n for n in case if n in F.LOCATION or n in F.VERTICAL_1D or n in F.SCALARS_0D]
    names += ["nAdvCellsForEdge", "advCellsForEdge", "adv_coefs", "adv_coefs_3rd"]
    for n in names:
        a, b = np.asarray(case[n]), np.asarray(got[n])
        assert a.shape == b.shape and np.array_equal(a, b), n


@pytest.mark.parametrize("fill", ["none", "repeat"])
def test_init_file_declaring_max_edges_10(tmp_path, fill):
    """MPAS-distributed meshes declare maxEdges = 10, maxEdges2 = 20 whatever their cells' degree
    (core_atmosphere/Registry.xml:13-16).  A file written that way reads back as the same case at
    those strides: every slot a cell or edge uses equals the maxEdges = 6 case's, the model-init
    precompute leaves the unused slots at 0, and the index padding is whatever the file held."""
    from mpas_dycore.mesh import MAX_EDGES2_ARRAYS, MAX_EDGES_ARRAYS, pad_max_edges
    case = jw_case(642, K=8, ns=3, moist=True, cache=False)
    p0, p1 = str(tmp_path / "me6.nc"), str(tmp_path / "me10.nc")
    mpas_files.write_init(p0, case, version=5)
    mpas_files.write_init(p1, pad_max_edges(case, 10, 20, fill), version=5)
    r0 = mpas_files.read_init(p0, config=case["config"])
    r1 = mpas_files.read_init(p1, config=case["config"])
    assert (r0["maxEdges"], r0["maxEdges2"], r1["maxEdges"], r1["maxEdges2"]) == (6, 12, 10, 20)
    noc, noe = r0["nEdgesOnCell"], r0["nEdgesOnEdge"]
    for names, cnt in ((MAX_EDGES_ARRAYS, noc), (MAX_EDGES2_ARRAYS, noe)):
        for n in names:
            a, b = np.asarray(r0[n]), np.asarray(r1[n])
            used = np.arange(b.shape[1])[None, :] < cnt[:, None]
            assert b.shape[1] in (10, 20) and a.shape[2:] == b.shape[2:], n
            assert np.array_equal(a[used[:, :a.shape[1]]], b[used]), n
            if b.dtype.kind == "f":
                assert not b[~used].any(), n
    for n, v in r0.items():
        if isinstance(v, np.ndarray) and n not in MAX_EDGES_ARRAYS + MAX_EDGES2_ARRAYS:
            assert np.array_equal(v, r1[n]), n
