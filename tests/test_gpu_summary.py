"""summarize_timestep on the device (mpas_atm_time_integration.F:6675-7018, called at 1794).

* The reduced values are exact (min / max select an element), so they must equal numpy's on the
  downloaded time level 2 bit for bit, and the located extremes must name the element the
  reference's cell-major / level-minor loop finds first (np.argmin / np.argmax on the (cell, k)
  array give that element).
* The reference itself, run with the three namelist switches on, prints the same log lines
  (15 significant digits, mpas_log.F:967-971): values within 1e-11 relative (the two dycores agree
  to ~1e-12 after one step), same level, same lat/lon.
* Four in-process blocks give the one-block values (MPI_MINLOC-style fold over blocks and ranks).
* Detailed mode aborts on a NaN in w or u, as the reference does (6926-6940).
"""
import math
import re

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PI = 2.0 * math.asin(1.0)


@pytest.fixture(scope="module")
def case():
    from mpas_dycore.cases import jw_case
    return jw_case(642, K=26, ns=3, moist=True, cache=False)


def _step(dy, case, detailed=True, sca=True, vel=True):
    dy.set_summary(global_minmax_vel=vel, detailed_minmax_vel=detailed, global_minmax_sca=sca)
    dt = float(case["dt"])
    dy.init_diagnostics(dt)
    dy.atm_timestep(dt, 1)
    dy.synchronize()
    return dy.summarize_timestep()


def _deg(lat, lon):
    lat = lat * 180.0 / PI
    lon = lon * 180.0 / PI
    return lat, (lon - 360.0 if lon > 180.0 else lon)


def _located(a, lat, lon, kind):
    i = int(np.argmin(a)) if kind == "min" else int(np.argmax(a))
    c, k = divmod(i, a.shape[1])
    la, lo = _deg(lat[c], lon[c])
    return {"value": a.flat[i], "k": k + 1, "index": c + 1, "lat": la, "lon": lo}


@pytest.fixture(scope="module")
def single(case):
    from mpas_dycore import Dycore
    dy = Dycore(case, device=0, moist_end=3)
    s = _step(dy, case)
    fields = {"w": dy.get("state", "w", 2)[:, :case["nVertLevels"]], "u": dy.get("state", "u", 2),
              "v": dy.get("diag", "v"), "scalars": dy.get("state", "scalars", 2)}
    dy.close()
    return s, fields


def test_summary_matches_numpy_bitwise(case, single):
    s, f = single
    w, u, v = f["w"], f["u"], f["v"]
    spd = np.sqrt(u * u + v * v)
    exp = {"w_min_at": _located(w, case["latCell"], case["lonCell"], "min"),
           "w_max_at": _located(w, case["latCell"], case["lonCell"], "max"),
           "u_min_at": _located(u, case["latEdge"], case["lonEdge"], "min"),
           "u_max_at": _located(u, case["latEdge"], case["lonEdge"], "max"),
           "wsp_max_at": _located(spd, case["latEdge"], case["lonEdge"], "max")}
    for n, e in exp.items():
        assert s[n] == e, f"{n}: {s[n]} != {e}"
    assert s["w_min"] == min(0.0, w.min()) and s["w_max"] == max(0.0, w.max())
    assert s["u_min"] == min(0.0, u.min()) and s["u_max"] == max(0.0, u.max())
    for i, (a, b) in enumerate(s["scalars"]):
        q = f["scalars"][:, :, i]
        assert a == min(0.0, q.min()) and b == max(0.0, q.max())
    assert s["nan_w"] == 0 and s["nan_u"] == 0


def test_summary_matches_reference_log(case, single):
    from oracle import ref_runner
    if not ref_runner.available():
        pytest.skip("oracle/_ref not built")
    res, _ = ref_runner.run_reference(case, nsteps=1, dt=float(case["dt"]), dump_steps=[1], nthreads=8, moist_end=3,
                                      print_minmax=7)
    log = res["log"]
    s, _ = single
    num = r"(-?[0-9.]+(?:E[-+][0-9]+)?)"
    for tag, key in (("min w", "w_min_at"), ("max w", "w_max_at"), ("min u", "u_min_at"), ("max u", "u_max_at"),
                     ("max wsp", "wsp_max_at")):
        m = re.search(rf"global {tag}: {num} k=\s*(\d+), {num} lat, {num} lon", log)
        assert m, f"no '{tag}' line in the reference log"
        val, k, lat, lon = float(m.group(1)), int(m.group(2)), float(m.group(3)), float(m.group(4))
        e = s[key]
        assert abs(e["value"] - val) <= 1e-11 * abs(val), (tag, e["value"], val)
        assert e["k"] == k, (tag, e["k"], k)
        assert abs(e["lat"] - lat) < 1e-9 and abs(e["lon"] - lon) < 1e-9, (tag, e, lat, lon)
    for i, (a, b) in enumerate(s["scalars"]):
        m = re.search(rf"global min, max scalar\s+{i + 1} {num} {num}", log)
        assert m, f"no scalar {i + 1} line"
        ra, rb = float(m.group(1)), float(m.group(2))
        assert abs(a - ra) <= 1e-11 * max(abs(ra), 1e-300) + 1e-300 and abs(b - rb) <= 1e-11 * abs(rb)


def test_summary_four_blocks_equal_one_block(case, single):
    from mpas_dycore import Dycore, decomp
    s1, _ = single
    blocks = decomp.decompose(case, decomp.partition_sfc(case["nCells"], 4))
    dy = Dycore.from_blocks(blocks, device=0, moist_end=3)
    s4 = _step(dy, case)
    dy.close()
    for key in ("w_min", "w_max", "u_min", "u_max", "scalars", "nan_w", "nan_u"):
        assert s4[key] == s1[key], key
    for key in ("w_min_at", "w_max_at", "u_min_at", "u_max_at", "wsp_max_at"):
        for a in ("value", "k", "lat", "lon"):  # index is local to the owning block
            assert s4[key][a] == s1[key][a], (key, a, s4[key], s1[key])


def test_summary_global_minmax_only(case, single):
    from mpas_dycore import Dycore
    _, f = single
    dy = Dycore(case, device=0, moist_end=3)
    s = _step(dy, case, detailed=False, sca=False)
    dy.close()
    assert s["w_min"] == min(0.0, f["w"].min()) and s["u_max"] == max(0.0, f["u"].max())
    assert s["log"][1].startswith("global min, max w")


def test_summary_detailed_nan_aborts(case):
    from mpas_dycore import Dycore, DycoreError
    dy = Dycore(case, device=0, moist_end=3)
    u = dy.get("state", "u", 1).copy()
    u[17, 3] = np.nan
    dy.set("state", "u", u, 1)
    with pytest.raises(DycoreError, match="NaN detected"):
        _step(dy, case)
    dy.close()


def test_summary_refused_until_finish_step(case):
    """With MPAS_DYC_PHYSICS_MICROPHYSICS the summary belongs to mpas_dyc_finish_step (atm_srk3
    reduces after the microphysics, 1650-1660 then 1794): between the step and finish_step
    get_summary refuses instead of returning the previous step's records."""
    from mpas_dycore import Dycore, DycoreError
    dt = case["dt"]
    dy = Dycore(case, device=0, moist_end=3)
    dy.init_diagnostics(dt)
    dy.set_physics(tendencies=False, microphysics=True)
    dy.atm_timestep(dt, 1)
    with pytest.raises(DycoreError, match="finish_step"):
        dy.summarize_timestep()
    dy.finish_step(dt)
    s = dy.summarize_timestep()
    dy.shift_time_levels()
    dy.close()
    assert np.isfinite(s["w_max"]) and np.isfinite(s["u_max"])
