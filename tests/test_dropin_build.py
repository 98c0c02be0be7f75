"""CPU: the Fortran drop-in harness is linked against libmpas_dycore.so and NOT against the
reference dycore module (its *_work routines are absent), so tests/test_gpu_dropin.py
exercises the product behind the reference's Fortran API."""
import os
import subprocess

import pytest

from oracle import ref_runner


@pytest.mark.parametrize("binary", [ref_runner.DROPIN_HARNESS, ref_runner.DROPIN_PHYS_HARNESS])
def test_dropin_links_product_not_reference(binary):
    if not ref_runner.available(binary):
        pytest.skip("make -C oracle dropin not run")
    b = binary
    ldd = subprocess.run(["ldd", b], capture_output=True, text=True).stdout
    line = [x for x in ldd.splitlines() if "libmpas_dycore.so" in x]
    assert line and "not found" not in line[0], ldd
    syms = subprocess.run(["nm", b], capture_output=True, text=True).stdout
    for sym in ("atm_srk3", "atm_timestep", "atm_dycore_to_host", "atm_dycore_from_host", "atm_dycore_wait"):
        assert f"_QMatm_time_integrationP{sym}" in syms, sym
    if binary == ref_runner.DROPIN_PHYS_HARNESS:   # the DO_PHYSICS hand-off is compiled in
        assert "_QMatm_time_integrationPphysics_to_device" in syms
    for ref_only in ("atm_advance_acoustic_step_work", "atm_compute_dyn_tend_work", "atm_recover_large_step_variables_work"):
        assert ref_only not in syms, f"reference routine {ref_only} linked into the drop-in harness"
    assert os.path.getsize(b) > 0
