"""CPU: the Fortran drop-in harness is linked against libmpas_dycore.so and NOT against the
reference dycore module (its *_work routines are absent), so tests/test_gpu_dropin.py
exercises the product behind the reference's Fortran API."""
import os
import subprocess

import pytest

from oracle import ref_runner


@pytest.mark.skipif(not ref_runner.available(ref_runner.DROPIN_HARNESS), reason="make -C oracle dropin not run")
def test_dropin_links_product_not_reference():
    b = ref_runner.DROPIN_HARNESS
    ldd = subprocess.run(["ldd", b], capture_output=True, text=True).stdout
    line = [x for x in ldd.splitlines() if "libmpas_dycore.so" in x]
    assert line and "not found" not in line[0], ldd
    syms = subprocess.run(["nm", b], capture_output=True, text=True).stdout
    assert "_QMatm_time_integrationPatm_srk3" in syms
    for ref_only in ("atm_advance_acoustic_step_work", "atm_compute_dyn_tend_work", "atm_recover_large_step_variables_work"):
        assert ref_only not in syms, f"reference routine {ref_only} linked into the drop-in harness"
    assert os.path.getsize(b) > 0
