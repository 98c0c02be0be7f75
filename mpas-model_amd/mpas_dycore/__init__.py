"""mpas_dycore: MI355X-native MPAS-Atmosphere split-explicit dycore (host side).

The compute path is the HIP library built from ../csrc (libmpas_dycore.so);
this package holds the C-ABI binding, the host mirror of the reference's
atm_time_integration interface and the synthetic mesh / initial-state tools.
"""
from .dycore import Dycore, DycoreError  # noqa: F401
