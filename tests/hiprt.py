"""Device buffers for the device-pointer tests: the package's binding of the
HIP runtime libpsn_lk.so is bound to (mcmtt_opticalflow_amd/hip.py; no torch)."""
from mcmtt_opticalflow_amd.hip import D2H, H2D, DeviceBuffer, rt  # noqa: F401


def hip():
    return rt()
