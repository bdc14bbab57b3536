"""Build-parameter guards of libpsn_lk.so (CPU, no GPU): a build parameter whose
LDS plan cannot fit the CU's 160 KB fails the compile (static_assert in
csrc/psn_lk_kernels.h) instead of producing a library that launches with
hipErrorInvalidValue. PSN_PYR_TILE=16 is the value that once built and failed
at 4K (the top-level tile's region needs ~210 KB at a 5-level pyramid)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"

pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC) and not shutil.which("hipcc"), reason="hipcc absent")


def _compile(tmp_path, *defs):
    src = tmp_path / "guard.hip"
    src.write_text('#include "psn_lk_kernels.h"\n')
    cmd = [HIPCC, "-x", "hip", "--offload-arch=gfx950", "-std=c++17", "-fsyntax-only",
           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "mcmtt_opticalflow_amd", "csrc"),
           *("-D" + d for d in defs), str(src)]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=120)


def test_default_build_parameters_compile(tmp_path):
    r = _compile(tmp_path)
    assert r.returncode == 0, r.stderr


@pytest.mark.parametrize("define,needle", [
    ("PSN_PYR_TILE=16", "PSN_PYR_TILE"),
    ("PSN_PYR_TILE=0", "PSN_PYR_TILE"),
    ("PSN_LG_JR_MAX_KB=200", "PSN_LG_JR_MAX_KB"),
])
def test_bad_build_parameter_fails_the_compile(tmp_path, define, needle):
    r = _compile(tmp_path, define)
    assert r.returncode != 0
    assert "static assertion failed" in r.stderr and needle in r.stderr, r.stderr


def test_largest_pyramid_tile_that_fits_compiles(tmp_path):
    """12 top-level pixels (measured and reverted in round 4 as slower) still fits."""
    r = _compile(tmp_path, "PSN_PYR_TILE=12")
    assert r.returncode == 0, r.stderr
