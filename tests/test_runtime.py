"""One ROCm runtime per process (CPU checks, no device work): libpsn_lk.so
binds the HIP / HSA / RCCL runtime it was built against by soname and, at
load, gives those objects the unversioned names PyTorch-ROCm's libraries ask
for (psn_runtime.cpp). Whichever of the two loads first, /proc/self/maps holds
exactly one libamdhip64, libhsa-runtime64, librccl and libamd_comgr file."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mcmtt_opticalflow_amd", "lib", "libpsn_lk.so")

PROBE = r"""
import json, sys
sys.path.insert(0, {root!r})
order = {order!r}
if order == "torch":
    import torch  # noqa: F401
from mcmtt_opticalflow_amd import _lib
_lib.load()
if order == "lib":
    import torch  # noqa: F401
print(json.dumps(_lib.runtime_info()))
"""


def _probe(order):
    p = subprocess.run([sys.executable, "-c", PROBE.format(root=ROOT, order=order)], capture_output=True, text=True,
                       timeout=300, env=dict(os.environ, HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", "")))
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.mark.skipif(not os.path.exists(LIB), reason="libpsn_lk.so not built")
def test_library_first_then_torch_maps_one_runtime():
    info = _probe("lib")
    assert info["one_runtime"], info["mapped"]
    for k in ("libamdhip64", "libhsa-runtime64", "librccl", "libamd_comgr"):
        assert len(info["mapped"][k]) == 1, (k, info["mapped"])
        assert info["mapped"][k][0].startswith("/opt/rocm"), (k, info["mapped"][k])
    assert info["unversioned_names_bound"] == 15
    assert info["hip_runtime_version"] == info["built_against_hip"]


@pytest.mark.skipif(not os.path.exists(LIB), reason="libpsn_lk.so not built")
def test_torch_first_then_library_maps_one_runtime():
    pytest.importorskip("torch")
    info = _probe("torch")
    assert info["one_runtime"], info["mapped"]
    # the library bound torch's copies (same sonames): one runtime, torch's
    assert "torch" in info["libamdhip64"]


@pytest.mark.skipif(not os.path.exists(LIB), reason="libpsn_lk.so not built")
def test_no_torch_in_the_library_process():
    info = _probe("none")
    assert info["one_runtime"], info["mapped"]
    assert info["mapped"]["libamdhip64"] and info["mapped"]["libamdhip64"][0].startswith("/opt/rocm")
