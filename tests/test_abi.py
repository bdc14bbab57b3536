"""CPU checks of the drop-in boundary: libpsn_lk.so loads without a GPU and
exports every function include/psn_lk.h declares; the host-only entry points
(no device work) behave like the reference interface they replace."""
import ctypes

import pytest

from mcmtt_opticalflow_amd import _lib


def test_header_declares_the_boundary():
    names = _lib.header_functions()
    for must in ("psn_lk_create", "psn_lk_push_frame", "psn_lk_push_frame_device", "psn_lk_track",
                 "psn_lk_track_device", "psn_calc_optical_flow_pyr_lk", "psn_comm_allgather",
                 "psn_lk_destroy", "psn_lk_last_error"):
        assert must in names


def test_library_exports_every_header_symbol():
    L = _lib.load()
    missing = [n for n in _lib.header_functions() if not hasattr(L, n)]
    assert not missing, missing


def test_abi_version():
    assert _lib.load().psn_lk_abi_version() == 5


def test_default_params_are_opencv_246_defaults():
    p = _lib.default_params()
    assert (p.win_w, p.win_h, p.max_level, p.term_type, p.max_count, p.flags) == (21, 21, 3, 3, 30, 0)
    assert p.epsilon == 0.01 and p.min_eig_threshold == 1e-4


@pytest.mark.parametrize("w,h,win,ml,exp", [
    (1920, 1080, 21, 3, 3), (640, 480, 60, 3, 2), (1920, 1080, 160, 3, 2), (30, 30, 21, 5, 0),
    (3840, 2160, 21, 4, 4), (768, 576, 40, 3, 3),
])
def test_effective_max_level_matches_oracle(oracle_mod, w, h, win, ml, exp):
    L = _lib.load()
    assert L.psn_lk_effective_max_level(w, h, win, win, ml) == exp
    assert oracle_mod.effective_max_level(w, h, win, win, ml) == exp


def test_bad_arguments_return_codes_not_crashes():
    L = _lib.load()
    out = ctypes.c_void_p()
    assert L.psn_lk_create(0, 0, 10, 4, 3, ctypes.byref(out)) == -1
    assert L.psn_lk_create(0, 10, 10, 4, 99, ctypes.byref(out)) == -1
    assert L.psn_lk_effective_max_level(0, 10, 3, 3, 3) == -1
    assert L.psn_lk_sync(None) == -1
    assert L.psn_lk_track(None, None, 0, None, None, None, None) == -1
    assert L.psn_comm_init(0, 0, 0, None, ctypes.byref(out)) == -1


@pytest.mark.parametrize("w,h,exp", [
    (3, 3, 1), (6400, 1, 1), (6401, 1, 0), (6400, 2621, 1), (6400, 2622, 0),
    (4095, 4095, 1), (4096, 4096, 0), (4200, 4200, 0), (4200, 100, 1), (0, 5, 0), (5, 0, 0),
])
def test_window_supported_predicate(w, h, exp):
    """psn_lk_window_supported: width <= 6400 and h * ceil(w/4) < 2^22 quads --
    the one predicate psn_lk_track and the Tracker2D host both apply (a square
    backward window box.w x box.w is out past box.w = 4095)."""
    L = _lib.load()
    assert L.psn_lk_window_supported(w, h) == exp
    assert exp == (0 < w <= 6400 and 0 < h and h * ((w + 3) // 4) < (1 << 22))
