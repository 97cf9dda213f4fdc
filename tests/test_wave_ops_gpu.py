"""Device self-test of the wave-level lane exchanges the window kernels sort
with (DPP row rotations, v_permlane16/32_swap) against ds_bpermute shuffles,
and of the bitonic sort / top-64 merge built on them."""
import ctypes

import pytest

from ksg import engine


@pytest.mark.gpu
def test_lane_exchanges_and_sort_match_shuffles():
    L = engine.load_library()
    L.ksg_debug_lane_selftest.argtypes = [ctypes.POINTER(ctypes.c_int32)]
    bad = ctypes.c_int32(-1)
    assert L.ksg_debug_lane_selftest(ctypes.byref(bad)) == 0
    assert bad.value == 0
