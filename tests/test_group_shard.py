"""The multi-GPU group's shard arithmetic (tt_group_tile_pixels, csrc/tt_group.hip) on the host: the
library deals exactly the tiles, in exactly the order, of the Python layouts (ttdist.tile_pixels), the
ranks' shards partition the screen, and bad arguments are refused. No GPU needed."""
import ctypes as C

import numpy as np
import pytest

import ttdist
import tthip


@pytest.mark.parametrize("W,H,world,tile", [(1920, 1080, 8, 64), (1920, 1080, 2, 64), (3840, 2160, 8, 64),
                                            (328, 200, 3, 64), (37, 29, 2, 16), (64, 64, 5, 64), (1000, 700, 4, 32),
                                            (17, 9, 7, 8)])
def test_library_shards_equal_the_python_layouts(W, H, world, tile):
    seen = np.zeros(W * H, np.int64)
    for r in range(world):
        lib = tthip.group_tile_pixels(W, H, world, r, tile)
        py = ttdist.tile_pixels(W, H, world, r, tile)
        assert np.array_equal(lib.astype(np.int64), py), (W, H, world, r)
        np.add.at(seen, lib.astype(np.int64), 1)
    assert np.all(seen == 1), "the ranks' shards partition the screen"


def test_one_rank_is_the_identity():
    assert np.array_equal(tthip.group_tile_pixels(40, 24, 1, 0), np.arange(40 * 24, dtype=np.uint32))


def test_truncated_copy_reports_the_full_count():
    L = tthip._group_lib()
    out = np.zeros(10, np.uint32)
    n = C.c_uint32()
    assert L.tt_group_tile_pixels(128, 128, 64, 2, 1, out.ctypes.data, 10, C.byref(n)) == tthip.TT_OK
    assert n.value == 2 * 64 * 64
    assert np.array_equal(out, tthip.group_tile_pixels(128, 128, 2, 1)[:10])


@pytest.mark.parametrize("args", [(0, 8, 64, 1, 0), (8, 8, 60, 1, 0), (8, 8, 0, 1, 0), (8, 8, 64, 0, 0),
                                  (8, 8, 64, 2, 2)])
def test_bad_shard_arguments_are_refused(args):
    n = C.c_uint32()
    assert tthip._group_lib().tt_group_tile_pixels(*args, None, 0, C.byref(n)) == tthip.TT_ERR_INVALID_ARG


def test_group_creation_without_a_gpu_fails_cleanly():
    if tthip.device_count() > 0:
        pytest.skip("a GPU is visible")
    L = tthip._group_lib()
    cfg = tthip.GroupConfig(width=64, height=64)
    h = C.c_void_p()
    devs = np.zeros(1, np.int32)
    assert L.tt_group_create(devs.ctypes.data, 1, C.byref(cfg), C.byref(h)) == tthip.TT_ERR_NO_DEVICE
    assert h.value is None
