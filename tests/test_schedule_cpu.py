"""K1's guided tile schedule (gt_smax_k1_schedule, the pure host function
plan_size_grid uses): generation g's workgroups [blk[g], blk[g+1]) take the
tiles [tile[g], tile[g+1]) interleaved, so every tile must be covered once,
in ascending order, with at most `resident` workgroups per generation, the
per-workgroup counts non-increasing from one generation to the next, and
the last generation short.  Pure host code: no GPU involved."""
import ctypes

import numpy as np
import pytest

import genometools_smax_amd as G

SCHED_MAX = 12


def schedule(nt, resident):
    L = G.lib()
    f = L.gt_smax_k1_schedule
    f.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    f.restype = ctypes.c_uint32
    blk = np.zeros(SCHED_MAX + 1, np.uint32)
    tile = np.zeros(SCHED_MAX + 1, np.uint32)
    n = f(nt, resident, blk.ctypes.data, tile.ctypes.data)
    return int(n), blk[: n + 1].astype(np.int64), tile[: n + 1].astype(np.int64)


@pytest.mark.parametrize("nt,resident", [(1, 6144), (50, 6144), (6144, 6144), (12000, 6144),
                                         (61000, 6144), (181234, 6144), (1449874, 6144),
                                         (5808000, 6144), (1449874, 5120), (7, 3), (1000, 1)])
def test_schedule_covers_every_tile_once(nt, resident):
    n, blk, tile = schedule(nt, resident)
    assert 1 <= n <= SCHED_MAX
    assert blk[0] == 0 and tile[0] == 0 and tile[n] == nt
    seen = np.zeros(nt, np.int64)
    per_wg = []
    for g in range(n):
        w = blk[g + 1] - blk[g]
        assert 1 <= w <= resident
        span = tile[g + 1] - tile[g]
        # workgroup j of the generation: tiles tile[g] + j + k*w below tile[g+1]
        counts = [len(range(tile[g] + j, tile[g + 1], w)) for j in range(w)]
        assert sum(counts) == span and min(counts) >= 1
        assert max(counts) - min(counts) <= 1
        per_wg.append(max(counts))
        seen[tile[g]:tile[g + 1]] += 1
    assert np.all(seen == 1)
    assert per_wg == sorted(per_wg, reverse=True)
    assert per_wg[-1] <= 2 or n == SCHED_MAX


def test_schedule_of_c3_and_a_shard():
    # (the A/B'd configurations): the first
    # generation fills every slot and takes about 2/3 of the tiles, and the
    # launch has a few generations, not the 8-16 equal ones of the static grid
    for nt, gens in ((1449874, 5), (181234, 4)):
        n, blk, tile = schedule(nt, 6144)
        assert n == gens
        assert blk[1] - blk[0] == 6144
        assert 2 * nt / 3 <= tile[1] <= 2 * nt / 3 + 6144
