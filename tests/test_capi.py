"""CPU-side checks of the C-ABI library (no compute calls without a GPU)."""
import ctypes
import os

import genometools_smax_amd as G


def test_library_builds_and_loads():
    assert os.path.exists(G.LIB_PATH)
    G.lib()


def test_every_declared_symbol_is_exported():
    lib = ctypes.CDLL(G.LIB_PATH)
    names = G.exported_symbols()
    assert "gt_smax_hip_enumerate" in names and "gt_smax_plan_run" in names
    for name in names:
        assert hasattr(lib, name), name


def test_struct_sizes_match_header():
    # GtSmaxLlv must equal Largelcpvalue on LP64 (two GtUword)
    assert ctypes.sizeof(G.GtSmaxLlv) == 16
    assert ctypes.sizeof(G.GtSmaxRecord) == 16
    assert G.RECORD_DTYPE.itemsize == 16
    assert ctypes.sizeof(G.GtSmaxBoundary) == 8 * (3 + 5 + 3 + 5 + 2)


def test_host_stitch_pure_function():
    # shard 0 ends inside a plateau of lcp 30 that shard 1's head closes
    b0, b1 = G.GtSmaxBoundary(), G.GtSmaxBoundary()
    b0.pend_valid, b0.pend_c, b0.pend_lcp = 1, 100, 30
    b0.pend_div.seen[0] = 0b0011
    b1.head_v, b1.head_f, b1.head_next = 30, 103, 7
    b1.head_div.seen[0] = 0b0100
    assert G.stitch_host([b0, b1], 0, 20) == (30, 99, 102)
    b1.head_div.seen[0] = 0b0010           # duplicate left symbol
    assert G.stitch_host([b0, b1], 0, 20) is None
    b1.head_div.seen[0] = 0b0100
    b1.head_next = 31                      # not a local maximum
    assert G.stitch_host([b0, b1], 0, 20) is None
