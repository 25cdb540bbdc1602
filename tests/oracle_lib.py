"""ctypes view of the CPU oracle (oracle/*.c) -- test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this
module; the product package never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "build", "liborc.so")

_u64p = ctypes.POINTER(ctypes.c_uint64)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(LIB)
        L.orc_encode_fasta.argtypes = [ctypes.c_char_p, ctypes.c_uint64, _u8p, _u64p, _u64p]
        L.orc_build_esa.argtypes = [_u8p, ctypes.c_uint64] + [ctypes.c_void_p] * 4 + [_u64p, ctypes.c_void_p]
        L.orc_free.argtypes = [ctypes.c_void_p]
        L.orc_index_fasta.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
        L.orc_decode_lcp.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, _u64p]
        L.orc_linsmax.argtypes = [_u8p, ctypes.c_void_p, ctypes.c_uint64, _u8p, ctypes.c_uint64,
                                  ctypes.c_uint64, _u64p, ctypes.c_uint64]
        L.orc_linsmax.restype = ctypes.c_uint64
        L.orc_linsmax_mt.argtypes = L.orc_linsmax.argtypes + [ctypes.c_int]
        L.orc_linsmax_mt.restype = ctypes.c_uint64
        L.orc_bottomup_smax.argtypes = [_u64p, _u64p, _u8p, ctypes.c_uint64, ctypes.c_uint64,
                                        _u64p, ctypes.c_uint64]
        L.orc_bottomup_smax.restype = ctypes.c_uint64
        L.orc_bottomup_smax_tables.argtypes = [_u8p, ctypes.c_void_p, ctypes.c_uint64, _u8p,
                                               ctypes.c_uint64, ctypes.c_uint64, _u64p,
                                               ctypes.c_uint64]
        L.orc_bottomup_smax_tables.restype = ctypes.c_uint64
        L.orc_lcp_intervals.argtypes = [_u8p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                        _u64p, ctypes.c_uint64]
        L.orc_lcp_intervals.restype = ctypes.c_uint64
        L.orc_maxpairs_blocks.argtypes = [_u8p, ctypes.c_void_p, ctypes.c_uint64, _u8p, _u64p,
                                          ctypes.c_uint64, ctypes.c_uint64, _u64p, ctypes.c_uint64]
        L.orc_maxpairs_blocks.restype = ctypes.c_uint64
        L.orc_brute_smax.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_uint64, _u64p, ctypes.c_uint64,
                                     _u64p, ctypes.c_uint64]
        L.orc_brute_smax.restype = ctypes.c_uint64
        L.orc_maxpairs.argtypes = [_u64p, _u64p, _u8p, ctypes.c_uint64, ctypes.c_uint, ctypes.c_void_p]
        L.orc_maxpairs.restype = ctypes.c_uint64
        L.orc_bottomup_events.argtypes = [_u64p, _u64p, ctypes.c_uint64, ctypes.c_void_p]
        L.orc_bottomup_events.restype = ctypes.c_uint64
        L.orc_bottomup_events_slots.argtypes = [_u64p, _u64p, ctypes.c_uint64, ctypes.c_void_p,
                                                 ctypes.c_void_p, _u64p]
        L.orc_bottomup_events_slots.restype = ctypes.c_uint64
        L.orc_dfs_events.argtypes = [_u64p, _u64p, ctypes.c_uint64, ctypes.c_void_p]
        L.orc_dfs_events.restype = ctypes.c_uint64
        L.orc_spmitv.argtypes = [_u64p, ctypes.c_uint64, _u8p, ctypes.c_uint64, ctypes.c_uint64,
                                 _u64p, _u64p]
        L.orc_spmitv.restype = ctypes.c_int
        L.orc_format_pair.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, _u64p,
                                      ctypes.c_uint64, ctypes.c_char_p, ctypes.c_int]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


def encode_fasta(path):
    with open(path, "rb") as fh:
        buf = fh.read()
    out = np.empty(len(buf) + 1, dtype=np.uint8)
    n = ctypes.c_uint64()
    ns = ctypes.c_uint64()
    rc = lib().orc_encode_fasta(buf, len(buf), _p(out, _u8p), ctypes.byref(n), ctypes.byref(ns))
    if rc != 0:
        raise ValueError("illegal symbol in %s" % path)
    return out[: n.value].copy(), ns.value


class Esa:
    """In-memory enhanced suffix array built by the oracle (gt layout)."""

    def __init__(self, text):
        text = np.ascontiguousarray(text, dtype=np.uint8)
        n = len(text)
        ptrs = [ctypes.c_void_p() for _ in range(4)]
        numllv = ctypes.c_uint64()
        bwtp = ctypes.c_void_p()
        rc = lib().orc_build_esa(_p(text, _u8p), n, *[ctypes.byref(p) for p in ptrs],
                                 ctypes.byref(numllv), ctypes.byref(bwtp))
        assert rc == 0
        sufp, lcpp, lcpbp, llvp = ptrs

        def grab(ptr, count, dtype):
            size = count * np.dtype(dtype).itemsize
            buf = (ctypes.c_uint8 * max(size, 1)).from_address(ptr.value)
            arr = np.frombuffer(buf, dtype=np.uint8, count=size).view(dtype).copy()
            lib().orc_free(ptr)
            return arr

        self.text = text
        self.n = n
        self.suftab = grab(sufp, n + 1, np.uint64)
        self.lcp = grab(lcpp, n + 1, np.uint64)
        self.lcpbytes = grab(lcpbp, n + 1, np.uint8)
        self.llv = grab(llvp, max(numllv.value, 0) * 2, np.uint64).reshape(-1, 2)
        self.bwt = grab(bwtp, n + 1, np.uint8)
        self.nonspecials = int(n - np.count_nonzero(text >= 254))
        self.separators = np.sort(np.flatnonzero(text == 255)).astype(np.uint64)


def index_fasta(fasta, indexname, suftab_bytes=8):
    rc = lib().orc_index_fasta(fasta.encode(), indexname.encode(), suftab_bytes)
    if rc != 0:
        raise RuntimeError("orc_index_fasta failed: %d" % rc)


def _triples(out, found):
    return out[: 3 * found].reshape(-1, 3).copy()


def linsmax(lcpbytes, llv, bwt, nonspecials, minlen, threads=1):
    """orc_linsmax; threads > 1 runs orc_linsmax_mt (same output, pthreads)."""
    llv = np.ascontiguousarray(llv, dtype=np.uint64).reshape(-1, 2)
    cap = max(16, nonspecials // 2 + 1)
    out = np.empty(3 * cap, dtype=np.uint64)
    args = (_p(lcpbytes, _u8p), llv.ctypes.data_as(ctypes.c_void_p), len(llv),
            _p(bwt, _u8p), nonspecials, minlen, _p(out, _u64p), cap)
    if threads > 1:
        found = lib().orc_linsmax_mt(*args, threads)
    else:
        found = lib().orc_linsmax(*args)
    assert found <= cap
    return _triples(out, found)


def bottomup_smax(esa, minlen):
    cap = max(16, esa.nonspecials // 2 + 1)
    out = np.empty(3 * cap, dtype=np.uint64)
    found = lib().orc_bottomup_smax(_p(esa.lcp, _u64p), _p(esa.suftab, _u64p), _p(esa.text, _u8p),
                                    esa.nonspecials, minlen, _p(out, _u64p), cap)
    assert found <= cap
    return _triples(out, found)


def bottomup_smax_tables(lcpbytes, llv, bwt, rows, minlen, cap=None):
    """orc_bottomup_smax_tables: the reference's stack traversal
    (esa-bottomup.c:116-273) over the mapped tables, rows [0, rows)."""
    llv = np.ascontiguousarray(llv, dtype=np.uint64).reshape(-1, 2)
    cap = cap or max(16, rows // 2 + 1)
    out = np.empty(3 * cap, dtype=np.uint64)
    found = lib().orc_bottomup_smax_tables(_p(lcpbytes, _u8p), llv.ctypes.data_as(ctypes.c_void_p),
                                           len(llv), _p(bwt, _u8p), rows, minlen, _p(out, _u64p),
                                           cap)
    assert found <= cap
    return _triples(out, found)


def lcp_intervals(lcpbytes, llv, nonspecials, cap):
    """orc_lcp_intervals: (lcp, lb, rb, father lcp, father lb), pop order."""
    llv = np.ascontiguousarray(llv, dtype=np.uint64).reshape(-1, 2)
    out = np.empty(5 * cap, dtype=np.uint64)
    found = lib().orc_lcp_intervals(_p(lcpbytes, _u8p), llv.ctypes.data_as(ctypes.c_void_p),
                                    len(llv), nonspecials, _p(out, _u64p), cap)
    assert found <= cap, (found, cap)
    return out[: 5 * found].reshape(-1, 5).copy()


def maxpairs_blocks(lcpbytes, llv, bwt, suftab, nonspecials, minlen, cap):
    """orc_maxpairs_blocks: maximal pairs by definition per block, unordered
    (suftab None: rows instead of positions)."""
    llv = np.ascontiguousarray(llv, dtype=np.uint64).reshape(-1, 2)
    out = np.empty(3 * cap, dtype=np.uint64)
    found = lib().orc_maxpairs_blocks(_p(lcpbytes, _u8p), llv.ctypes.data_as(ctypes.c_void_p),
                                      len(llv), _p(bwt, _u8p),
                                      _p(suftab, _u64p) if suftab is not None else None, nonspecials,
                                      minlen, _p(out, _u64p), cap)
    assert found <= cap, (found, cap)
    return _triples(out, found)


def brute_smax(text, minlen):
    text = np.ascontiguousarray(text, dtype=np.uint8)
    n = len(text)
    cap = n * n + 16
    out = np.empty(3 * cap, dtype=np.uint64)
    occ = np.empty(cap, dtype=np.uint64)
    found = lib().orc_brute_smax(_p(text, _u8p), n, minlen, _p(out, _u64p), cap, _p(occ, _u64p), cap)
    trip = _triples(out, found)
    res = []
    o = 0
    for length, first, cnt in trip:
        res.append((int(length), tuple(int(x) for x in occ[o: o + int(cnt)])))
        o += int(cnt)
    return res


def maxpairs(esa, minlen):
    pp = ctypes.c_void_p()
    cnt = lib().orc_maxpairs(_p(esa.lcp, _u64p), _p(esa.suftab, _u64p), _p(esa.text, _u8p),
                             esa.nonspecials, minlen, ctypes.byref(pp))
    if cnt == 0:
        return np.zeros((0, 3), dtype=np.uint64)
    buf = (ctypes.c_uint64 * (3 * cnt)).from_address(pp.value)
    arr = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 3).copy()
    lib().orc_free(pp)
    return arr


def bottomup_events(esa):
    """gt_esa_bottomup event stream (7-word records, see orc_bottomup_events)."""
    pp = ctypes.c_void_p()
    cnt = lib().orc_bottomup_events(_p(esa.lcp, _u64p), _p(esa.suftab, _u64p), esa.nonspecials,
                                    ctypes.byref(pp))
    if cnt == 0:
        return np.zeros((0, 7), dtype=np.uint64)
    buf = (ctypes.c_uint64 * (7 * cnt)).from_address(pp.value)
    arr = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 7).copy()
    lib().orc_free(pp)
    return arr


def bottomup_events_slots(esa):
    """orc_bottomup_events plus each event's stack slots (father, son; NONE =
    2^64-1) and the number of slots allocated -- the reference's
    GtESAVisitorInfo objects (esa-bottomup.c:20-110)."""
    pp, ps = ctypes.c_void_p(), ctypes.c_void_p()
    ns = ctypes.c_uint64()
    cnt = lib().orc_bottomup_events_slots(_p(esa.lcp, _u64p), _p(esa.suftab, _u64p),
                                          esa.nonspecials, ctypes.byref(pp), ctypes.byref(ps),
                                          ctypes.byref(ns))
    if cnt == 0:
        return np.zeros((0, 7), np.uint64), np.zeros((0, 2), np.uint64), ns.value
    ev = np.frombuffer((ctypes.c_uint64 * (7 * cnt)).from_address(pp.value),
                       dtype=np.uint64).reshape(-1, 7).copy()
    sl = np.frombuffer((ctypes.c_uint64 * (2 * cnt)).from_address(ps.value),
                       dtype=np.uint64).reshape(-1, 2).copy()
    lib().orc_free(pp)
    lib().orc_free(ps)
    return ev, sl, ns.value


def dfs_events(esa):
    """gt_depthfirstesa + elcp L/B lines (-enumlcpitvtree), orc_dfs_events."""
    pp = ctypes.c_void_p()
    cnt = lib().orc_dfs_events(_p(esa.lcp, _u64p), _p(esa.suftab, _u64p), esa.nonspecials,
                               ctypes.byref(pp))
    if cnt == 0:
        return np.zeros((0, 7), dtype=np.uint64)
    buf = (ctypes.c_uint64 * (7 * cnt)).from_address(pp.value)
    arr = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 7).copy()
    lib().orc_free(pp)
    return arr


def format_pairs(pairs, separators):
    sep = np.ascontiguousarray(separators, dtype=np.uint64)
    buf = ctypes.create_string_buffer(256)
    lines = []
    for length, p1, p2 in pairs:
        k = lib().orc_format_pair(int(length), int(p1), int(p2), _p(sep, _u64p), len(sep), buf, 256)
        if k > 0:
            lines.append(buf.value.decode())
    return lines


def smax_pairs(intervals, suftab):
    """All occurrence pairs of each smax interval, as (len, pos1, pos2)."""
    out = []
    for length, lb, rb in intervals:
        occ = [int(suftab[k]) for k in range(int(lb), int(rb) + 1)]
        for a in range(len(occ)):
            for b in range(a + 1, len(occ)):
                out.append((int(length), occ[a], occ[b]))
    return out


def pack_bwt_ref(bwt):
    """numpy restatement of the packed-BWT layout (GT_SMAX_PK_GROUPS,
    include/gt_smax_hip.h): group gi holds rows 16*(gi-1) .. +15; bit q / 16+q
    the symbol's bits 0 / 1, bit 32+q a special (>= 254, code bits 0); rows
    outside the table are zero.  Returns (groups, is_dna)."""
    bwt = np.asarray(bwt, dtype=np.uint8)
    n = len(bwt)
    ng = n // 16 + 134
    rows = np.zeros(ng * 16, dtype=np.uint8)
    valid = np.zeros(ng * 16, dtype=bool)
    rows[16: 16 + n] = bwt
    valid[16: 16 + n] = True
    sp = valid & (rows >= 254)
    b0 = (valid & ~sp & ((rows & 1) != 0)).reshape(ng, 16)
    b1 = (valid & ~sp & ((rows & 2) != 0)).reshape(ng, 16)
    s = sp.reshape(ng, 16)
    w = 1 << np.arange(16, dtype=np.uint64)
    out = ((b0 * w).sum(1).astype(np.uint64) | ((b1 * w).sum(1).astype(np.uint64) << np.uint64(16))
           | ((s * w).sum(1).astype(np.uint64) << np.uint64(32)))
    is_dna = not np.any((bwt > 3) & (bwt < 254))
    return out, is_dna


def spmitv_lines(events, text, nonspecials):
    """`gt dev sfxmap -spmitv` output (src/match/esa-spmitvs.c:25-69) from a
    gt_esa_bottomup event stream (7-word records: the oracle's or the GPU's):
    the spmitvs visitor restated in orc_spmitv, printed as
    gt_esa_spmitvs_visitor_print_results does (src/match/esa_spmitvs_visitor.c:
    203-226).  maxlen = the longest sequence (gt_encseq_max_seq_length),
    totallength = the text length with separators."""
    text = np.ascontiguousarray(text, dtype=np.uint8)
    ev = np.ascontiguousarray(events, dtype=np.uint64).reshape(-1, 7)
    n = len(text)
    seps = np.flatnonzero(text == 255)
    bounds = np.concatenate([[-1], seps, [n]])
    maxlen = int((np.diff(bounds) - 1).max()) if n else 0
    counts = np.zeros(4 * (maxlen + 1), dtype=np.uint64)
    unnec = ctypes.c_uint64()
    rc = lib().orc_spmitv(_p(ev, _u64p), len(ev), _p(text, _u8p), n, maxlen, _p(counts, _u64p),
                          ctypes.byref(unnec))
    if rc != 0:
        raise AssertionError("orc_spmitv: a reference assertion fails on this event stream")
    c = counts.reshape(-1, 4).astype(np.int64)
    lines = ["unnecessaryleaves=%d (%.2f)" % (unnec.value, unnec.value / nonspecials)]
    for idx in range(maxlen + 1):
        w, ww, nw = int(c[idx, 0]), int(c[idx, 1]), int(c[idx, 2])
        if w != 0 or nw != 0:
            lines.append("wholeleaf[%d]:num=%d (%.2f), width=%d (%.2f)"
                         % (idx, w, w / (w + nw), ww, ww / n))
    return lines
