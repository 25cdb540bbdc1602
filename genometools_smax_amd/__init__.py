"""genometools_smax_amd -- MI355X supermaximal-repeat finder behind
GenomeTools' ESA interfaces.

Host-side mirror (Python) of the pieces of the reference the smax path sits
behind.  The compute path is the HIP library lib/libgtsmax_hip.so
(csrc/smax_kernels.hip, C-ABI in include/gt_smax_hip.h); there is no CPU
fallback: every entry point raises if the library or a HIP device is missing.

  EsaIndex            mmap of a `gt suffixerator -suf -lcp -bwt` index,
                      restating Suffixarray / gt_mapsuffixarray
                      (src/match/sarr-def.h:101-126, src/match/esa-map.c:296-515)
  enumerate_smax      gt_smax_hip_enumerate_to_buffer -> (lcp, lb, rb) rows in
                      ascending lb, the order gt_esa_bottomup pops them
  SmaxPlan            device-resident plan over tables already in HBM
  repfind_smax_lines  `gt repfind -smax` output: one line per occurrence pair,
                      format of gt_simpleexactselfmatchoutput
                      (src/tools/gt_repfind.c:49-84, src/match/querymatch.c:130-190)
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GT_SMAX_LIB") or os.path.join(_HERE, "lib", "libgtsmax_hip.so")   # GT_SMAX_LIB: A/B diagnostics
BIN_DIR = os.path.join(_HERE, "bin")

PAD_FRONT = 256
PAD_BACK = 32768


class SmaxError(RuntimeError):
    """Error reported through the C-ABI's errbuf (GtError analogue)."""


class GtSmaxLlv(ctypes.Structure):
    _fields_ = [("position", ctypes.c_uint64), ("value", ctypes.c_uint64)]


class GtSmaxInput(ctypes.Structure):
    _fields_ = [
        ("lcptab", ctypes.c_void_p),
        ("llvtab", ctypes.c_void_p),
        ("numllv", ctypes.c_uint64),
        ("bwttab", ctypes.c_void_p),
        ("suftab", ctypes.c_void_p),
        ("suftab_bytes", ctypes.c_int),
        ("totallength", ctypes.c_uint64),
        ("nonspecials", ctypes.c_uint64),
    ]


class GtSmaxDevShard(ctypes.Structure):
    _fields_ = [
        ("lcp_dev", ctypes.c_void_p),
        ("bwt_dev", ctypes.c_void_p),
        ("llv_dev", ctypes.c_void_p),
        ("numllv", ctypes.c_uint64),
        ("base", ctypes.c_uint64),
        ("local_len", ctypes.c_uint64),
        ("begin", ctypes.c_uint64),
        ("end", ctypes.c_uint64),
        ("nonspecials", ctypes.c_uint64),
        ("device", ctypes.c_int),
        ("bwtpk_dev", ctypes.c_void_p),
    ]


class GtSmaxDiv(ctypes.Structure):
    _fields_ = [("seen", ctypes.c_uint64 * 4), ("dup", ctypes.c_uint64)]


class GtSmaxBoundary(ctypes.Structure):
    _fields_ = [
        ("pend_valid", ctypes.c_uint64),
        ("pend_c", ctypes.c_uint64),
        ("pend_lcp", ctypes.c_uint64),
        ("pend_div", GtSmaxDiv),
        ("head_v", ctypes.c_uint64),
        ("head_f", ctypes.c_uint64),
        ("head_next", ctypes.c_uint64),
        ("head_div", GtSmaxDiv),
        ("shard_begin", ctypes.c_uint64),
        ("shard_end", ctypes.c_uint64),
    ]


class GtMaxpairsDevInput(ctypes.Structure):
    _fields_ = [
        ("lcp_dev", ctypes.c_void_p),
        ("bwt_dev", ctypes.c_void_p),
        ("llv_dev", ctypes.c_void_p),
        ("numllv", ctypes.c_uint64),
        ("suf_dev", ctypes.c_void_p),
        ("suf_bytes", ctypes.c_int),
        ("nonspecials", ctypes.c_uint64),
        ("device", ctypes.c_int),
    ]


class GtLcpitvDevInput(ctypes.Structure):
    _fields_ = [
        ("lcp_dev", ctypes.c_void_p),
        ("llv_dev", ctypes.c_void_p),
        ("numllv", ctypes.c_uint64),
        ("suf_dev", ctypes.c_void_p),
        ("suf_bytes", ctypes.c_int),
        ("nonspecials", ctypes.c_uint64),
        ("device", ctypes.c_int),
    ]


_LEAF_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64,
                            ctypes.c_uint64, ctypes.c_uint64)
_BRANCH_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64,
                              ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64)
_ITV_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                           ctypes.c_uint64)


_TEXT_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64)


class GtLcpitvVisitor(ctypes.Structure):
    _fields_ = [("leaf_edge", _LEAF_CB), ("branching_edge", _BRANCH_CB), ("lcp_interval", _ITV_CB)]


_vp = ctypes.c_void_p
_u64 = ctypes.c_uint64
_LEAF_INFO_CB = ctypes.CFUNCTYPE(ctypes.c_int, _vp, ctypes.c_int, _u64, _u64, _vp, _u64)
_BRANCH_INFO_CB = ctypes.CFUNCTYPE(ctypes.c_int, _vp, ctypes.c_int, _u64, _u64, _vp, _u64, _u64,
                                   _u64, _vp)
_ITV_INFO_CB = ctypes.CFUNCTYPE(ctypes.c_int, _vp, _u64, _u64, _u64, _vp)
_INFO_NEW_CB = ctypes.CFUNCTYPE(_vp, _vp)
_INFO_DEL_CB = ctypes.CFUNCTYPE(None, _vp, _vp)


class GtLcpitvInfoVisitor(ctypes.Structure):
    _fields_ = [("leaf_edge", _LEAF_INFO_CB), ("branching_edge", _BRANCH_INFO_CB),
                ("lcp_interval", _ITV_INFO_CB), ("info_new", _INFO_NEW_CB),
                ("info_delete", _INFO_DEL_CB)]


class GtSmaxRecord(ctypes.Structure):
    _fields_ = [("lb", ctypes.c_uint64), ("lcp", ctypes.c_uint32), ("width", ctypes.c_uint32)]


BOUNDARY_BYTES = ctypes.sizeof(GtSmaxBoundary)
RECORD_DTYPE = np.dtype([("lb", "<u8"), ("lcp", "<u4"), ("width", "<u4")])

_lib = None


def lib():
    """The HIP library; raises (never falls back) when it is not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise SmaxError("HIP library missing: %s (run __graft_entry__.build())" % LIB_PATH)
        if (os.environ.get("GT_SMAX_DEBUG") or os.environ.get("GT_SMAX_STAMPS")) and \
                os.path.abspath(LIB_PATH) == os.path.join(_HERE, "lib", "libgtsmax_hip.so"):
            # the production library reads no diagnostic switch: say so rather
            # than run the production kernels under a diagnostic's name
            raise SmaxError("GT_SMAX_DEBUG/GT_SMAX_STAMPS need the diagnostic build: "
                            "GT_SMAX_LIB=genometools_smax_amd/lib/diag/libgtsmax_hip.so")
        # torch first: its bundled HIP runtime (soname libamdhip64.so.7) then
        # also serves this library.  Loaded the other way round, torch's
        # libtorch_hip (NEEDED libamdhip64.so, RPATH $ORIGIN) would map a
        # second HIP/HSA runtime into the process and find no GPU.
        import torch  # noqa: F401
        L = ctypes.CDLL(LIB_PATH)
        vp, u64, u32, ci = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint, ctypes.c_int
        cs, sz = ctypes.c_char_p, ctypes.c_size_t
        L.gt_smax_hip_enumerate_to_buffer.argtypes = [ctypes.POINTER(GtSmaxInput), u32, ci,
                                                      ctypes.POINTER(vp), ctypes.POINTER(u64), cs, sz]
        L.gt_smax_free.argtypes = [vp]
        L.gt_smax_release_cache.argtypes = []
        L.gt_smax_hip_prepare.argtypes = [u64, u64, ci]
        L.gt_smax_hip_prepare.restype = ci
        L.gt_smax_pack_bwt.argtypes = [vp, u64, vp]
        L.gt_smax_encode_fasta.argtypes = [ctypes.c_char_p, u64, vp, ctypes.POINTER(u64),
                                           ctypes.POINTER(u64), cs, sz]
        L.gt_smax_device_count.restype = ci
        L.gt_smax_build_id.restype = ctypes.c_char_p
        L.gt_smax_plan_scan_kernel.restype = ctypes.c_char_p
        L.gt_smax_plan_scan_kernel.argtypes = [vp]
        if hasattr(L, "gt_smax_plan_k1b_waves"):   # (older builds loaded by the A/B tools lack it)
            L.gt_smax_plan_k1b_waves.restype = ctypes.c_uint32
            L.gt_smax_plan_k1b_waves.argtypes = [vp]
        L.gt_smax_dev_alloc_table.argtypes = [ci, u64, ctypes.POINTER(vp), cs, sz]
        L.gt_smax_dev_free_table.argtypes = [ci, vp]
        L.gt_smax_plan_create.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(GtSmaxDevShard), u32, u64,
                                          cs, sz]
        L.gt_smax_plan_delete.argtypes = [vp]
        L.gt_smax_plan_run.argtypes = [vp, vp]
        L.gt_smax_plan_run_part.argtypes = [vp, ci, vp]
        L.gt_smax_plan_records.argtypes = [vp]
        L.gt_smax_plan_records.restype = vp
        L.gt_smax_plan_count_dev.argtypes = [vp]
        L.gt_smax_plan_count_dev.restype = vp
        L.gt_smax_plan_boundary_dev.argtypes = [vp]
        L.gt_smax_plan_boundary_dev.restype = vp
        L.gt_smax_plan_capacity.argtypes = [vp]
        L.gt_smax_plan_capacity.restype = u64
        L.gt_smax_plan_num_tiles.argtypes = [vp]
        L.gt_smax_plan_num_tiles.restype = u64
        L.gt_smax_plan_stitch.argtypes = [vp, vp, ci, ci, vp]
        L.gt_smax_stitch_host.argtypes = [ctypes.POINTER(GtSmaxBoundary), ci, ci, u32,
                                          ctypes.POINTER(GtSmaxRecord)]
        L.gt_smax_plan_fetch_count.argtypes = [vp, ctypes.POINTER(u64)]
        L.gt_smax_plan_fetch_triples.argtypes = [vp, vp, u64, ctypes.POINTER(u64)]
        L.gt_smax_plan_timing.argtypes = [vp, ci]
        L.gt_smax_plan_timing_stride.argtypes = [vp, ci]
        L.gt_smax_plan_timing_read.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ci)]
        L.gt_smax_plan_copy_boundary.argtypes = [vp, vp, vp]
        L.gt_smax_plan_error_bits.argtypes = [vp]
        L.gt_smax_plan_error_bits.restype = ctypes.c_uint32
        L.gt_smax_plan_deferred_tiles.argtypes = [vp]
        L.gt_smax_plan_deferred_tiles.restype = ctypes.c_uint32
        L.gt_smax_plan_debug_tiles.argtypes = [vp, vp, vp, ctypes.POINTER(ctypes.c_uint32)]
        L.gt_smax_plan_debug_windows.argtypes = [vp, vp]
        L.gt_maxpairs_hip_enumerate_to_buffer.argtypes = [ctypes.POINTER(GtSmaxInput), u32,
                                                          ctypes.POINTER(vp), ctypes.POINTER(u64), cs, sz]
        L.gt_maxpairs_plan_create.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(GtMaxpairsDevInput),
                                              u32, cs, sz]
        L.gt_maxpairs_plan_create_stream.argtypes = [ctypes.POINTER(vp),
                                                     ctypes.POINTER(GtMaxpairsDevInput), u32, vp, cs, sz]
        L.gt_maxpairs_plan_delete.argtypes = [vp]
        L.gt_maxpairs_plan_count.argtypes = [vp, vp]
        L.gt_maxpairs_plan_total.argtypes = [vp, ctypes.POINTER(u64)]
        L.gt_maxpairs_plan_emit.argtypes = [vp, vp, u64, vp]
        L.gt_maxpairs_plan_emit_ordered.argtypes = [vp, vp, u64, vp]
        L.gt_maxpairs_plan_candidates.argtypes = [vp]
        L.gt_maxpairs_plan_candidates.restype = u64
        L.gt_seqpos_map_dev.argtypes = [vp, u64, vp, u64, vp, ci, vp]
        L.gt_repfind_pairs_lines_dev.argtypes = [vp, u64, vp, u64, ci, _TEXT_CB, vp, cs, sz]
        L.gt_repfind_smax_lines.argtypes = [vp, u64, vp, u64, vp, u64, _TEXT_CB, vp, cs, sz]
        L.gt_repfind_maxpairs_lines.argtypes = [ctypes.POINTER(GtSmaxInput), u32, vp, u64, _TEXT_CB,
                                                vp, cs, sz]
        L.gt_lcpitv_hip_enumerate_to_buffer.argtypes = [ctypes.POINTER(GtSmaxInput),
                                                        ctypes.POINTER(vp), ctypes.POINTER(u64), cs, sz]
        L.gt_lcpitv_plan_create.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(GtLcpitvDevInput), cs, sz]
        L.gt_lcpitv_plan_create_stream.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(GtLcpitvDevInput),
                                                   vp, cs, sz]
        L.gt_lcpitv_plan_delete.argtypes = [vp]
        L.gt_lcpitv_plan_intervals.argtypes = [vp, ctypes.POINTER(vp)]
        L.gt_lcpitv_plan_intervals.restype = u64
        L.gt_lcpitv_plan_num_events.argtypes = [vp]
        L.gt_lcpitv_plan_num_events.restype = u64
        L.gt_lcpitv_plan_events.argtypes = [vp, vp, vp]
        L.gt_esa_bottomup_hip.argtypes = [ctypes.POINTER(GtSmaxInput), ctypes.POINTER(GtLcpitvVisitor),
                                          vp, cs, sz]
        L.gt_esa_bottomup_info_hip.argtypes = [ctypes.POINTER(GtSmaxInput),
                                               ctypes.POINTER(GtLcpitvInfoVisitor), vp, cs, sz]
        _lib = L
    return _lib


def exported_symbols():
    """Every function the include/*.h headers declare (checked by tests)."""
    import glob
    import re
    names = set()
    for hdr in sorted(glob.glob(os.path.join(os.path.dirname(_HERE), "include", "*.h"))):
        with open(hdr) as fh:
            text = fh.read()
        text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)    # comments cite reference names
        text = re.sub(r"//[^\n]*", " ", text)
        names.update(re.findall(r"\b(gt_\w+)\s*\(", text))
    return sorted(names)


def _errbuf():
    return ctypes.create_string_buffer(1024)


def _check(rc, eb):
    if rc != 0:
        raise SmaxError(eb.value.decode(errors="replace") or "gt_smax error")


# --------------------------------------------------------------- ESA index

class EsaIndex:
    """Memory-mapped gt ESA (.prj .lcp .llv .bwt [.suf]).

    Restates inputsuffixarray/gt_mapsuffixarray (src/match/esa-map.c:296-515):
    .prj keys checked as scanprjfileuintkeysviafileptr does (:55-214), table
    sizes checked against totallength+1, nonspecials = totallength -
    specialcharacters (src/match/esa-seqread.c:56-57).  The .suf width is
    inferred from its size (8 B GtUword, or 4 B from -suftabuint).
    """

    def __init__(self, indexname, need_suftab=True):
        self.indexname = indexname
        self.prj = self._read_prj(indexname + ".prj")
        p = self.prj
        for key in ("totallength", "specialcharacters", "integersize", "littleendian",
                    "readmode", "mirrored"):
            if key not in p:
                raise SmaxError("%s.prj: missing key %s" % (indexname, key))
        if p["integersize"] not in (32, 64):
            raise SmaxError("%s.prj contains illegal line defining the integer size" % indexname)
        if p["littleendian"] != 1:
            raise SmaxError("index was built on a big endian computer")
        if p["readmode"] > 3:
            raise SmaxError("illegal readmode %d" % p["readmode"])
        if p["mirrored"] > 1:
            raise SmaxError("illegal mirroring flag %d" % p["mirrored"])
        if p["readmode"] != 0 or p["mirrored"] != 0:
            raise SmaxError("smax supports forward, non-mirrored indexes only "
                            "(readmode=%d mirrored=%d)" % (p["readmode"], p["mirrored"]))
        self.totallength = n = p["totallength"]
        self.nonspecials = n - p["specialcharacters"]
        self.lcptab = self._map(".lcp", np.uint8, n + 1)
        self.bwttab = self._map(".bwt", np.uint8, n + 1)
        llvpath = indexname + ".llv"
        size = os.path.getsize(llvpath) if os.path.exists(llvpath) else 0
        if size % 16:
            raise SmaxError("%s: size %d not a multiple of 16" % (llvpath, size))
        if size:
            self.llvtab = np.memmap(llvpath, dtype=np.uint64, mode="r").reshape(-1, 2)
        else:
            self.llvtab = np.zeros((0, 2), dtype=np.uint64)
        if "largelcpvalues" in p and p["largelcpvalues"] != len(self.llvtab):
            raise SmaxError("%s.llv holds %d entries, .prj says %d"
                            % (indexname, len(self.llvtab), p["largelcpvalues"]))
        self.suftab = None
        if need_suftab and os.path.exists(indexname + ".suf"):
            ssize = os.path.getsize(indexname + ".suf")
            if ssize == 8 * (n + 1):
                self.suftab = np.memmap(indexname + ".suf", dtype=np.uint64, mode="r")
            elif ssize == 4 * (n + 1):
                self.suftab = np.memmap(indexname + ".suf", dtype=np.uint32, mode="r")
            else:
                raise SmaxError("%s.suf: number of mapped units does not match %d"
                                % (indexname, n + 1))

    def _map(self, suffix, dtype, count):
        path = self.indexname + suffix
        if not os.path.exists(path):
            raise SmaxError("cannot open file \"%s\"" % path)
        size = os.path.getsize(path)
        if size != count * np.dtype(dtype).itemsize:
            raise SmaxError("%s: number of mapped units (of size %d) = %d != %d"
                            % (path, np.dtype(dtype).itemsize, size // np.dtype(dtype).itemsize,
                               count))
        return np.memmap(path, dtype=dtype, mode="r")

    @staticmethod
    def _read_prj(path):
        if not os.path.exists(path):
            raise SmaxError("cannot open file \"%s\"" % path)
        out = {}
        with open(path) as fh:
            for line in fh:
                line = line.strip()
                if not line or line.startswith("dbfile="):
                    continue
                key, _, val = line.partition("=")
                try:
                    out[key] = float(val) if "." in val else int(val)
                except ValueError:
                    out[key] = val
        return out

    def separators(self):
        """Separator positions = sort({suftab[k]-1 : bwt[k] == 255})
        (equals the .ssp contents)."""
        if self.suftab is None:
            raise SmaxError("suftab required for sequence numbers")
        k = np.flatnonzero(np.asarray(self.bwttab) == 255)
        return np.sort(np.asarray(self.suftab)[k].astype(np.uint64) - 1)


# ------------------------------------------------------------- host-buffer API

def _check_lengths(totallength, nonspecials, lcptab=None, bwttab=None, suftab=None):
    """The C layer reads totallength+1 table entries (nonspecials+1 of the
    suffix array): refuse shorter host arrays instead of reading past them."""
    n, N = int(totallength), int(nonspecials)
    if n < 0 or N < 0 or N > n:
        raise SmaxError("bad lengths: totallength=%d nonspecials=%d" % (n, N))
    for name, tab, need in (("lcptab", lcptab, n + 1), ("bwttab", bwttab, n + 1),
                            ("suftab", suftab, N + 1)):
        if tab is not None and len(tab) < need:
            raise SmaxError("%s holds %d entries, needs %d (totallength=%d, nonspecials=%d)"
                            % (name, len(tab), need, n, N))


def enumerate_smax(lcptab, llvtab, bwttab, totallength, nonspecials, minlen, num_gpus=1):
    """All smax intervals as an (k,3) uint64 array of (lcp, lb, rb), lb ascending.

    Thin wrapper over gt_smax_hip_enumerate_to_buffer."""
    lcptab = np.ascontiguousarray(lcptab, dtype=np.uint8)
    bwttab = np.ascontiguousarray(bwttab, dtype=np.uint8)
    llvtab = np.ascontiguousarray(llvtab, dtype=np.uint64).reshape(-1, 2)
    _check_lengths(totallength, nonspecials, lcptab, bwttab)
    inp = GtSmaxInput()
    inp.lcptab = lcptab.ctypes.data
    inp.llvtab = llvtab.ctypes.data if len(llvtab) else None
    inp.numllv = len(llvtab)
    inp.bwttab = bwttab.ctypes.data
    inp.suftab = None
    inp.suftab_bytes = 0
    inp.totallength = int(totallength)
    inp.nonspecials = int(nonspecials)
    out = ctypes.c_void_p()
    cnt = ctypes.c_uint64()
    eb = _errbuf()
    rc = lib().gt_smax_hip_enumerate_to_buffer(ctypes.byref(inp), int(minlen), int(num_gpus),
                                               ctypes.byref(out), ctypes.byref(cnt), eb, len(eb))
    _check(rc, eb)
    n = cnt.value
    if n == 0:
        if out.value:
            lib().gt_smax_free(out)
        return np.zeros((0, 3), dtype=np.uint64)
    return np.asarray(_OwnedTriples(out.value, n))


class _OwnedTriples:
    """The C layer's malloc'd (k,3) uint64 triples exposed to numpy without a
    copy; freed (gt_smax_free) when the last array view goes away."""

    def __init__(self, ptr, k):
        self._ptr = ptr
        self.__array_interface__ = {"shape": (k, 3), "typestr": "<u8",
                                    "data": (ptr, False), "version": 3}

    def __del__(self):
        if self._ptr:
            lib().gt_smax_free(ctypes.c_void_p(self._ptr))
            self._ptr = None


def enumerate_maxpairs(lcptab, llvtab, bwttab, suftab, totallength, nonspecials, minlen):
    """All maximal pairs of length >= minlen as an (k,3) uint64 array of
    (len, pos1, pos2), pos1 < pos2 (gt_maxpairs_hip_enumerate_to_buffer: the
    pairs of `gt repfind -l minlen` in the reference's emission order)."""
    lcptab = np.ascontiguousarray(lcptab, dtype=np.uint8)
    bwttab = np.ascontiguousarray(bwttab, dtype=np.uint8)
    llvtab = np.ascontiguousarray(llvtab, dtype=np.uint64).reshape(-1, 2)
    suftab = np.ascontiguousarray(suftab)
    if suftab.dtype not in (np.uint32, np.uint64):
        suftab = suftab.astype(np.uint64)
    _check_lengths(totallength, nonspecials, lcptab, bwttab, suftab)
    inp = GtSmaxInput()
    inp.lcptab = lcptab.ctypes.data
    inp.llvtab = llvtab.ctypes.data if len(llvtab) else None
    inp.numllv = len(llvtab)
    inp.bwttab = bwttab.ctypes.data
    inp.suftab = suftab.ctypes.data
    inp.suftab_bytes = suftab.dtype.itemsize
    inp.totallength = int(totallength)
    inp.nonspecials = int(nonspecials)
    out = ctypes.c_void_p()
    cnt = ctypes.c_uint64()
    eb = _errbuf()
    rc = lib().gt_maxpairs_hip_enumerate_to_buffer(ctypes.byref(inp), int(minlen), ctypes.byref(out),
                                                   ctypes.byref(cnt), eb, len(eb))
    _check(rc, eb)
    n = cnt.value
    if n == 0:
        if out.value:
            lib().gt_smax_free(out)
        return np.zeros((0, 3), dtype=np.uint64)
    return np.asarray(_OwnedTriples(out.value, n))


def _text_sink():
    chunks = []

    def cb(_data, text, nbytes):
        chunks.append(ctypes.string_at(text, nbytes))
        return 0
    return chunks, _TEXT_CB(cb)


def format_smax_lines(records, occpos, separators):
    """`gt repfind -smax` pair lines formatted on the GPU
    (gt_repfind_smax_lines): records is a RECORD_DTYPE array whose lb indexes
    occpos (text positions); returns the text as bytes."""
    rec = np.ascontiguousarray(records, dtype=RECORD_DTYPE)
    occ = np.ascontiguousarray(occpos, dtype=np.uint64)
    sep = np.ascontiguousarray(separators, dtype=np.uint64)
    chunks, cb = _text_sink()
    eb = _errbuf()
    _check(lib().gt_repfind_smax_lines(rec.ctypes.data, len(rec), occ.ctypes.data, len(occ),
                                       sep.ctypes.data, len(sep), cb, None, eb, len(eb)), eb)
    return b"".join(chunks)


def repfind_pairs_lines_dev(pairs_ptr, count, sep_ptr, nsep, device=0):
    """Device (len, pos1, pos2) triples -> gt repfind lines (bytes)."""
    chunks, cb = _text_sink()
    eb = _errbuf()
    _check(lib().gt_repfind_pairs_lines_dev(pairs_ptr, int(count), sep_ptr, int(nsep), int(device),
                                            cb, None, eb, len(eb)), eb)
    return b"".join(chunks)


class LcpitvPlan:
    """Device-resident lcp-interval tree and visitor event stream
    (gt_lcpitv_plan_*)."""

    def __init__(self, lcp_ptr, llv_ptr, numllv, suf_ptr, suf_bytes, nonspecials, device=0,
                 stream=None):
        """stream=None: gt_lcpitv_plan_create (synchronous); else the tree is
        built on that stream (gt_lcpitv_plan_create_stream)."""
        inp = GtLcpitvDevInput()
        inp.lcp_dev, inp.llv_dev, inp.numllv = lcp_ptr, llv_ptr, numllv
        inp.suf_dev, inp.suf_bytes = suf_ptr, suf_bytes
        inp.nonspecials, inp.device = nonspecials, device
        self._p = ctypes.c_void_p()
        eb = _errbuf()
        if stream is None:
            rc = lib().gt_lcpitv_plan_create(ctypes.byref(self._p), ctypes.byref(inp), eb, len(eb))
        else:
            rc = lib().gt_lcpitv_plan_create_stream(ctypes.byref(self._p), ctypes.byref(inp), stream,
                                                    eb, len(eb))
        _check(rc, eb)
        self.device = device

    def intervals(self):
        """(count, device pointer) of the pop-ordered 5-word records."""
        ptr = ctypes.c_void_p()
        n = lib().gt_lcpitv_plan_intervals(self._p, ctypes.byref(ptr))
        return n, ptr.value

    def num_events(self):
        return lib().gt_lcpitv_plan_num_events(self._p)

    def events(self, out_ptr, stream=0):
        if lib().gt_lcpitv_plan_events(self._p, out_ptr, stream) != 0:
            raise SmaxError("gt_lcpitv_plan_events failed")

    def close(self):
        if self._p:
            lib().gt_lcpitv_plan_delete(self._p)
            self._p = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MaxpairsPlan:
    """Device-resident maximal pairs over HBM tables (gt_maxpairs_plan_*)."""

    def __init__(self, lcp_ptr, bwt_ptr, llv_ptr, numllv, suf_ptr, suf_bytes, nonspecials, minlen,
                 device=0, stream=None):
        """stream: build on that stream (gt_maxpairs_plan_create_stream)."""
        inp = GtMaxpairsDevInput()
        inp.lcp_dev, inp.bwt_dev, inp.llv_dev = lcp_ptr, bwt_ptr, llv_ptr
        inp.numllv, inp.suf_dev, inp.suf_bytes = numllv, suf_ptr, suf_bytes
        inp.nonspecials, inp.device = nonspecials, device
        self._p = ctypes.c_void_p()
        eb = _errbuf()
        if stream is None:
            rc = lib().gt_maxpairs_plan_create(ctypes.byref(self._p), ctypes.byref(inp), int(minlen),
                                               eb, len(eb))
        else:
            rc = lib().gt_maxpairs_plan_create_stream(ctypes.byref(self._p), ctypes.byref(inp),
                                                      int(minlen), stream, eb, len(eb))
        _check(rc, eb)
        self.device = device

    def count(self, stream=0):
        if lib().gt_maxpairs_plan_count(self._p, stream) != 0:
            raise SmaxError("gt_maxpairs_plan_count failed")

    def total(self):
        t = ctypes.c_uint64()
        if lib().gt_maxpairs_plan_total(self._p, ctypes.byref(t)) != 0:
            raise SmaxError("gt_maxpairs_plan_total failed")
        return t.value

    def candidates(self):
        """Rows with a non-empty walk (LCP >= minlen), fixed at plan creation."""
        return int(lib().gt_maxpairs_plan_candidates(self._p))

    def emit(self, out_ptr, capacity, stream=0):
        if lib().gt_maxpairs_plan_emit(self._p, out_ptr, int(capacity), stream) != 0:
            raise SmaxError("gt_maxpairs_plan_emit failed")

    def emit_ordered(self, out_ptr, capacity, stream=0):
        """Pairs in the reference's emission order (synchronises)."""
        if lib().gt_maxpairs_plan_emit_ordered(self._p, out_ptr, int(capacity), stream) != 0:
            raise SmaxError("gt_maxpairs_plan_emit_ordered failed")

    def close(self):
        if self._p:
            lib().gt_maxpairs_plan_delete(self._p)
            self._p = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def seqpos_map_dev(sep_ptr, nsep, pairs_ptr, count, out_ptr, device=0, stream=0):
    """(len, pos1, pos2) -> (len, seqnum1, relpos1, seqnum2, relpos2) on the GPU."""
    if lib().gt_seqpos_map_dev(sep_ptr, int(nsep), pairs_ptr, int(count), out_ptr, device, stream) != 0:
        raise SmaxError("gt_seqpos_map_dev failed")


def _input(lcptab, llvtab, bwttab, suftab, totallength, nonspecials):
    keep = []
    lcptab = np.ascontiguousarray(lcptab, dtype=np.uint8)
    llvtab = np.ascontiguousarray(llvtab, dtype=np.uint64).reshape(-1, 2)
    _check_lengths(totallength, nonspecials, lcptab, bwttab, suftab)
    keep += [lcptab, llvtab]
    inp = GtSmaxInput()
    inp.lcptab = lcptab.ctypes.data
    inp.llvtab = llvtab.ctypes.data if len(llvtab) else None
    inp.numllv = len(llvtab)
    if bwttab is not None:
        bwttab = np.ascontiguousarray(bwttab, dtype=np.uint8)
        keep.append(bwttab)
        inp.bwttab = bwttab.ctypes.data
    if suftab is not None:
        suftab = np.ascontiguousarray(suftab)
        if suftab.dtype not in (np.uint32, np.uint64):
            suftab = suftab.astype(np.uint64)
        keep.append(suftab)
        inp.suftab = suftab.ctypes.data
        inp.suftab_bytes = suftab.dtype.itemsize
    inp.totallength = int(totallength)
    inp.nonspecials = int(nonspecials)
    return inp, keep


def enumerate_lcp_intervals(lcptab, llvtab, totallength, nonspecials):
    """Every lcp-interval of depth > 0 with its father, bottom-up (pop)
    order: (k,5) uint64 of (lcp, lb, rb, fatherlcp, fatherlb)
    (gt_lcpitv_hip_enumerate_to_buffer)."""
    inp, keep = _input(lcptab, llvtab, None, None, totallength, nonspecials)
    out = ctypes.c_void_p()
    cnt = ctypes.c_uint64()
    eb = _errbuf()
    _check(lib().gt_lcpitv_hip_enumerate_to_buffer(ctypes.byref(inp), ctypes.byref(out),
                                                   ctypes.byref(cnt), eb, len(eb)), eb)
    n = cnt.value
    if n == 0:
        return np.zeros((0, 5), dtype=np.uint64)
    buf = (ctypes.c_uint64 * (5 * n)).from_address(out.value)
    arr = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 5).copy()
    lib().gt_smax_free(out)
    return arr


def esa_bottomup(lcptab, llvtab, suftab, totallength, nonspecials, leaf_edge=None,
                 branching_edge=None, lcp_interval=None):
    """gt_esa_bottomup over the GPU lcp-interval tree (gt_esa_bottomup_hip):
    leaf_edge(firstsucc, fd, flb, leafnumber), branching_edge(firstsucc, fd,
    flb, sd, slb, srb), lcp_interval(lcp, lb, rb); a truthy return stops."""
    inp, keep = _input(lcptab, llvtab, None, suftab, totallength, nonspecials)
    v = GtLcpitvVisitor()
    cbs = []
    if leaf_edge is not None:
        cbs.append(_LEAF_CB(lambda d, f, fd, flb, leaf: int(bool(leaf_edge(f, fd, flb, leaf)))))
        v.leaf_edge = cbs[-1]
    if branching_edge is not None:
        cbs.append(_BRANCH_CB(lambda d, f, fd, flb, sd, slb, srb:
                              int(bool(branching_edge(f, fd, flb, sd, slb, srb)))))
        v.branching_edge = cbs[-1]
    if lcp_interval is not None:
        cbs.append(_ITV_CB(lambda d, lcp, lb, rb: int(bool(lcp_interval(lcp, lb, rb)))))
        v.lcp_interval = cbs[-1]
    eb = _errbuf()
    _check(lib().gt_esa_bottomup_hip(ctypes.byref(inp), ctypes.byref(v), None, eb, len(eb)), eb)


def esa_bottomup_info(lcptab, llvtab, suftab, totallength, nonspecials, info_new,
                      info_delete=None, leaf_edge=None, branching_edge=None, lcp_interval=None):
    """gt_esa_bottomup with per-node visitor state (gt_esa_bottomup_info_hip):
    info_new() -> a non-zero int handle (the GtESAVisitorInfo), info_delete(h);
    leaf_edge(firstsucc, fd, flb, finfo, leafnumber), branching_edge(firstsucc,
    fd, flb, finfo, sd, slb, srb, sinfo), lcp_interval(lcp, lb, rb, info), with
    the handles (sinfo 0 for none); a truthy return stops."""
    inp, keep = _input(lcptab, llvtab, None, suftab, totallength, nonspecials)
    v = GtLcpitvInfoVisitor()
    cbs = [_INFO_NEW_CB(lambda d: int(info_new()))]
    v.info_new = cbs[-1]
    if info_delete is not None:
        cbs.append(_INFO_DEL_CB(lambda x, d: info_delete(x or 0)))
        v.info_delete = cbs[-1]
    if leaf_edge is not None:
        cbs.append(_LEAF_INFO_CB(lambda d, f, fd, flb, fi, leaf:
                                 int(bool(leaf_edge(f, fd, flb, fi or 0, leaf)))))
        v.leaf_edge = cbs[-1]
    if branching_edge is not None:
        cbs.append(_BRANCH_INFO_CB(lambda d, f, fd, flb, fi, sd, slb, srb, si:
                                   int(bool(branching_edge(f, fd, flb, fi or 0, sd, slb, srb,
                                                           si or 0)))))
        v.branching_edge = cbs[-1]
    if lcp_interval is not None:
        cbs.append(_ITV_INFO_CB(lambda d, lcp, lb, rb, i: int(bool(lcp_interval(lcp, lb, rb, i or 0)))))
        v.lcp_interval = cbs[-1]
    eb = _errbuf()
    _check(lib().gt_esa_bottomup_info_hip(ctypes.byref(inp), ctypes.byref(v), None, eb, len(eb)), eb)


def enumerate_index(index, minlen, num_gpus=1):
    return enumerate_smax(index.lcptab, index.llvtab, index.bwttab, index.totallength,
                          index.nonspecials, minlen, num_gpus)


# ------------------------------------------------------------------ output

def _seqnum(sep, p):
    return np.searchsorted(sep, p, side="left")


def repfind_smax_lines(intervals, suftab, separators):
    """`gt repfind`-format lines for every occurrence pair of each interval.

    Pairs are emitted per interval in occurrence order; each line orders
    pos1 < pos2 and maps both to (seqnum, relpos) as
    gt_simpleexactselfmatchoutput does (src/tools/gt_repfind.c:49-84).  The
    occurrence positions are gathered from suftab here; pairs and text are
    generated on the GPU (format_smax_lines)."""
    itv = np.asarray(intervals, dtype=np.uint64).reshape(-1, 3)
    if len(itv) == 0:
        return []
    width = (itv[:, 2] - itv[:, 1] + 1).astype(np.int64)
    starts = np.concatenate([[0], np.cumsum(width)[:-1]]).astype(np.int64)
    rows = np.repeat(itv[:, 1].astype(np.int64) - starts, width) + np.arange(int(width.sum()))
    occ = np.asarray(suftab)[rows].astype(np.uint64)
    rec = np.empty(len(itv), dtype=RECORD_DTYPE)
    rec["lb"], rec["lcp"], rec["width"] = starts, itv[:, 0], width
    return format_smax_lines(rec, occ, separators).decode().splitlines()


# ------------------------------------------------------- device-resident API

class DeviceTable:
    """Padded device byte table (gt_smax_dev_alloc_table)."""

    def __init__(self, device, length):
        self.device = device
        self.length = int(length)
        p = ctypes.c_void_p()
        eb = _errbuf()
        _check(lib().gt_smax_dev_alloc_table(device, self.length, ctypes.byref(p), eb, len(eb)), eb)
        self.ptr = p.value

    def free(self):
        if self.ptr:
            lib().gt_smax_dev_free_table(self.device, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class SmaxPlan:
    """One shard's smax pass over device-resident tables (gt_smax_plan_*).

    lcp_ptr/bwt_ptr are device pointers laid out as GtSmaxDevShard requires
    (DeviceTable, or torch tensors with PAD_FRONT/PAD_BACK slack).  Every
    stream handed to run / run_part / stitch / copy_boundary must stay alive
    until close(): the delete fences the plan's buffers on those streams
    (include/gt_smax_hip.h, gt_smax_plan_delete)."""

    def __init__(self, lcp_ptr, bwt_ptr, llv_ptr, numllv, base, local_len, begin, end,
                 nonspecials, minlen, device=0, capacity=0, bwtpk_ptr=None):
        sh = GtSmaxDevShard()
        sh.lcp_dev, sh.bwt_dev, sh.llv_dev = lcp_ptr, bwt_ptr, llv_ptr
        sh.bwtpk_dev = bwtpk_ptr
        sh.numllv, sh.base, sh.local_len = int(numllv), int(base), int(local_len)
        sh.begin, sh.end, sh.nonspecials, sh.device = int(begin), int(end), int(nonspecials), device
        self.shard = sh
        self.minlen = int(minlen)
        p = ctypes.c_void_p()
        eb = _errbuf()
        _check(lib().gt_smax_plan_create(ctypes.byref(p), ctypes.byref(sh), self.minlen,
                                         int(capacity), eb, len(eb)), eb)
        self.plan = p.value

    def run(self, stream=0):
        if lib().gt_smax_plan_run(self.plan, stream or None) != 0:
            raise SmaxError("gt_smax_plan_run failed")

    def run_part(self, part, stream=0):
        """Part 0: the scan (boundary record final); part 1: the compaction."""
        if lib().gt_smax_plan_run_part(self.plan, int(part), stream or None) != 0:
            raise SmaxError("gt_smax_plan_run_part(%d) failed" % part)

    def stitch(self, all_boundaries_ptr, nshards, shard_index, stream=0):
        if lib().gt_smax_plan_stitch(self.plan, all_boundaries_ptr, nshards, shard_index,
                                     stream or None) != 0:
            raise SmaxError("gt_smax_plan_stitch failed")

    @property
    def records_ptr(self):
        return lib().gt_smax_plan_records(self.plan)

    @property
    def count_ptr(self):
        return lib().gt_smax_plan_count_dev(self.plan)

    @property
    def boundary_ptr(self):
        return lib().gt_smax_plan_boundary_dev(self.plan)

    @property
    def capacity(self):
        return lib().gt_smax_plan_capacity(self.plan)

    @property
    def num_tiles(self):
        return lib().gt_smax_plan_num_tiles(self.plan)

    def enable_timing(self, nslots, stride=1):
        """Record hipEvents around the scan kernel of every stride-th of the
        next runs (nslots of them)."""
        if lib().gt_smax_plan_timing(self.plan, int(nslots)) != 0:
            raise SmaxError("gt_smax_plan_timing failed")
        if lib().gt_smax_plan_timing_stride(self.plan, int(stride)) != 0:
            raise SmaxError("gt_smax_plan_timing_stride failed")

    def kernel_ms(self):
        """(sum of scan-kernel milliseconds, launches timed)."""
        ms = ctypes.c_double()
        n = ctypes.c_int()
        if lib().gt_smax_plan_timing_read(self.plan, ctypes.byref(ms), ctypes.byref(n)) != 0:
            raise SmaxError("gt_smax_plan_timing_read failed")
        return ms.value, n.value

    def boundary_tensor(self):
        """The plan's device boundary record (GtSmaxBoundary, BOUNDARY_BYTES)
        as a zero-copy torch uint8 tensor: final after run_part(0), so it can
        be a collective's send buffer directly (no copy_boundary launch)."""
        import torch

        class _Dev:
            pass
        d = _Dev()
        d.__cuda_array_interface__ = {"shape": (BOUNDARY_BYTES,), "typestr": "|u1",
                                      "data": (int(self.boundary_ptr), False), "version": 3}
        t = torch.as_tensor(d, device="cuda")
        if t.data_ptr() != int(self.boundary_ptr):
            raise SmaxError("boundary_tensor: torch copied the boundary record")
        return t

    def copy_boundary(self, dst_ptr, stream=0):
        if lib().gt_smax_plan_copy_boundary(self.plan, dst_ptr, stream or None) != 0:
            raise SmaxError("gt_smax_plan_copy_boundary failed")

    def error_bits(self):
        return lib().gt_smax_plan_error_bits(self.plan)

    def scan_kernel(self):
        """Name of the K1 variant this plan launches (gt_smax_plan_scan_kernel)."""
        return lib().gt_smax_plan_scan_kernel(self.plan).decode()

    def k1b_waves(self):
        """Waves per K1b workgroup of this plan (gt_smax_plan_k1b_waves)."""
        return lib().gt_smax_plan_k1b_waves(self.plan)

    def deferred_tiles(self):
        return lib().gt_smax_plan_deferred_tiles(self.plan)

    def debug_tiles(self):
        """Diagnostic: (per-tile counts, deferred tile ids) of the last run."""
        import numpy as np
        counts = np.zeros(self.num_tiles, dtype=np.uint32)
        deferred = np.zeros(self.num_tiles, dtype=np.uint32)
        n = ctypes.c_uint32()
        if lib().gt_smax_plan_debug_tiles(self.plan, counts.ctypes.data, deferred.ctypes.data,
                                          ctypes.byref(n)) != 0:
            raise SmaxError("gt_smax_plan_debug_tiles failed")
        return counts, deferred[: n.value].copy()

    def debug_windows(self):
        """Diagnostic: the plan's per-tile .llv window words, (num_tiles, 2)
        uint32 (gt_smax_plan_debug_windows)."""
        import numpy as np
        w = np.zeros((self.num_tiles, 2), dtype=np.uint32)
        if lib().gt_smax_plan_debug_windows(self.plan, w.ctypes.data) != 0:
            raise SmaxError("gt_smax_plan_debug_windows failed")
        return w

    def fetch_count(self):
        c = ctypes.c_uint64()
        if lib().gt_smax_plan_fetch_count(self.plan, ctypes.byref(c)) != 0:
            raise SmaxError("gt_smax_plan_fetch_count failed")
        return c.value

    def fetch_triples(self):
        """The plan's records (after run / stitch) as an (k,3) uint64 array of
        (lcp, lb, rb), ascending lb (gt_smax_plan_fetch_triples)."""
        k = self.fetch_count()
        out = np.empty((max(k, 1), 3), dtype=np.uint64)
        c = ctypes.c_uint64()
        if lib().gt_smax_plan_fetch_triples(self.plan, out.ctypes.data, k, ctypes.byref(c)) != 0:
            raise SmaxError("gt_smax_plan_fetch_triples failed (%d records, capacity %d)"
                            % (c.value, self.capacity))
        return out[: c.value]

    def close(self):
        if self.plan:
            lib().gt_smax_plan_delete(self.plan)
            self.plan = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def pk_groups(local_len):
    """GT_SMAX_PK_GROUPS: u64 groups of a packed BWT of local_len rows."""
    return int(local_len) // 16 + 134


def pack_bwt(bwt):
    """Host packing of a DNA BWT (gt_smax_pack_bwt): (groups, is_dna)."""
    bwt = np.ascontiguousarray(bwt, dtype=np.uint8)
    out = np.zeros(pk_groups(len(bwt)), dtype=np.uint64)
    rc = lib().gt_smax_pack_bwt(bwt.ctypes.data, len(bwt), out.ctypes.data)
    return out, rc == 0


def encode_fasta(buf):
    """FASTA bytes -> (encoded text, number of sequences): gt_smax_encode_fasta
    (the GPU suffixerator's host-side reader; no GPU involved)."""
    buf = bytes(buf)
    out = np.empty(len(buf) + 1, dtype=np.uint8)
    n, ns = ctypes.c_uint64(), ctypes.c_uint64()
    eb = _errbuf()
    _check(lib().gt_smax_encode_fasta(buf, len(buf), out.ctypes.data, ctypes.byref(n), ctypes.byref(ns),
                                      eb, len(eb)), eb)
    return out[: n.value].copy(), ns.value


def release_cache():
    """Frees the runtime's cached device and pinned buffers."""
    lib().gt_smax_release_cache()


def prepare(totallength, nonspecials, num_gpus=1):
    """gt_smax_hip_prepare: asynchronous warm-up of the devices, staging ring
    and device buffers for a first enumerate_smax call over an index of
    these sizes; the next call waits for it."""
    if lib().gt_smax_hip_prepare(int(totallength), int(nonspecials), int(num_gpus)) != 0:
        raise SmaxError("gt_smax_hip_prepare: cannot start the warm-up thread")


def stitch_host(boundaries, shard_index, minlen):
    """Host form of the boundary stitch (pure function of the records)."""
    arr = (GtSmaxBoundary * len(boundaries))(*boundaries)
    rec = GtSmaxRecord()
    ok = lib().gt_smax_stitch_host(arr, len(boundaries), shard_index, int(minlen), ctypes.byref(rec))
    if ok:
        return (int(rec.lcp), int(rec.lb), int(rec.lb) + int(rec.width) - 1)
    return None


def device_count():
    return lib().gt_smax_device_count()


def build_id():
    """Hash of the scan kernels' sources and flags (gt_smax_build_id)."""
    return lib().gt_smax_build_id().decode()


# ------------------------------------------------------- ESA construction (F1)

class GtSmaxEsaDev(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int),
        ("totallength", ctypes.c_uint64),
        ("nonspecials", ctypes.c_uint64),
        ("numllv", ctypes.c_uint64),
        ("maxbranchdepth", ctypes.c_uint64),
        ("averagelcp", ctypes.c_double),
        ("sort_rounds", ctypes.c_int),
        ("lcptab_dev", ctypes.c_void_p),
        ("bwttab_dev", ctypes.c_void_p),
        ("llvtab_dev", ctypes.c_void_p),
        ("suftab_dev", ctypes.c_void_p),
        ("bwtpk_dev", ctypes.c_void_p),
    ]


def _esa_lib():
    L = lib()
    if not getattr(L, "_esa_ready", False):
        vp, u64, ci, cs, sz = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t
        L.gt_smax_esa_build.argtypes = [ci, vp, u64, ci, ctypes.POINTER(GtSmaxEsaDev), cs, sz]
        L.gt_smax_esa_download.argtypes = [ctypes.POINTER(GtSmaxEsaDev), vp, vp, vp, vp, cs, sz]
        L.gt_smax_esa_release.argtypes = [ctypes.POINTER(GtSmaxEsaDev)]
        L.gt_smax_esa_download_packed.argtypes = [ctypes.POINTER(GtSmaxEsaDev), vp, cs, sz]
        L.gt_smax_synth_total_length.argtypes = [ci, u64, ctypes.POINTER(u64)]
        L.gt_smax_synth_generate.argtypes = [ci, u64, u64, vp, u64, ctypes.POINTER(u64), ci]
        L._esa_ready = True
    return L


class DeviceEsa:
    """Enhanced suffix array built in HBM by gt_smax_esa_build (the
    `gt suffixerator -suf -lcp -bwt` replacement for the smax inputs)."""

    def __init__(self, text, device=0, keep_suftab=False):
        text = np.ascontiguousarray(text, dtype=np.uint8)
        self.esa = GtSmaxEsaDev()
        eb = _errbuf()
        _check(_esa_lib().gt_smax_esa_build(device, text.ctypes.data, len(text), int(keep_suftab),
                                            ctypes.byref(self.esa), eb, len(eb)), eb)
        self.device = device
        self.totallength = self.esa.totallength
        self.nonspecials = self.esa.nonspecials
        self.numllv = self.esa.numllv

    def download(self, suftab=False):
        m = self.totallength + 1
        lcp = np.empty(m, dtype=np.uint8)
        bwt = np.empty(m, dtype=np.uint8)
        llv = np.empty((max(self.numllv, 1), 2), dtype=np.uint64)
        suf = np.empty(m, dtype=np.uint64) if suftab else None
        eb = _errbuf()
        _check(_esa_lib().gt_smax_esa_download(ctypes.byref(self.esa), lcp.ctypes.data, bwt.ctypes.data,
                                               llv.ctypes.data, suf.ctypes.data if suftab else None,
                                               eb, len(eb)), eb)
        return {"lcptab": lcp, "bwttab": bwt, "llvtab": llv[: self.numllv], "suftab": suf}

    def plan(self, minlen, begin=None, end=None, capacity=0, packed=True):
        """Single-shard (or sub-range) smax plan over the device tables: the
        builder's packed BWT (packed=False: the byte BWT, which the plan then
        packs itself at plan time)."""
        N = self.nonspecials
        begin = 1 if begin is None else begin
        end = N if end is None else end
        return SmaxPlan(self.esa.lcptab_dev, self.esa.bwttab_dev, self.esa.llvtab_dev, self.numllv,
                        0, self.totallength + 1, begin, end, N, minlen, self.device, capacity,
                        bwtpk_ptr=self.esa.bwtpk_dev if packed else None)

    def packed_bwt(self):
        """The builder's packed BWT groups (GT_SMAX_PK_GROUPS) on the host."""
        out = np.empty(pk_groups(self.totallength + 1), dtype=np.uint64)
        eb = _errbuf()
        _check(_esa_lib().gt_smax_esa_download_packed(ctypes.byref(self.esa), out.ctypes.data,
                                                      eb, len(eb)), eb)
        return out

    def maxpairs_plan(self, minlen, stream=None):
        """Maximal pairs over the device tables (needs keep_suftab=True)."""
        if not self.esa.suftab_dev:
            raise SmaxError("maxpairs needs the suffix array: build with keep_suftab=True")
        return MaxpairsPlan(self.esa.lcptab_dev, self.esa.bwttab_dev, self.esa.llvtab_dev, self.numllv,
                            self.esa.suftab_dev, 4, self.nonspecials, minlen, self.device, stream)

    def lcpitv_plan(self, stream=None):
        """lcp-interval tree + visitor events over the device tables."""
        return LcpitvPlan(self.esa.lcptab_dev, self.esa.llvtab_dev, self.numllv,
                          self.esa.suftab_dev or None, 4, self.nonspecials, self.device, stream)

    def release(self):
        if self.esa.lcptab_dev:
            _esa_lib().gt_smax_esa_release(ctypes.byref(self.esa))

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


class GtSmaxEsa64Dev(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int),
        ("totallength", ctypes.c_uint64),
        ("nonspecials", ctypes.c_uint64),
        ("row_lo", ctypes.c_uint64),
        ("row_hi", ctypes.c_uint64),
        ("numllv", ctypes.c_uint64),
        ("maxbranchdepth", ctypes.c_uint64),
        ("averagelcp", ctypes.c_double),
        ("sort_rounds", ctypes.c_int),
        ("batches", ctypes.c_int),
        ("lcptab_dev", ctypes.c_void_p),
        ("bwttab_dev", ctypes.c_void_p),
        ("bwtpk_dev", ctypes.c_void_p),
        ("llvtab_dev", ctypes.c_void_p),
        ("suftab_dev", ctypes.c_void_p),
    ]


def _esa64_lib():
    L = _esa_lib()
    if not getattr(L, "_esa64_ready", False):
        vp, u64, ci, cs, sz = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t
        L.gt_smax_esa64_build.argtypes = [ci, vp, u64, u64, u64, ci, u64, ctypes.POINTER(GtSmaxEsa64Dev),
                                          cs, sz]
        L.gt_smax_esa64_download.argtypes = [ctypes.POINTER(GtSmaxEsa64Dev), vp, vp, vp, vp, vp, cs, sz]
        L.gt_smax_esa64_release.argtypes = [ctypes.POINTER(GtSmaxEsa64Dev)]
        L._esa64_ready = True
    return L


class DeviceEsa64:
    """Rows [row_lo, row_hi) of a GPU-built ESA of any length
    (gt_smax_esa64_build: 64-bit suffix array, bucketed, range-restricted)."""

    def __init__(self, text, device=0, row_lo=0, row_hi=0, keep_suftab=False, batch_max=0):
        text = np.ascontiguousarray(text, dtype=np.uint8)
        self.esa = GtSmaxEsa64Dev()
        eb = _errbuf()
        _check(_esa64_lib().gt_smax_esa64_build(device, text.ctypes.data, len(text), int(row_lo),
                                                int(row_hi), int(keep_suftab), int(batch_max),
                                                ctypes.byref(self.esa), eb, len(eb)), eb)
        self.device = device
        self.totallength = self.esa.totallength
        self.nonspecials = self.esa.nonspecials
        self.numllv = self.esa.numllv
        self.row_lo, self.row_hi = self.esa.row_lo, self.esa.row_hi

    def download(self, suftab=False):
        L = self.row_hi - self.row_lo
        lcp = np.empty(L, dtype=np.uint8)
        bwt = np.empty(L, dtype=np.uint8)
        llv = np.empty((max(self.numllv, 1), 2), dtype=np.uint64)
        pk = np.empty(pk_groups(L), dtype=np.uint64)
        suf = np.empty(L, dtype=np.uint64) if suftab else None
        eb = _errbuf()
        _check(_esa64_lib().gt_smax_esa64_download(ctypes.byref(self.esa), lcp.ctypes.data,
                                                   bwt.ctypes.data, llv.ctypes.data,
                                                   suf.ctypes.data if suftab else None, pk.ctypes.data,
                                                   eb, len(eb)), eb)
        return {"lcptab": lcp, "bwttab": bwt, "llvtab": llv[: self.numllv], "suftab": suf,
                "bwtpk": pk}

    def plan(self, minlen, begin=None, end=None, capacity=0, packed=True):
        """smax plan over rows [begin, end) (default: all the rows held may
        own: the tables must hold LCP[begin-1 .. end])."""
        N = self.nonspecials
        begin = max(1, self.row_lo + 1) if begin is None else begin
        end = min(N, self.row_hi - 1) if end is None else end
        return SmaxPlan(self.esa.lcptab_dev, self.esa.bwttab_dev, self.esa.llvtab_dev, self.numllv,
                        self.row_lo, self.row_hi - self.row_lo, begin, end, N, minlen, self.device,
                        capacity, bwtpk_ptr=self.esa.bwtpk_dev if packed else None)

    def release(self):
        if self.esa.lcptab_dev:
            _esa64_lib().gt_smax_esa64_release(ctypes.byref(self.esa))

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


SYNTH_KINDS = {"uniform": 0, "human": 1, "plant": 2}


def synth_genome(kind, bases, seed, threads=None):
    """Deterministic synthetic genome (encoded symbols) -- gt_smax_synth_generate."""
    k = SYNTH_KINDS[kind] if isinstance(kind, str) else int(kind)
    n = ctypes.c_uint64()
    if _esa_lib().gt_smax_synth_total_length(k, int(bases), ctypes.byref(n)) != 0:
        raise SmaxError("bad synthetic genome request")
    out = np.empty(n.value, dtype=np.uint8)
    threads = threads or min(16, os.cpu_count() or 1)
    if _esa_lib().gt_smax_synth_generate(k, int(bases), int(seed), out.ctypes.data, n.value,
                                         ctypes.byref(n), int(threads)) != 0:
        raise SmaxError("synthetic genome generation failed")
    return out
