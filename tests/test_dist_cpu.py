"""Multi-rank (world_size 2 and 3, gloo on CPU) test of the sharded smax path's
exchange step.

Each rank owns a suffix-array range, computes on the host what K0/K1 compute
on its GPU for that range -- the plateaus it resolves locally and its
152-byte boundary record (tail plateau still open at the shard end, head run
at the shard start) -- all-gathers the boundary records over gloo exactly as
bench.py does over RCCL, and resolves the spanning plateaus with the
library's stitch (gt_smax_stitch_host, the host build of the stitch kernel).
The union over ranks must equal the oracle's single-shard answer.  The
splits are placed inside plateaus, including a shard that lies entirely
inside one (passthrough).  No GPU: the C library is only loaded, its stitch
is host code.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import genometools_smax_amd as G
import oracle_lib as O
from conftest import oracle_esa


def _exact_lcp(esa):
    N = esa.nonspecials
    L = esa.lcp[: N + 1].astype(np.int64).copy()
    L[0] = 0
    L[N] = 0
    return L


def _seen_add(seen, c):
    """seen: list of 4 ints; returns True on a duplicate symbol < 254."""
    if c >= 254:
        return False
    w, bit = c >> 6, 1 << (c & 63)
    if seen[w] & bit:
        return True
    seen[w] |= bit
    return False


def shard_view(L, B, N, begin, end, minlen):
    """Host restatement of one shard's K0+K1 outputs: locally resolved
    intervals (lcp, lb, rb) and the boundary record."""
    local = []
    b = G.GtSmaxBoundary()
    b.shard_begin, b.shard_end = begin, end
    for c in range(begin, end):
        l = int(L[c])
        if l < minlen or l <= L[c - 1]:
            continue
        j = c
        while j + 1 < end and L[j + 1] == l:
            j += 1
        if j + 1 == end and end < N and L[end] == l:        # runs into the next shard
            seen = [0, 0, 0, 0]
            if not any(_seen_add(seen, int(B[k])) for k in range(c - 1, end)):
                b.pend_valid, b.pend_c, b.pend_lcp = 1, c, l
                for w in range(4):
                    b.pend_div.seen[w] = seen[w]
            continue
        if L[j + 1] < l:
            seen = [0, 0, 0, 0]
            if not any(_seen_add(seen, int(B[k])) for k in range(c - 1, j + 1)):
                local.append((l, c - 1, j))
    v = int(L[begin])
    b.head_v = v
    seen = [0, 0, 0, 0]
    f, nxt, dup = 2**64 - 1, 0, 0
    if v >= minlen and begin < end:
        g = begin
        while True:
            if _seen_add(seen, int(B[g])):
                dup = 1
                break
            h = g + 1
            if L[h] != v:
                f, nxt = h, int(L[h])
                break
            if h >= end:
                break
            g = h
    else:
        f, nxt = begin, v
    b.head_f, b.head_next = f, nxt
    for w in range(4):
        b.head_div.seen[w] = seen[w]
    b.head_div.dup = dup
    return local, b


def _worker(rank, world, port, splits, minlen, name, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        esa = oracle_esa(name)
        N = esa.nonspecials
        L, B = _exact_lcp(esa), esa.bwt
        begin, end = splits[rank], splits[rank + 1]
        local, bnd = shard_view(L, B, N, begin, end, minlen)
        send = torch.frombuffer(bytearray(bytes(bnd)), dtype=torch.uint8)
        recv = [torch.zeros(G.BOUNDARY_BYTES, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(recv, send)
        bnds = [G.GtSmaxBoundary.from_buffer_copy(r.numpy().tobytes()) for r in recv]
        stitched = G.stitch_host(bnds, rank, minlen)
        mine = local + ([stitched] if stitched else [])
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        if rank == 0:
            out_q.put(sorted(x for part in gathered for x in part))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, splits, minlen, name="Atinsert.fna"):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.start_processes(_worker, args=(world, _free_port(), splits, minlen, name, q),
                       nprocs=world, join=True, start_method="spawn")
    return q.get()


def _plan(minlen, name="Atinsert.fna"):
    esa = oracle_esa(name)
    ref = O.linsmax(esa.lcpbytes, esa.llv, esa.bwt, esa.nonspecials, minlen)
    ref = sorted((int(l), int(lb), int(rb)) for l, lb, rb in ref)
    wide = max(ref, key=lambda t: t[2] - t[1])
    return esa, ref, wide


@pytest.mark.parametrize("minlen", [4, 8])
def test_two_ranks_split_inside_plateau(minlen):
    esa, ref, (l, lb, rb) = _plan(minlen)
    assert rb - lb >= 2
    splits = [1, lb + 2, esa.nonspecials]
    assert _run(2, splits, minlen) == ref


def test_three_ranks_passthrough_shard():
    esa, ref, (l, lb, rb) = _plan(4)
    assert rb - lb >= 3, "need a plateau of >= 3 rows for a passthrough shard"
    splits = [1, lb + 2, lb + 3, esa.nonspecials]
    assert _run(3, splits, 4) == ref


def test_two_ranks_even_split_matches_oracle():
    esa, ref, _ = _plan(8)
    N = esa.nonspecials
    splits = [1, 1 + (N - 1) // 2, N]      # bench.py's split rule for world 2
    assert _run(2, splits, 8) == ref
