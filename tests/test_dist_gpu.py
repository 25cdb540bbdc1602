"""Multi-rank device path of the sharded smax pass on one GPU.

Each spawned rank (world_size 2 or 3, all on cuda:0, gloo process group)
runs exactly the step bench.py runs per rank:

    plan.run_part(0) -> plan.copy_boundary -> all-gather of the boundary
    records -> plan.run_part(1) -> plan.stitch (smax_stitch_kernel)

The boundary records are staged through host memory for gloo (bench.py's
--dist-backend gloo rehearsal; the driver's 8-GPU run uses RCCL on device
memory, same bytes).  The ranks' record lists, concatenated in rank order,
must equal the CPU oracle's single-shard answer bit for bit -- order
included.  Two table layouts:
  - shard-local tables (each rank holds LCP[begin-1 .. end], its BWT rows and
    its .llv entries, as the host-table entry point uploads them), at1MB with
    splits inside plateaus and a shard lying entirely inside one;
  - full tables per rank (bench.py: the GPU suffixerator output, each rank
    planning over its own range), 100 Mbp uniform and 30 Mbp human-like.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import genometools_smax_amd as G
import oracle_lib as O
from conftest import oracle_esa

pytestmark = pytest.mark.gpu


def _padded(host, length):
    t = torch.zeros(G.PAD_FRONT + length + G.PAD_BACK, dtype=torch.uint8, device="cuda")
    t[G.PAD_FRONT: G.PAD_FRONT + len(host)] = torch.from_numpy(np.ascontiguousarray(host))
    return t, t.data_ptr() + G.PAD_FRONT


def _exchange(plan, world, rank):
    """The rank's step as bench.py runs it: scan (part 0), boundary copy and
    all-gather, compaction (part 1), stitch."""
    stream = torch.cuda.current_stream().cuda_stream
    plan.run_part(0, stream)
    send = torch.zeros(G.BOUNDARY_BYTES, dtype=torch.uint8, device="cuda")
    plan.copy_boundary(send.data_ptr(), stream)
    hrecv = torch.zeros(G.BOUNDARY_BYTES * world, dtype=torch.uint8)
    dist.all_gather_into_tensor(hrecv, send.cpu())
    plan.run_part(1, stream)
    recv = hrecv.cuda()
    plan.stitch(recv.data_ptr(), world, rank, stream)
    torch.cuda.synchronize()
    return plan.fetch_triples()


def _worker_local(rank, world, port, splits, minlen, name, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        e = oracle_esa(name)
        N = e.nonspecials
        begin, end = splits[rank], splits[rank + 1]
        base = begin - 1
        length = end - base + 1                      # LCP[begin-1 .. end]
        lcp_t, lcp_p = _padded(e.lcpbytes[base: base + length], length)
        bwt_t, bwt_p = _padded(e.bwt[base: min(base + length, e.n + 1)], length)
        pos = e.llv[:, 0] if len(e.llv) else np.zeros(0, np.uint64)
        mine = e.llv[(pos >= base) & (pos < base + length)]
        llv_t = torch.from_numpy(np.ascontiguousarray(
            np.vstack([mine, np.zeros((1, 2), np.uint64)]).view(np.int64))).cuda()
        # capacity: at most one interval per two rows
        plan = G.SmaxPlan(lcp_p, bwt_p, llv_t.data_ptr(), len(mine), base, length, begin, end, N,
                          minlen, device=0, capacity=(end - begin) // 2 + 16)
        trip = _exchange(plan, world, rank)
        plan.close()
        parts = [None] * world
        dist.all_gather_object(parts, trip)
        if rank == 0:
            np.savez(out_path, got=np.concatenate(parts).reshape(-1, 3))
        del lcp_t, bwt_t, llv_t
    finally:
        dist.destroy_process_group()


def _worker_full(rank, world, port, kind, bases, seed, minlen, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        text = G.synth_genome(kind, bases, seed, threads=4)
        esa = G.DeviceEsa(text, device=0)
        N = esa.nonspecials
        begin = 1 + (N - 1) * rank // world           # bench.py's split rule
        end = 1 + (N - 1) * (rank + 1) // world
        plan = esa.plan(minlen, begin, end, capacity=(end - begin) // 2 + 16)
        trip = _exchange(plan, world, rank)
        plan.close()
        parts = [None] * world
        dist.all_gather_object(parts, trip)
        if rank == 0:
            host = esa.download()
            want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], N, minlen, threads=4)
            np.savez(out_path, got=np.concatenate(parts).reshape(-1, 3), want=want)
        esa.release()
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(fn, world, *args):
    """Runs fn on world spawned ranks; rank 0 saves the result into a file
    (a pipe-backed queue would block rank 0 on a large put while the parent
    waits in join)."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "result.npz")
        mp.start_processes(fn, args=(world, _free_port()) + args + (out,), nprocs=world,
                           join=True, start_method="spawn")
        with np.load(out) as f:
            return {k: f[k] for k in f.files}


def _widest(name, minlen):
    e = oracle_esa(name)
    ref = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, minlen)
    k = int(np.argmax(ref[:, 2] - ref[:, 1]))
    return e, ref, [int(x) for x in ref[k]]


@pytest.mark.parametrize("minlen", [8, 20])
def test_two_ranks_local_tables_split_inside_plateau(minlen):
    e, ref, (l, lb, rb) = _widest("at1MB", minlen)
    assert rb - lb >= 2
    got = _spawn(_worker_local, 2, [1, lb + 2, e.nonspecials], minlen, "at1MB")["got"]
    assert np.array_equal(got, ref), (len(got), len(ref))


def test_three_ranks_local_tables_passthrough_shard():
    e, ref, (l, lb, rb) = _widest("at1MB", 8)
    assert rb - lb >= 3
    got = _spawn(_worker_local, 3, [1, lb + 2, lb + 3, e.nonspecials], 8, "at1MB")["got"]
    assert np.array_equal(got, ref), (len(got), len(ref))


def test_three_ranks_local_tables_even_split():
    e = oracle_esa("at1MB")
    N = e.nonspecials
    ref = O.linsmax(e.lcpbytes, e.llv, e.bwt, N, 20)
    got = _spawn(_worker_local, 3, [1 + (N - 1) * r // 3 for r in range(4)], 20, "at1MB")["got"]
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("world,kind,bases,seed", [(2, "uniform", 100_000_000, 42),
                                                   (3, "human", 30_000_000, 5)])
def test_full_tables_bench_split(world, kind, bases, seed):
    r = _spawn(_worker_full, world, kind, bases, seed, 20)
    got, want = r["got"], r["want"]
    assert len(want) > 100
    assert np.array_equal(got, want), (len(got), len(want))


# ---------------------------------------------------------------- > 1 device
# The measured multi-GPU configuration: one process per device, the nccl
# backend (RCCL over xGMI), boundary records all-gathered in device memory
# from the plan's own zero-copy boundary tensor, exactly bench.py's step.
# Needs as many visible devices as ranks; skipped on a one-GPU box.

def _worker_nccl(rank, world, port, kind, bases, seed, minlen, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", rank=rank, world_size=world,
                            device_id=torch.device("cuda", rank))
    try:
        text = G.synth_genome(kind, bases, seed, threads=4)
        n = len(text)
        N = n - int(np.count_nonzero(text >= 254))
        begin = 1 + (N - 1) * rank // world
        end = 1 + (N - 1) * (rank + 1) // world
        esa = G.DeviceEsa64(text, device=rank, row_lo=begin - 1, row_hi=end + 1)
        plan = esa.plan(minlen, begin, end, capacity=(end - begin) // 2 + 16)
        stream = torch.cuda.current_stream().cuda_stream
        recv = torch.zeros(G.BOUNDARY_BYTES * world, dtype=torch.uint8, device="cuda")
        send = plan.boundary_tensor()
        for _ in range(3):                       # repeated steps, as the bench runs them
            plan.run_part(0, stream)
            work = dist.all_gather_into_tensor(recv, send, async_op=True)
            plan.run_part(1, stream)
            work.wait()
            plan.stitch(recv.data_ptr(), world, rank, stream)
        torch.cuda.synchronize()
        trip = plan.fetch_triples()
        plan.close()
        esa.release()
        parts = [None] * world
        dist.all_gather_object(parts, trip)
        if rank == 0:
            full = G.DeviceEsa(text, device=0)
            host = full.download()
            full.release()
            want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], N, minlen, threads=4)
            np.savez(out_path, got=np.concatenate(parts).reshape(-1, 3), want=want)
    finally:
        dist.destroy_process_group()


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs >= 2 visible GPUs")
@pytest.mark.parametrize("world", [2, 4, 8])
def test_nccl_ranks_one_per_device(world):
    if torch.cuda.device_count() < world:
        pytest.skip("needs %d visible GPUs" % world)
    r = _spawn(_worker_nccl, world, "human", 30_000_000, 5, 20)
    assert len(r["want"]) > 100
    assert np.array_equal(r["got"], r["want"]), (len(r["got"]), len(r["want"]))


# ------------------------------------------------ bench.py's own rank launch
# `python bench.py --gpus N` from a plain process (no torchrun): the parent
# starts the N ranks itself; the line must report N ranks that all took part
# in the collective, with the stitched records bit-exact.

def _bench_line(args, timeout=600):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                        "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args,
                       capture_output=True, text=True, env=env, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_self_launch_two_ranks_one_gpu():
    out = _bench_line(["--gpus", "2", "--one-gpu", "--dist-backend", "gloo", "--bases", "2e7",
                       "--steps", "3", "--warmup", "1", "--prime-s", "0"])
    assert out["n_gpus"] == 2
    assert out["dist"]["world_size"] == 2 and out["dist"]["allreduce_ranks"] == 2
    assert out["parity"].startswith("bit-exact")
    assert out["smax_intervals"] > 100


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs >= 2 visible GPUs")
def test_bench_self_launch_nccl_one_rank_per_device():
    out = _bench_line(["--gpus", "2", "--bases", "3e7", "--steps", "3", "--warmup", "1",
                       "--prime-s", "0"])
    assert out["n_gpus"] == 2
    assert out["dist"]["backend"] == "nccl" and out["dist"]["allreduce_ranks"] == 2
    assert out["dist"]["distinct_devices"] == 2
    assert out["parity"].startswith("bit-exact")
