"""bench.py's own rank launcher (no GPU): `python bench.py --gpus N` from a
plain process starts N ranks with the torch.distributed.run environment, and
a --gpus / WORLD_SIZE mismatch is an error (the driver's
N-GPU line must measure N ranks).  The hidden --launch-probe flag makes each
rank print what it was handed and exit before importing torch."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                        "MASTER_PORT")}
    env.update(kw)
    return env


def test_launcher_starts_n_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--launch-probe", "1"],
                       capture_output=True, text=True, env=_env(), timeout=120)
    assert r.returncode == 0, r.stderr
    got = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert sorted(int(g["RANK"]) for g in got) == [0, 1, 2, 3]
    for g in got:
        assert g["WORLD_SIZE"] == "4" and g["LOCAL_WORLD_SIZE"] == "4"
        assert g["LOCAL_RANK"] == g["RANK"]
        assert g["MASTER_ADDR"] == "127.0.0.1"
    assert len({g["MASTER_PORT"] for g in got}) == 1


def test_launcher_propagates_rank_failure():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--launch-probe", "fail1"],
                       capture_output=True, text=True, env=_env(), timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr)


def test_gpus_world_size_mismatch_is_an_error():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-probe", "1"],
                       capture_output=True, text=True,
                       env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"), timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=3" in r.stderr


def test_single_gpu_runs_in_process():
    r = subprocess.run([sys.executable, BENCH, "--launch-probe", "1"],
                       capture_output=True, text=True, env=_env(), timeout=120)
    assert r.returncode == 0, r.stderr
    got = json.loads(r.stdout.strip())
    assert got["WORLD_SIZE"] is None
