"""bench.py starts its own ranks when no launcher set WORLD_SIZE.

CPU: `bench.spawn_ranks` gives every child the torch.distributed.run environment, a working
gloo rendezvous on 127.0.0.1, and returns a failing rank's status after stopping the others.
GPU: `python bench.py --gpus 2 --dist-backend gloo` (no torch.distributed.run; both ranks on the
one leased GPU) ends with rc 0 and a dp2 line.
"""

import json
import os
import subprocess
import sys
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402

_CHILD_OK = r"""
import json, os, sys
import torch, torch.distributed as dist
dist.init_process_group("gloo")
t = torch.tensor([float(os.environ["RANK"]) + 1.0])
dist.all_reduce(t)
if os.environ["RANK"] == "0":
    print(json.dumps({"world": dist.get_world_size(), "sum": t.item(),
                      "local": os.environ["LOCAL_RANK"], "addr": os.environ["MASTER_ADDR"]}))
dist.destroy_process_group()
"""

_CHILD_FAIL = r"""
import os, sys, time
if os.environ["RANK"] == "1":
    sys.exit(3)
time.sleep(120)   # a rank that would wait forever for its peer
"""


def test_spawn_ranks_sets_the_launcher_environment(tmp_path, capfd):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    rc = bench.spawn_ranks(3, [sys.executable, "-c", _CHILD_OK], env=env)
    out = capfd.readouterr().out
    assert rc == 0, out
    j = json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])
    assert j == {"world": 3, "sum": 6.0, "local": "0", "addr": "127.0.0.1"}


def test_spawn_ranks_stops_the_others_when_one_fails():
    t0 = time.time()
    rc = bench.spawn_ranks(2, [sys.executable, "-c", _CHILD_FAIL])
    assert rc == 3
    assert time.time() - t0 < 60  # the sleeping rank was terminated, not waited for


@pytest.mark.gpu
def test_bench_gpus2_without_launcher_runs_two_ranks(cuda_device):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run(
        [sys.executable, "-u", os.path.join(REPO, "bench.py"), "--gpus", "2", "--dist-backend",
         "gloo", "--config", "cfg1", "--steps", "5", "--warmup", "3", "--profile-steps", "0",
         "--collate-bench", "0", "--infer-bench", "0", "--cpu-baseline", "0"],
        capture_output=True, text=True, timeout=300, env=env)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-4000:]  # rank 0 alone prints
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["config"]["parallelism"] == "dp2", j
    assert j["config"]["global_batch"] == 2 * 32 and j["value"] > 0, j
    assert j.get("launcher", "").startswith("bench.py spawned"), j
