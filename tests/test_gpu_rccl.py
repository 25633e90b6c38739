"""The RCCL code path on the one GPU a test box has (VERDICT r2 "exercise the RCCL code").

* SearchEngine under a one-rank "nccl" process group (fresh child process, group initialised
  before any GPU work): the round's all_gather of scores and the winner-image broadcast run on
  RCCL, and the searches equal the no-group run bit for bit (tests/rccl_child.py).
* bench.py under torch.distributed.run with one rank: its init_process_group("nccl"), barriers,
  all_reduce(MAX) of the timed region and the engine's all_gather, at a tiny N and T.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env():
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_search_engine_over_one_rank_rccl_group_matches_no_group():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_child.py"), str(_free_port())],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    print(out)
    assert out["backend"] == "nccl" and out["dist_with"] is True and out["dist_without"] is False
    assert out["identical"] == {"random": True, "zo": True}
    assert out["all_reduce"] == 3.0 and out["random_best"] >= 0


def test_bench_under_torchrun_one_rank_nccl():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "1", "--warmup", "1", "--n-total", "16", "--T", "10", "--no-extras",
           "--no-cpu-baseline", "--no-live-traffic"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    print({k: line[k] for k in ("value", "n_gpus", "scaling", "config")})
    assert line["n_gpus"] == 1 and line["config"]["process_group"] == "nccl"
    assert line["value"] > 0 and line["config"]["global_batch"] == 16
