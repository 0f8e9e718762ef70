"""bench.py's multi-rank path, rehearsed on one GPU.

The driver's SCALE run launches `bench.py --gpus N` for N = 2, 4, 8 on a whole node; no multi-GPU
node is ours to use.  These tests run the same code path as child processes on the one-GPU box:
MBLS_BENCH_SAME_DEVICE=1 puts both ranks on device 0 and MBLS_BENCH_BACKEND=gloo replaces RCCL
(which refuses two ranks on one device).  Pinned: the rank launcher (bench.py launch_ranks), the
world-size bookkeeping of the JSON line, and sharded_msm.gather_partials' exchange + EC sum --
config #4's sharded MSM digest at N = 2 equals the N = 1 digest (the 1-GPU result is pinned to
the oracle by tests/test_gpu_parity.py)."""
import json
import os
import subprocess
import sys

import pytest

import helpers as H

pytestmark = pytest.mark.gpu
BENCH = os.path.join(H.ROOT, "bench.py")
ARGS = ["--msm-total-log", "21", "--steps", "2", "--warmup", "1", "--no-cpu", "--no-mix", "--msm-batch", "0",
        "--no-stage-profile"]


def _run(gpus, extra_env=None, timeout=240):
    env = dict(os.environ)
    env.update(extra_env or {})
    p = subprocess.run([sys.executable, BENCH, "--gpus", str(gpus)] + ARGS, env=env, capture_output=True, text=True,
                       timeout=timeout)
    line = None
    for ln in p.stdout.splitlines():
        if ln.startswith("{") and '"metric"' in ln:
            line = json.loads(ln)
    return p.returncode, line, p.stderr[-2000:]


@pytest.fixture(scope="module")
def n1():
    rc, line, err = _run(1)
    assert rc == 0 and line, err
    return line


def test_bench_two_ranks_same_device_matches_one(n1):
    rc, line, err = _run(2, {"MBLS_BENCH_SAME_DEVICE": "1", "MBLS_BENCH_BACKEND": "gloo"})
    assert rc == 0 and line, err
    assert line["n_gpus"] == 2
    assert len(line["rank_devices"]) == 2 and sorted(d["rank"] for d in line["rank_devices"]) == [0, 1]
    assert line["config"]["parallelism"] == "msm-shard2"
    a, b = line["config4_msm_sharded"], n1["config4_msm_sharded"]
    assert a["result_digest"] == b["result_digest"], (a, b)
    # weak scaling: every rank ran the headline MSM on its own 2^20 points
    assert line["config"]["msm_points_per_gpu"] == n1["config"]["msm_points_per_gpu"]


def test_bench_refuses_more_ranks_than_gpus():
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("this box has 2+ GPUs: the refusal path is not reachable")
    rc, line, err = _run(2, timeout=120)
    assert rc == 2 and line is None, (rc, err)
    assert "needs 2 visible GPUs" in err
