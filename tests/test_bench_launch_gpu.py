"""bench.py's multi-rank launch path, end to end on the one GPU of the test box:
`bench.py --gpus 2` starts torch.distributed.run itself (two ranks, gloo,
host-staged exchange through TorchTransport), each rank simulates its half of
ONE 20k-peer config4 graph, and the summed events must equal a 1-rank run of
the same graph and schedule (the partitioned engine is exact).
The driver's 8-GPU run takes the same path with the nccl (RCCL) backend."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _bench(gpus):
    env = dict(os.environ, GS_DIST_BACKEND="gloo")
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(gpus), "--peers", "20000",
           "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--transport", "torch"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_two_ranks_equal_one():
    one = _bench(1)
    two = _bench(2)
    assert two["n_gpus"] == 2 and two["config"]["parallelism"] == "partition2"
    assert two["exchange"]["transport"] == "TorchTransport"
    assert two["events_per_step"] == one["events_per_step"]
    assert two["events_per_step"]["deliveries"] > 0
