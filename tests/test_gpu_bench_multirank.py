"""GPU: bench.py's multi-rank path as the driver runs it (torch.distributed.run, one process per rank,
gloo rendezvous, host-side plan preflight, watchdog, max-over-ranks timing, per-rank exchange profile)
with two ranks on the one GPU of the box (--same-device: no RCCL, the one-sided transfer between the
two processes over IPC).  Checks the JSON contract of the line, not the speed."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_same_device():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", "29543", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--same-device", "--ncells", "10242",
           "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-configs1", "--acoustic-reps", "3"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=ROOT)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3 and out["warmup"] == 1 and out["value"] > 0
    assert out["preflight"]["ok"] and len(out["ranks"]) == 2
    assert "one-sided" in out["config"]["parallelism"] and out["config"]["hip_graph"]
    assert all(rk["exchanges"] == 52 for rk in out["ranks"])
