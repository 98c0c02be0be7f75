"""bench.py's multi-rank control flow on the CPU (gloo), up to the first GPU call.

The driver's N = 2, 4, 8 scaling runs are the first time bench.py runs with world > 1 on GPUs.
Before any rank touches its GPU, bench.py plans every rank's RCCL messages with the library's own
planner in a host-only context and checks across ranks (gloo all_gather) that the sends and
receives pair up (mpas_dycore.preflight); --preflight-only stops there.  A phase that hangs later
(ncclCommInitRank, an RCCL group) is ended by the watchdog with one JSON line naming the phase and
the last enqueued exchange, exit status 3."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _json_lines(text):
    out = []
    for ln in text.splitlines():
        ln = ln.strip()
        if ln.startswith("{"):
            try:
                out.append(json.loads(ln))
            except ValueError:
                pass
    return out


@pytest.mark.parametrize("nranks", [2, 4])
def test_bench_preflight_world(nranks):
    port = 29500 + 37 * nranks
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nranks}",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", str(nranks), "--preflight-only", "--ncells", "2562", "--levels", "26"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [j for j in _json_lines(r.stdout) if "preflight" in j]
    assert len(lines) == 1, r.stdout[-2000:]
    j = lines[0]
    assert j["n_gpus"] == nranks and j["preflight"]["ok"]
    assert j["preflight"]["plan_keys"] > 40 and j["preflight"]["messages"] > 0
    assert j["rccl_version"] > 20000


def test_watchdog_names_the_phase():
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "w = bench.Watchdog(1, True); w.phase('rccl_init (ncclCommInitRank) and upload', 1.0); time.sleep(30)"
            % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60, cwd=ROOT)
    assert r.returncode == 3
    j = _json_lines(r.stdout)[0]
    assert j["rank"] == 1 and j["phase"].startswith("rccl_init") and j["value"] is None


_AGREE = """
import os, sys
sys.path.insert(0, %r)
import torch.distributed as dist
import bench
dist.init_process_group("gloo")
r, w = dist.get_rank(), dist.get_world_size()
err = "rank %%d: one-sided wait timed out" %% r if r == w - 1 else ""
first = bench.agree_on_failure(dist, w, err)
ok = bench.agree_on_failure(dist, w, "")
open(os.path.join(%r, "r%%d.txt" %% r), "w").write("%%s|%%s" %% (first, ok))
dist.destroy_process_group()
"""


def test_transport_fallback_is_agreed_by_every_rank(tmp_path):
    """bench.py's fallback from the one-sided transfer to RCCL: when one rank's warm-up fails, every
    rank gets the same (first failing rank's) message and rebuilds over RCCL together; when none
    fails, none does."""
    script = tmp_path / "agree.py"
    script.write_text(_AGREE % (ROOT, str(tmp_path)))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
                        "--master-addr", "127.0.0.1", "--master-port", "29617", str(script)],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    got = [(tmp_path / f"r{i}.txt").read_text() for i in range(3)]
    assert got == ["rank 2: one-sided wait timed out|None"] * 3, got
