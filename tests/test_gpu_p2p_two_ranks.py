"""GPU: two processes (ranks) on the one GPU, each stepping its block of a 2-way split, every halo
message through the one-sided transfer between processes -- the peer's fields and flag arena mapped
over IPC, the set-up all-gathers through gloo (mpas_dyc_comm_init_host), no RCCL -- give one block's
values bit for bit after 3 steps (tools/p2p_two_ranks.py).  The path of `bench.py --gpus N` on a node,
with the two GPUs' memory in one device.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# buffers-moist: the case that caught send buffers in uncached memory (stale halo values in about one
# run in four: profiles/r05_p2p_buffers_race.log)
@pytest.mark.parametrize("args", [[], ["--moist"], ["--pull", "0"], ["--pull", "0", "--moist"]],
                         ids=["pull", "pull-moist", "buffers", "buffers-moist"])
def test_two_ranks_one_sided_bitwise(args):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", "29531", os.path.join(ROOT, "tools", "p2p_two_ranks.py")] + args
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and lines, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads(lines[-1])
    assert out["p2p_active"] and out["bitwise"], out
