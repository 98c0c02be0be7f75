#!/usr/bin/env python3
"""Start tools/p2p_ipc_check as two processes on one GPU (ranks 0 and 1, a rendezvous directory for
the IPC handles) for a few message sizes, in both modes of the library's one-sided transfer (buffers:
k_p2p_post / k_p2p_get on uncached send buffers; pull: k_p2p_pull reading the peer's ordinary device
memory); print their JSON lines; exit non-zero if any received double was wrong, a wait timed out or
a process failed.

    python tools/p2p_ipc_check.py [--sizes 1000 100000 1000000] [--iters 2000]
"""
import argparse
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="+", default=[1000, 100000, 1000000])
    ap.add_argument("--iters", type=int, default=2000)
    a = ap.parse_args()
    exe = os.path.join(ROOT, "tools", "p2p_ipc_check")
    ok = True
    for mode, n in [(m, n) for m in ("buffers", "pull") for n in a.sizes]:
        with tempfile.TemporaryDirectory() as d:
            procs = [subprocess.Popen([exe, str(r), d, str(n), str(a.iters), mode], stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True) for r in (0, 1)]
            for p in procs:
                try:
                    out, _ = p.communicate(timeout=240)
                except subprocess.TimeoutExpired:
                    p.kill()
                    out, _ = p.communicate()
                    ok = False
                sys.stdout.write(out)
                ok = ok and p.returncode == 0
            sys.stdout.flush()
    print("p2p_ipc_check:", "ok" if ok else "FAILED")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
