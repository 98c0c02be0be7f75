"""Run the Fortran drop-in harness at configs[2] size and keep its stderr / timing (diagnostics)."""
import os
import subprocess
import sys
import tempfile

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpas-model_amd")]
from mpas_dycore.cases import jw_case  # noqa: E402
from oracle import ref_runner  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 163842
prof = sys.argv[2:]  # e.g. rocprofv3 --kernel-trace --stats -d gpurun_out/dprof -o run --output-format csv --
c = jw_case(n, K=56, ns=1, order=3)
tmp = tempfile.mkdtemp(prefix="dropin_")
ind, outd = os.path.join(tmp, "in"), os.path.join(tmp, "out")
ref_runner.write_inputs(c, ind, 10, float(c["dt"]), [10], 1, 1, dump_only=["state.u"])
env = dict(os.environ, OMP_NUM_THREADS="1", OMP_STACKSIZE="1G")
import time
env.update(dict(a.split("=", 1) for a in os.environ.get("PROBE_ENV", "").split() if "=" in a))
pr = subprocess.Popen(prof + [ref_runner.DROPIN_HARNESS, ind, outd], cwd=tmp, env=env, stdout=subprocess.PIPE,
                      stderr=subprocess.PIPE, text=True)
aff = set()
while pr.poll() is None:
    try:
        for tid in os.listdir(f"/proc/{pr.pid}/task"):
            for line in open(f"/proc/{pr.pid}/task/{tid}/status"):
                if line.startswith("Cpus_allowed_list"):
                    aff.add((tid, line.split()[1]))
    except OSError:
        pass
    time.sleep(0.5)
out, err = pr.communicate()
print("rc", pr.returncode, "threads/affinity seen:", sorted(aff)[:12], len(aff))
print("stderr tail:", err[-1500:])
print(open(os.path.join(outd, "timing.txt")).read())
