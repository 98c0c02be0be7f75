# Quick GPU evidence: GPU suite without the full-size configs, default bench, rocprofv3 kernel stats.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 700 python -u -m pytest tests -v -m "gpu and not slow" -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs1 > gpurun_out/prof.log 2>&1
echo EXIT $?
tail -3 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/bench.log | cut -c1-600
