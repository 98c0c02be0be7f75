# GPU check: parity tests, smoke, bench and a rocprofv3 kernel-trace profile.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 300 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 900 python bench.py --steps 5 --warmup 2 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs1 > gpurun_out/prof.log 2>&1
echo EXIT $?
tail -3 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/bench.log
