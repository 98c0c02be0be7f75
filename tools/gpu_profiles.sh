# Round-end evidence: GPU parity suite, default bench (configs[2] mesh + configs[1] line), moist
# bench (configs[3]), and the rocprofv3 kernel-trace summary of the default bench.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 300 > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --moist --no-cpu-baseline --no-configs1 > gpurun_out/bench_moist.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs1 > gpurun_out/prof.log 2>&1
echo EXIT $?
tail -2 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/bench.log | cut -c1-400; tail -1 gpurun_out/bench_moist.log | cut -c1-300
