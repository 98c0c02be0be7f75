# Round-2 evidence run: whole GPU suite (incl. the full-size BASELINE configs), default bench
# (configs[2] mesh at order 3 + configs[1] line), and the rocprofv3 kernel-trace summary.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 1000 python -u -m pytest tests -v -m gpu -x --timeout 900 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs1 > gpurun_out/prof.log 2>&1 &&
timeout -k 10 400 python tools/rank_emulation.py --parts 1 2 4 8 > gpurun_out/rank_emulation.log 2>&1 &&
timeout -k 10 400 python tools/rank_emulation.py --parts 1 8 --no-graph > gpurun_out/rank_emulation_eager.log 2>&1
echo EXIT $?
tail -3 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/bench.log | cut -c1-500
