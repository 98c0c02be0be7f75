# The whole GPU suite and the default bench line at HEAD
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 1000 python -u -m pytest tests -v -m gpu -x --timeout 900 --timeout-method thread > gpurun_out/pytest_gpu_head.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_head.log 2>&1
echo EXIT $?
tail -2 gpurun_out/pytest_gpu_head.log; tail -1 gpurun_out/bench_head.log | cut -c1-300
