# Kernel trace of 8 RCCL blocks on one GPU (the 8-GPU decomposition's kernels, split-phase exchanges)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 300 python bench.py --blocks 8 --rccl-local --steps 5 --warmup 2 --no-cpu-baseline --no-configs1 > gpurun_out/b8.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8b -o run --output-format csv -- python3 bench.py --blocks 8 --rccl-local --steps 3 --warmup 1 --no-cpu-baseline --no-configs1 > gpurun_out/prof8b.log 2>&1
echo EXIT $?; tail -1 gpurun_out/b8.log | cut -c1-300
