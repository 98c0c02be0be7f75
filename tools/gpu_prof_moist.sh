# Kernel stats of the moist configuration (BASELINE configs[3]: ns = 6, monotone transport)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profm -o run --output-format csv -- python3 bench.py --moist --steps 3 --warmup 1 --no-cpu-baseline --no-configs1 > gpurun_out/profm.log 2>&1
echo EXIT $?
