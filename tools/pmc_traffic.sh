# HBM traffic per kernel: two separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE),
# as MI355X_MICROARCH.md "HBM" / "rocprofv3 PMC slots" prescribe.  Eager launches
# (no graph) so every dispatch carries its own counters.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-configs1 --no-graph --acoustic-reps 5 ${BENCH_ARGS}" &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o fetch --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o write --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_write.log 2>&1
echo EXIT $?
