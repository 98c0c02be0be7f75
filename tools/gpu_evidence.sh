# Round evidence at HEAD: default bench (configs[2] + configs[1] line), moist bench (configs[3]),
# var-res bench (configs[4] analogue), rocprofv3 kernel stats, PMC traffic (two passes), rank emulation
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --moist --no-cpu-baseline --no-configs1 > gpurun_out/bench_moist.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs1 > gpurun_out/prof.log 2>&1 &&
bash tools/pmc_traffic.sh > gpurun_out/pmc.log 2>&1 &&
timeout -k 10 400 python tools/rank_emulation.py --parts 1 2 4 8 > gpurun_out/rank_emulation.log 2>&1 &&
timeout -k 10 300 python tools/rank_emulation.py --parts 1 8 --no-graph > gpurun_out/rank_emulation_eager.log 2>&1
echo EXIT $?
tail -1 gpurun_out/bench.log | cut -c1-300; tail -1 gpurun_out/bench_moist.log | cut -c1-200; tail -3 gpurun_out/rank_emulation.log; tail -3 gpurun_out/rank_emulation_eager.log
