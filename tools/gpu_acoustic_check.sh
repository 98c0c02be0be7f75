# Acoustic sub-step: bench.py's HIP-event figure next to the rocprofv3 trace of the same run
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-configs1 > gpurun_out/bench_ac.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profac -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs1 > gpurun_out/profac.log 2>&1
echo EXIT $?
tail -1 gpurun_out/bench_ac.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); r=j['roofline']; print(j['ms_per_step'], r['frac'], r['ms_per_substep'], r['ms_kernels'])"
tail -1 gpurun_out/profac.log | cut -c1-50; python3 tools/acoustic_from_trace.py gpurun_out/profac/run_kernel_trace.csv 20 | tail -4
