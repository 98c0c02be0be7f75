# Fused acoustic sub-step: bitwise tests, then a same-box A/B of bench.py with and without it.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_decomp.py tests/test_gpu_parity.py -v -x --timeout 300 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-configs1 > gpurun_out/bench_fused.log 2>&1 &&
MPAS_DYCORE_FUSED=0 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-configs1 > gpurun_out/bench_unfused.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-configs1 > gpurun_out/bench_fused2.log 2>&1
echo EXIT $?
tail -3 gpurun_out/pytest_fused.log
for f in bench_fused bench_unfused bench_fused2; do python -c "import json,sys; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step'],3), round(d['roofline']['frac'],4), round(d['roofline']['ms_per_substep'],4), d['roofline']['ms_kernels'])" || true; done
