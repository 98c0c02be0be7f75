# fused pack/unpack + LBC: tests, then the single-block bench and 8 RCCL blocks (fused vs kernels)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_decomp.py tests/test_gpu_baseline_configs.py tests/test_gpu_lbc.py -v -x --timeout 300 --timeout-method thread > gpurun_out/pytest_pack.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-configs1 > gpurun_out/bench_1.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --blocks 8 --rccl-local --no-cpu-baseline --no-configs1 > gpurun_out/bench_8rccl_fused.log 2>&1 &&
MPAS_DYCORE_FUSED_PACK=0 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --blocks 8 --rccl-local --no-cpu-baseline --no-configs1 > gpurun_out/bench_8rccl_kernel.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --blocks 8 --rccl-local --no-cpu-baseline --no-configs1 > gpurun_out/bench_8rccl_fused2.log 2>&1
echo EXIT $?
tail -3 gpurun_out/pytest_pack.log
for f in 1 8rccl_fused 8rccl_kernel 8rccl_fused2; do python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$f.log').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['roofline']['frac'])"; done
