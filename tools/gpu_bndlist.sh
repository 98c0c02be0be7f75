# Compact phase-2 lists: decomposition / split-phase GPU tests, then a same-box A/B of 8 RCCL blocks
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && rm -f gpurun_out/ab8.log &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_decomp.py tests/test_gpu_baseline_configs.py tests/test_gpu_varres.py tests/test_gpu_summary.py tests/test_gpu_dropin.py > gpurun_out/pytest_bnd.log 2>&1 &&
for r in 1 2; do for L in exp/lib_head.so mpas-model_amd/csrc/libmpas_dycore.so; do
echo "== $L" >> gpurun_out/ab8.log
MPAS_DYCORE_LIB=$L timeout -k 10 300 python bench.py --blocks 8 --rccl-local --steps 5 --warmup 2 --no-cpu-baseline --no-configs1 >> gpurun_out/ab8.log 2>&1 || exit 1; done; done
echo EXIT $?; tail -3 gpurun_out/pytest_bnd.log; grep -h "==\|ms_per_step" gpurun_out/ab8.log | sed 's/.*"ms_per_step": \([0-9.]*\).*/\1/'
