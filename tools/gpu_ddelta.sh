# Damping-delta change: single-block parity, kernel families, decomposition, LBC, physics, restart; then A/B
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && rm -f gpurun_out/ab.log &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_decomp.py tests/test_gpu_lbc.py tests/test_gpu_physics.py tests/test_gpu_restart.py tests/test_gpu_baseline_configs.py > gpurun_out/pytest_ddelta.log 2>&1 &&
for r in 1 2 3; do for L in exp/lib_head.so mpas-model_amd/csrc/libmpas_dycore.so; do
echo "== $L" >> gpurun_out/ab.log
MPAS_DYCORE_LIB=$L timeout -k 10 200 python tools/kbench.py --steps 10 >> gpurun_out/ab.log 2>&1 || exit 1; done; done
echo EXIT $?; tail -3 gpurun_out/pytest_ddelta.log; grep -h "==\|ms_dt" gpurun_out/ab.log | cut -c1-110
