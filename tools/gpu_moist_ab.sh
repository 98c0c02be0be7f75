# Transport load-order changes: moist / physics / family / LBC GPU tests, then a same-box moist A/B
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && rm -f gpurun_out/abm.log &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_baseline_configs.py tests/test_gpu_physics.py tests/test_gpu_lbc.py tests/test_gpu_configs.py tests/test_gpu_decomp.py > gpurun_out/pytest_moist.log 2>&1 &&
for r in 1 2; do for L in exp/lib_base_h.so exp/lib_m_ne.so mpas-model_amd/csrc/libmpas_dycore.so; do
echo "== $L" >> gpurun_out/abm.log
MPAS_DYCORE_LIB=$L timeout -k 10 250 python tools/kbench.py --moist --steps 10 >> gpurun_out/abm.log 2>&1 || exit 1; done; done
echo EXIT $?; tail -3 gpurun_out/pytest_moist.log; grep -h "==\|ms_dt" gpurun_out/abm.log | cut -c1-100
