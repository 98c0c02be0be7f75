cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 300 > gpurun_out/pytest_gpu.log 2>&1 &&
for r in ${AB_ROUNDS:-1 2}; do for L in ${AB_LIBS:-exp/lib_b.so mpas-model_amd/csrc/libmpas_dycore.so}; do
MPAS_DYCORE_LIB=$L timeout -k 10 200 python tools/kbench.py --steps ${AB_STEPS:-5} >> gpurun_out/ab.log 2>&1 || exit 1; done; done
echo EXIT $?; tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/ab.log | grep ms_dt
