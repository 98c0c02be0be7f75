# configs[2] drop-in: bits vs the Python host, ms/dt of the Fortran host vs the Python host
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_full_configs.py -v -x -k dropin --timeout 850 --timeout-method thread > gpurun_out/pytest_dropin_full.log 2>&1
echo EXIT $?
tail -3 gpurun_out/pytest_dropin_full.log; tail -2 gpurun_out/progress.log
