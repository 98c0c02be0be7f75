cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_lbc.py -v -x --timeout 300 --timeout-method thread > gpurun_out/pytest_lbc.log 2>&1
echo EXIT $?
tail -30 gpurun_out/pytest_lbc.log
