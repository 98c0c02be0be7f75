# The whole GPU suite, full-size BASELINE configs included
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 1080 python -u -m pytest tests -v -m gpu -x --timeout 900 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1
echo EXIT $?
tail -4 gpurun_out/pytest_gpu_full.log; grep -c PASSED gpurun_out/pytest_gpu_full.log
