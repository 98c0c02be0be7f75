# Round-end evidence at HEAD: the whole GPU suite, then tools/gpu_evidence.sh (benches, kernel stats,
# PMC traffic, rank emulation)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 1080 python -u -m pytest tests -v -m gpu -x --timeout 900 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1 &&
bash tools/gpu_evidence.sh
echo EXIT $?
tail -3 gpurun_out/pytest_gpu_full.log
