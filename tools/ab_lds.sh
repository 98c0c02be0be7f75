cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 300 > gpurun_out/pytest_gpu.log 2>&1 &&
for r in 1 2 3; do for L in 0 1; do
MPAS_DYCORE_LDS=$L timeout -k 10 200 python tools/kbench.py --steps 20 >> gpurun_out/ab.log 2>&1 || exit 1; echo "lds=$L" >> gpurun_out/ab.log; done; done
echo EXIT $?; tail -3 gpurun_out/pytest_gpu.log; grep -A1 ms_dt gpurun_out/ab.log | cut -c1-90
