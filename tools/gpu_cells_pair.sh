# Pair-layout acoustic cell phase: bitwise tests, then a same-box A/B (MPAS_DYCORE_CELLS_PAIR=0 / 1)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && rm -f gpurun_out/abp.log &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cells_pair.py tests/test_gpu_kernels.py > gpurun_out/pytest_cells_pair.log 2>&1 &&
for r in 1 2 3; do for v in 0 1; do
echo "== pair=$v" >> gpurun_out/abp.log
MPAS_DYCORE_CELLS_PAIR=$v timeout -k 10 200 python tools/kbench.py --steps 10 >> gpurun_out/abp.log 2>&1 || exit 1; done; done
echo EXIT $?; tail -3 gpurun_out/pytest_cells_pair.log; grep -h "==\|ms_dt" gpurun_out/abp.log | cut -c1-160
