# Same-box A/B of two libraries (AB_A, AB_B), whole dt and acoustic kernels, 3 rounds
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && rm -f gpurun_out/ab.log &&
for r in 1 2 3; do for L in $AB_A $AB_B; do
echo "== $L" >> gpurun_out/ab.log
MPAS_DYCORE_LIB=$L timeout -k 10 200 python tools/kbench.py --steps 10 >> gpurun_out/ab.log 2>&1 || exit 1; done; done
echo EXIT $?; grep -h "==\|ms_dt" gpurun_out/ab.log | cut -c1-110
