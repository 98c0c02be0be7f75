# Same-box A/B of whole-step time and the acoustic kernels: AB_LIBS alternated AB_ROUNDS times
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && rm -f gpurun_out/ab.log &&
for r in ${AB_ROUNDS:-1 2 3}; do for L in ${AB_LIBS:-exp/lib_base.so mpas-model_amd/csrc/libmpas_dycore.so}; do
echo "== $L" >> gpurun_out/ab.log
MPAS_DYCORE_LIB=$L timeout -k 10 200 python tools/kbench.py --steps ${AB_STEPS:-10} >> gpurun_out/ab.log 2>&1 || exit 1; done; done
echo EXIT $?; grep -h "==\|ms_dt\|acoustic" gpurun_out/ab.log | cut -c1-300
