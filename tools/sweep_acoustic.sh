cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && : > gpurun_out/sweep.log
python -c "import sys; sys.path.insert(0,'mpas-model_amd'); from mpas_dycore.cases import jw_case; jw_case(163842,K=56,ns=1)" >> gpurun_out/sweep.log 2>&1 || exit 1
for lib in mpas-model_amd/csrc/libmpas_dycore.so exp/libmpas_dycore_t8_w4.so exp/libmpas_dycore_t16_w4.so exp/libmpas_dycore_t8_w2.so exp/libmpas_dycore_t32_w8.so; do
  for f in 1 0; do
    echo "== $lib fused=$f" >> gpurun_out/sweep.log
    MPAS_DYCORE_FUSED=$f MPAS_DYCORE_LIB=$lib timeout -k 10 200 python tools/kbench.py --steps 3 --reps 40 >> gpurun_out/sweep.log 2>&1 || exit 1
  done
done
echo DONE >> gpurun_out/sweep.log
