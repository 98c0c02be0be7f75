cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
for v in xcd noxcd; do
  for c in FETCH_SIZE WRITE_SIZE; do
    MPAS_DYCORE_LIB=exp/lib_$v.so timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmc_${v}_$c -o $v$c --output-format csv -- python3 tools/kbench.py --reps 5 --steps 1 --no-graph > gpurun_out/pmc_${v}_$c.log 2>&1 || exit 1
  done
done
echo done
