# rocprofv3 kernel stats of tools/kbench.py for several library / env variants (A/B per kernel),
# after the GPU parity suite on the in-tree library
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 300 > gpurun_out/pytest_gpu.log 2>&1 &&
MPAS_DYCORE_LDS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pv_a -o a --output-format csv -- python3 tools/kbench.py --steps 3 --reps 5 > gpurun_out/pv_a.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pv_b -o b --output-format csv -- python3 tools/kbench.py --steps 3 --reps 5 > gpurun_out/pv_b.log 2>&1 &&
MPAS_DYCORE_LIB=exp/lib_t8.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pv_c -o c --output-format csv -- python3 tools/kbench.py --steps 3 --reps 5 > gpurun_out/pv_c.log 2>&1
echo EXIT $?; tail -2 gpurun_out/pytest_gpu.log
