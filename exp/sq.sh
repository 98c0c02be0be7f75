cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SMEM -d gpurun_out/sq1 -o sq1 --output-format csv -- python3 tools/kbench.py --reps 5 --steps 1 --no-graph > gpurun_out/sq1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_LDS -d gpurun_out/sq2 -o sq2 --output-format csv -- python3 tools/kbench.py --reps 5 --steps 1 --no-graph > gpurun_out/sq2.log 2>&1
echo EXIT $?
