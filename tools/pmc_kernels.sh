# Per-kernel execution counters (SQ wave-state buckets, TA busy, GRBM clock) of the kbench
# workload, eager launches so each dispatch carries its own counters; one rocprofv3 --pmc pass
# per counter group (MI355X_MICROARCH.md "rocprofv3 PMC slots").  Summarise with
# tools/pmc_kernels.py gpurun_out/pmck.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/pmck &&
ARGS="--steps 1 --no-graph --reps 5" &&
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM -d gpurun_out/pmck/sq -o sq --output-format csv -- python3 tools/kbench.py $ARGS > gpurun_out/pmck/sq.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM -d gpurun_out/pmck/sq2 -o sq2 --output-format csv -- python3 tools/kbench.py $ARGS > gpurun_out/pmck/sq2.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmck/ta -o ta --output-format csv -- python3 tools/kbench.py $ARGS > gpurun_out/pmck/ta.log 2>&1
echo EXIT $?
