# Kernel trace of one rank's block of an 8-way split (rank emulation), to see where a rank's dt goes
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8 -o run --output-format csv -- python3 tools/rank_emulation.py --parts 8 --steps 10 > gpurun_out/prof8.log 2>&1
echo EXIT $?; tail -2 gpurun_out/prof8.log; find gpurun_out/prof8 -name "*.csv" | head
