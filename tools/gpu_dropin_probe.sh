cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 300 python -u tools/py_step_probe.py > gpurun_out/py_probe.log 2>&1 &&
PROBE_ENV="MPAS_DYCORE_WAIT_EVERY_STEP=1" timeout -k 10 300 python -u tools/dropin_probe.py 163842 > gpurun_out/dropin_probe_wait.log 2>&1
echo EXIT $?
cat gpurun_out/py_probe.log | tail -3; grep -h "step \|total\|after2" gpurun_out/dropin_probe_wait.log | cut -c1-400
