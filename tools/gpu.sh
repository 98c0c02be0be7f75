# One runner for every GPU-box job (replaces the one-off tools/gpu_*.sh of rounds 1-2).
#
#   gpurun -- 'bash tools/gpu.sh STEP [STEP ...]'
#
# Steps run in order and the run stops at the first failure (each GPU step has its own time
# limit).  Output goes to gpurun_out/<step>.log; a summary line per step goes to stdout.
#   tests            pytest -m "gpu and not slow"            (TESTS="files or -k expr" to narrow)
#   tests_full       pytest -m gpu (full-size BASELINE configs included)
#   bench            bench.py default line (configs[2] mesh, configs[1] line, cpu_baseline)
#   bench_fast       bench.py without cpu_baseline / configs[1] (BENCH_ARGS extra arguments)
#   bench55          bench_fast at 55 levels (the reference's default nVertLevels)
#   moist            bench.py --moist (configs[3])
#   varres           bench.py --varres 835586 (configs[4])
#   prof             rocprofv3 --kernel-trace --stats of bench.py (gpurun_out/prof)
#   pmc              two rocprofv3 --pmc passes, FETCH_SIZE and WRITE_SIZE (gpurun_out/pmc_*)
#   rank             tools/rank_emulation.py --parts 1 2 4 8
#   prof8            rocprofv3 kernel trace of one rank's block of an 8-way split (rank emulation)
#   rank8            every block of the 8-way split alone, compute only and then with its real exchange
#                    lists looped back (tools/rank_emulation.py --exchange), one after the other
#   prof8p           the same with the one-sided transfer (MPAS_DYCORE_P2P=1) in the exchange run (gpurun_out/prof8p)
#   prof8e           rocprofv3 kernel traces of rank8's two modes (gpurun_out/prof8c, gpurun_out/prof8e)
#   blocks8          bench.py --blocks 8 --rccl-local (the 8-GPU decomposition on one device)
#   prof8b           rocprofv3 kernel trace of blocks8 (gpurun_out/prof8b)
#   ab8              blocks8 with the fused exchange packs / unpacks off and on (MPAS_DYCORE_FUSED_PACK), AB_ROUNDS rounds
#   ab               same-box A/B of AB_LIBS (default exp/lib_base.so vs the in-tree library),
#                    AB_ROUNDS rounds of tools/kbench.py (AB_ARGS extra arguments)
#   kprof            rocprofv3 kernel stats of tools/kbench.py for each of AB_LIBS (gpurun_out/kprof_<i>)
#   kpmc             two rocprofv3 --pmc passes (SQ wait/active cycles; TA/TCP/TCC traffic) of one
#                    eager tools/kbench.py dt for each of AB_LIBS (gpurun_out/kpmc_<lib>_<set>)
#   maxedges         bench.py with the mesh declared maxEdges 6 vs 10 (AB_ROUNDS rounds), and from an init file
#                    declaring maxEdges 10 (tools/write_init.py)
#   tworanks         tools/p2p_two_ranks.py: two ranks on the GPU, one-sided transfer over IPC, bitwise vs one block
#   bench2same       bench.py --gpus 2 --same-device: the multi-rank bench path (torchrun, two processes) on the one GPU
#   ipc              tools/p2p_ipc_check: the one-sided protocol between two processes on the GPU (IPC)
#   floor            tools/gather_floor: the gather kernels next to load-only replays of their index streams
#   smoke            __graft_entry__.smoke()
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out || exit 1
B="--no-cpu-baseline --no-configs1"
last() { tail -1 "$1" | cut -c1-${2:-400}; }
step() {
  case "$1" in
    tests) timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m "gpu and not slow" ${TESTS:-tests} > gpurun_out/tests.log 2>&1; r=$?; tail -2 gpurun_out/tests.log; return $r ;;
    tests_full) timeout -k 10 1100 python -u -m pytest -x -v --durations=30 --timeout 900 --timeout-method thread -m gpu ${TESTS:-tests} > gpurun_out/tests_full.log 2>&1; r=$?; tail -2 gpurun_out/tests_full.log; return $r ;;
    bench) timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 && last gpurun_out/bench.log 700 ;;
    bench_fast) timeout -k 10 300 python bench.py --steps 10 --warmup 2 $B ${BENCH_ARGS} > gpurun_out/bench_fast.log 2>&1 && last gpurun_out/bench_fast.log ;;
    bench55) timeout -k 10 300 python bench.py --steps 10 --warmup 2 $B --levels 55 > gpurun_out/bench55.log 2>&1 && last gpurun_out/bench55.log ;;
    moist) timeout -k 10 400 python bench.py --steps 10 --warmup 2 --moist $B > gpurun_out/moist.log 2>&1 && last gpurun_out/moist.log 300 ;;
    varres) timeout -k 10 600 python bench.py --steps 5 --warmup 1 --varres 835586 $B > gpurun_out/varres.log 2>&1 && last gpurun_out/varres.log 300 ;;
    prof) timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 $B ${PROF_ARGS} > gpurun_out/prof.log 2>&1 && last gpurun_out/prof.log 200 ;;
    pmc) A="--steps 1 --warmup 1 $B --no-graph --acoustic-reps 5 ${BENCH_ARGS}" &&
         timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o fetch --output-format csv -- python3 bench.py $A > gpurun_out/pmc_fetch.log 2>&1 &&
         timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o write --output-format csv -- python3 bench.py $A > gpurun_out/pmc_write.log 2>&1 && echo "pmc done" ;;
    rank) timeout -k 10 400 python tools/rank_emulation.py --parts 1 2 4 8 > gpurun_out/rank.log 2>&1 && tail -4 gpurun_out/rank.log ;;
    prof8) timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8 -o run --output-format csv -- python3 tools/rank_emulation.py --parts 8 --steps 10 > gpurun_out/prof8.log 2>&1 && echo "prof8 done" ;;
    rank8) timeout -k 10 400 python tools/rank_emulation.py --parts 1 8 --blocks all > gpurun_out/rank8.log 2>&1 &&
           timeout -k 10 400 python tools/rank_emulation.py --parts 8 --blocks all --exchange >> gpurun_out/rank8.log 2>&1 &&
           grep blocks gpurun_out/rank8.log ;;
    rcclenv) rm -f gpurun_out/rcclenv.log
           for E in "X=0" "NCCL_P2P_LL_THRESHOLD=1048576" "NCCL_P2P_LL_THRESHOLD=1048576 NCCL_NCHANNELS_PER_PEER=1" "NCCL_NCHANNELS_PER_PEER=4" "NCCL_PROTO=LL" ${RCCL_ENVS}; do
             echo "== $E" >> gpurun_out/rcclenv.log
             env $E timeout -k 10 300 python tools/rank_emulation.py --parts 8 --blocks 0 4 --exchange >> gpurun_out/rcclenv.log 2>&1 || return 1
           done; grep -h "==\|blocks" gpurun_out/rcclenv.log | cut -c1-160 ;;
    abenv) rm -f gpurun_out/abenv.log   # same library, ENVS="A=1;A=0" variants, AB_ROUNDS rounds of tools/kbench.py
           IFS=';' read -ra VS <<< "${ENVS:-X=0}"
           for r in ${AB_ROUNDS:-1 2 3}; do for E in "${VS[@]}"; do
             echo "== $E" >> gpurun_out/abenv.log
             env $E timeout -k 10 250 python tools/kbench.py --steps ${AB_STEPS:-10} ${AB_ARGS} >> gpurun_out/abenv.log 2>&1 || return 1
           done; done; grep -h "==\|ms_dt" gpurun_out/abenv.log | cut -c1-130 ;;
    envsweep) rm -f gpurun_out/envsweep.log   # ENVS="A=1 B=2;C=3" (';' between variants), EMU_ARGS for rank_emulation.py
           IFS=';' read -ra VS <<< "${ENVS:-X=0}"
           for r in ${AB_ROUNDS:-1}; do for E in "${VS[@]}"; do
             echo "== $E" >> gpurun_out/envsweep.log
             env $E timeout -k 10 300 python tools/rank_emulation.py ${EMU_ARGS:---parts 8 --blocks 0 4 --exchange} >> gpurun_out/envsweep.log 2>&1 || return 1
           done; done; grep -h "==\|blocks" gpurun_out/envsweep.log | cut -c1-160 ;;
    prof8e) timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8c -o run --output-format csv -- python3 tools/rank_emulation.py --parts ${PROF_PARTS:-8} --blocks ${PROF_BLOCKS:-all} --steps 3 > gpurun_out/prof8c.log 2>&1 &&
            timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8e -o run --output-format csv -- python3 tools/rank_emulation.py --parts 8 --blocks all --steps 3 --exchange > gpurun_out/prof8e.log 2>&1 && echo "prof8e done" ;;
    prof8p) timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8c -o run --output-format csv -- python3 tools/rank_emulation.py --parts ${PROF_PARTS:-8} --blocks ${PROF_BLOCKS:-all} --steps 3 > gpurun_out/prof8c.log 2>&1 &&
            MPAS_DYCORE_P2P=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8p -o run --output-format csv -- python3 tools/rank_emulation.py --parts ${PROF_PARTS:-8} --blocks ${PROF_BLOCKS:-all} --steps 3 --exchange > gpurun_out/prof8p.log 2>&1 && echo "prof8p done" ;;
    blocks8) timeout -k 10 400 python bench.py --blocks 8 --rccl-local --steps 5 --warmup 2 $B > gpurun_out/blocks8.log 2>&1 && last gpurun_out/blocks8.log 300 ;;
    ab8) rm -f gpurun_out/ab8.log
        for r in ${AB_ROUNDS:-1 2 3}; do for F in 0 1; do
          echo "== MPAS_DYCORE_FUSED_PACK=$F" >> gpurun_out/ab8.log
          MPAS_DYCORE_FUSED_PACK=$F timeout -k 10 300 python bench.py --blocks 8 --rccl-local --steps 5 --warmup 2 $B >> gpurun_out/ab8.log 2>&1 || return 1
        done; done; grep -h "==\|ms_per_step" gpurun_out/ab8.log | sed 's/.*"ms_per_step": \([0-9.]*\).*/ms_per_step \1/' ;;
    prof8b) timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8b -o run --output-format csv -- python3 bench.py --blocks 8 --rccl-local --steps 3 --warmup 1 $B > gpurun_out/prof8b.log 2>&1 && echo "prof8b done" ;;
    ab) rm -f gpurun_out/ab.log
        for r in ${AB_ROUNDS:-1 2 3}; do for L in ${AB_LIBS:-exp/lib_base.so mpas-model_amd/csrc/libmpas_dycore.so}; do
          echo "== $L" >> gpurun_out/ab.log
          MPAS_DYCORE_LIB=$L timeout -k 10 250 python tools/kbench.py --steps ${AB_STEPS:-10} ${AB_ARGS} >> gpurun_out/ab.log 2>&1 || return 1
        done; done; grep -h "==\|ms_dt" gpurun_out/ab.log | cut -c1-130 ;;
    kprof) i=0; for L in ${AB_LIBS:-exp/lib_base.so mpas-model_amd/csrc/libmpas_dycore.so}; do
          MPAS_DYCORE_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kprof_$i -o run --output-format csv -- python3 tools/kbench.py --steps ${AB_STEPS:-10} ${AB_ARGS} > gpurun_out/kprof_$i.log 2>&1 || return 1
          echo "kprof_$i = $L"; i=$((i+1)); done ;;
    kpmc) i=0; for L in ${AB_LIBS:-mpas-model_amd/csrc/libmpas_dycore.so}; do j=0
          for C in "${KPMC_SET1:-SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES}" "${KPMC_SET2:-TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum}"; do
            MPAS_DYCORE_LIB=$L timeout -s KILL 240 rocprofv3 --pmc $C -d gpurun_out/kpmc_${i}_$j -o pmc --output-format csv -- python3 tools/kbench.py --steps 1 --reps 1 --no-graph > gpurun_out/kpmc_${i}_$j.log 2>&1 || return 1
            j=$((j+1)); done; echo "kpmc_$i = $L"; i=$((i+1)); done ;;
    maxedges) rm -f gpurun_out/maxedges.log
        for r in ${AB_ROUNDS:-1 2}; do for M in "" "--max-edges 10,20"; do
          echo "== bench $M" >> gpurun_out/maxedges.log
          timeout -k 10 300 python bench.py --steps 10 --warmup 2 $B $M >> gpurun_out/maxedges.log 2>&1 || return 1
        done; done
        timeout -k 10 400 python tools/write_init.py --max-edges 10,20 /tmp/x1.163842.me10.init.nc >> gpurun_out/maxedges.log 2>&1 || return 1
        echo "== bench --init (maxEdges 10)" >> gpurun_out/maxedges.log
        timeout -k 10 400 python bench.py --steps 10 --warmup 2 $B --init /tmp/x1.163842.me10.init.nc --dt 360 --len-disp 60000 >> gpurun_out/maxedges.log 2>&1 || return 1
        grep -h "==\|ms_per_step" gpurun_out/maxedges.log | sed 's/.*"ms_per_step": \([0-9.]*\).*"kernel_layout": \({[^}]*}\).*/ms_per_step \1 \2/' ;;
    floor) timeout -k 10 400 python tools/gather_floor.py ${FLOOR_ARGS} > gpurun_out/floor.log 2>&1; r=$?; cat gpurun_out/floor.log; return $r ;;
    tworanks) rm -f gpurun_out/tworanks.log   # two ranks on the one GPU, one-sided transfer, no RCCL
              for A in "" "--moist" "--pull 0"; do
                timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 tools/p2p_two_ranks.py $A >> gpurun_out/tworanks.log 2>&1 || { tail -30 gpurun_out/tworanks.log; return 1; }
              done; grep bitwise gpurun_out/tworanks.log ;;
    bench2same) timeout -k 10 400 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --same-device --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-configs1 ${B} > gpurun_out/bench2same.log 2>&1 && last gpurun_out/bench2same.log 400 ;;
    ipc) timeout -k 10 600 python tools/p2p_ipc_check.py ${IPC_ARGS} > gpurun_out/ipc.log 2>&1; r=$?; cat gpurun_out/ipc.log; return $r ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && last gpurun_out/smoke.log ;;
    *) echo "unknown step $1"; return 2 ;;
  esac
}
for s in "$@"; do
  echo "### $s"
  step "$s" || { echo "### $s FAILED ($?)"; exit 1; }
done
echo "### all steps ok"
