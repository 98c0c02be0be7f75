# repeated two-rank runs of the one-sided transfer (the buffers mode and pull), to catch intermittent
# hand-off failures: every run must match one block bit for bit.  CASES: ';'-separated argument sets,
# ENVS: ';'-separated environment settings (each case runs under each setting); a failing run prints
# its JSON line (the fields that differ and by how much)
set -o pipefail
IFS=';' read -ra CS <<< "${CASES:---pull 0 --moist;--pull 0;--moist}"
IFS=';' read -ra ES <<< "${ENVS:-MPAS_DYCORE_P2P=1}"
for i in $(seq 1 ${RUNS:-10}); do for E in "${ES[@]}"; do for A in "${CS[@]}"; do
  out=$(env $E timeout -k 10 200 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 tools/p2p_two_ranks.py $A 2>/dev/null)
  rc=$?
  if [ $rc -eq 0 ]; then echo "run $i [$E] [$A] ok"; else echo "run $i [$E] [$A] FAIL rc=$rc $(echo "$out" | grep '^{' || true)"; mkdir -p gpurun_out/trfail; echo "$out" > "gpurun_out/trfail/run${i}_$(echo "$E$A" | tr -dc a-z0-9_)".txt; fi
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
done; done; done
exit 0
