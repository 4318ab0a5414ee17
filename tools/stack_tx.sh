#!/usr/bin/env bash
# pip's TCP TX path at volume (oracle/stack_tx_bench.cpp) on pip's own build and on the
# drop-in's three modes; every line carries the wire digest.  GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/stack_tx
mkdir -p "$OUT"
B=oracle/_ref
run() {  # $1 = binary, rest = args
  # rc 3 = pip's timer thread resent a segment (a >1 s stall somewhere): recorded in the line, not fatal
  timeout -k 10 ${T:-120} "$B/$1" "${@:2}" >> "$OUT/stack_tx.jsonl" 2>> "$OUT/stack_tx.err"
  local rc=$?
  [ $rc -eq 0 ] || [ $rc -eq 3 ] || { echo "rc=$rc $*"; exit 1; }
  tail -1 "$OUT/stack_tx.jsonl"
}
[ "${ONLY_PIPE:-0}" = 1 ] || for mss in ${MSS:-1460 8960}; do
  # wire bytes: every byte hashed, equal across the four
  run stack_tx_ref --mss $mss --bytes $((64 << 20)) --verify
  run stack_tx_amd --mode sync --mss $mss --bytes $((16 << 20)) --verify
  run stack_tx_ref --mss $mss --bytes $((16 << 20)) --verify
  for m in capture capture_zc; do run stack_tx_amd --mode $m --mss $mss --bytes $((64 << 20)) --verify; done
  # throughput (fields digest)
  for w in ${WRITES:-1048576 4194304 16777216}; do
    run stack_tx_ref --mss $mss --bytes $((1 << 30)) --write $w
    run stack_tx_zero --mode zero --mss $mss --bytes $((1 << 30)) --write $w
    for m in capture capture_zc; do run stack_tx_amd --mode $m --mss $mss --bytes $((1 << 30)) --write $w; done
  done
  run stack_tx_amd --mode sync --mss $mss --bytes $((32 << 20))
done
# pipelined: K connections written in turn, each write's batch overlapping the next write
for mss in ${MSS:-1460 8960}; do
  for k in ${CONNS:-2 4}; do
    for w in ${PWRITES:-1048576 4194304}; do
      run stack_tx_ref --mss $mss --bytes $((1 << 30)) --write $w --conns $k
      run stack_tx_zero --mode zero --mss $mss --bytes $((1 << 30)) --write $w --conns $k
      run stack_tx_amd --mode capture_zc --mss $mss --bytes $((1 << 30)) --write $w --conns $k
      run stack_tx_amd --mode capture_zc --mss $mss --bytes $((1 << 30)) --write $w --conns $k --pipeline
    done
  done
done
