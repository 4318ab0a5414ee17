#!/usr/bin/env bash
# pip's TCP TX path at volume over IPv6 (oracle/stack_tx_bench.cpp --family 6): wire digests
# across pip's build and the drop-in's modes, then throughput lines.  GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/stack_tx6
mkdir -p "$OUT"
B=oracle/_ref
run() {
  timeout -k 10 ${T:-120} "$B/$1" --family 6 "${@:2}" >> "$OUT/stack_tx6.jsonl" 2>> "$OUT/stack_tx6.err"
  local rc=$?
  [ $rc -eq 0 ] || [ $rc -eq 3 ] || { echo "rc=$rc $*"; exit 1; }
  tail -1 "$OUT/stack_tx6.jsonl" | cut -c1-200
}
for mss in ${MSS:-1440 8940}; do
  run stack_tx_ref --mss $mss --bytes $((64 << 20)) --verify
  run stack_tx_amd --mode sync --mss $mss --bytes $((16 << 20)) --verify
  run stack_tx_ref --mss $mss --bytes $((16 << 20)) --verify
  for m in capture capture_zc; do run stack_tx_amd --mode $m --mss $mss --bytes $((64 << 20)) --verify; done
  run stack_tx_ref --mss $mss --bytes $((64 << 20)) --conns 2 --verify
  run stack_tx_amd --mode capture_zc --pipeline --conns 2 --mss $mss --bytes $((64 << 20)) --verify
  for w in 1048576 4194304; do
    run stack_tx_ref --mss $mss --bytes $((1 << 30)) --write $w
    run stack_tx_zero --mode zero --mss $mss --bytes $((1 << 30)) --write $w
    run stack_tx_amd --mode capture_zc --mss $mss --bytes $((1 << 30)) --write $w
    run stack_tx_amd --mode capture_zc --pipeline --conns 4 --mss $mss --bytes $((1 << 30)) --write $w
  done
done
echo "== stack_tx6 done"
