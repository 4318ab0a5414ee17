#!/usr/bin/env bash
# pip's UDP TX path at volume (oracle/stack_udp_bench.cpp: pip_udp::output per datagram)
# on pip's own build, on checksums that return 0 (the path's ceiling) and on the
# drop-in's modes; every line carries its digest.  GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/stack_udp
mkdir -p "$OUT"
B=oracle/_ref
run() {  # $1 = binary, rest = args
  timeout -k 10 ${T:-120} "$B/$1" "${@:2}" >> "$OUT/stack_udp.jsonl" 2>> "$OUT/stack_udp.err" || { echo "rc=$? $*"; exit 1; }
  tail -1 "$OUT/stack_udp.jsonl"
}
for fl in ${FAMS:-"6 8952" "4 8972" "4 1472"}; do
  set -- $fl; fam=$1; len=$2
  # wire bytes: every byte hashed, equal across pip's build and every mode
  run stack_udp_ref --family $fam --len $len --bytes $((64 << 20)) --verify
  run stack_udp_amd --mode sync --family $fam --len $len --bytes $((8 << 20)) --verify
  run stack_udp_ref --family $fam --len $len --bytes $((8 << 20)) --verify
  for m in capture capture_zc; do run stack_udp_amd --mode $m --family $fam --len $len --bytes $((64 << 20)) --verify; done
  run stack_udp_amd --mode capture_zc --pipeline --family $fam --len $len --bytes $((64 << 20)) --verify
  # throughput (header digest)
  run stack_udp_ref --family $fam --len $len --bytes $((1 << 30))
  run stack_udp_zero --mode zero --family $fam --len $len --bytes $((1 << 30))
  for b in ${BATCHES:-256 1024 4096}; do
    for m in capture capture_zc; do run stack_udp_amd --mode $m --family $fam --len $len --batch $b --bytes $((1 << 30)); done
    run stack_udp_amd --mode capture_zc --pipeline --family $fam --len $len --batch $b --bytes $((1 << 30))
  done
done
echo "== stack_udp done"
