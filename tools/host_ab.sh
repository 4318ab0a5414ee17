#!/usr/bin/env bash
# Host-side A/B of the TX path: the current drop-in + libpipck against the copies in
# pip_amd/lib/ab_base (LD_LIBRARY_PATH wins over the benches' RUNPATH), rounds
# alternated, on pip's UDP (1,472-B datagrams) and TCP (MSS 1,460, 4 connections)
# TX paths, capture + zero-copy, pipelined.  Digests must agree.  GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/host_ab
mkdir -p "$OUT"
B=oracle/_ref
for r in 1 2 3; do
  for arm in base cur; do
    if [ $arm = base ]; then LP="$PWD/pip_amd/lib/ab_base"; else LP=""; fi
    for spec in "stack_udp_amd --mode capture_zc --pipeline --family 4 --len 1472 --batch 1024 --bytes $((1 << 30))" \
                "stack_tx_amd --mode capture_zc --pipeline --conns 4 --mss 1460 --bytes $((1 << 30)) --write $((4 << 20))"; do
      set -- $spec
      line=$(LD_LIBRARY_PATH="$LP" timeout -k 10 120 "$B/$1" "${@:2}" 2>> "$OUT/err.log") || { rc=$?; [ $rc -eq 3 ] || { echo "rc=$rc $spec"; exit 1; }; }
      echo "{\"arm\": \"$arm\", \"round\": $r, \"line\": $line}" | tee -a "$OUT/host_ab.jsonl" | cut -c1-220
    done
  done
done
