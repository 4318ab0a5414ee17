#!/usr/bin/env bash
# Round-4 GPU session on one box: GPU tests, then the VERDICT r03 measurement
# arms (XCD-weighted deal on cfg2, k_hdr result stream at 256M headers with
# PMC passes) and a same-box A/B of this build against round 3's library.
# STEPS picks a subset (boxid tests xw hdr box bench ab); the first failure stops.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${TAG:-s1}"
OUT="gpurun_out/r04_$TAG"
mkdir -p "$OUT"
for step in ${STEPS:-tests xw hdr ab}; do
  echo "== $step $(date +%T)"
  case $step in
    boxid) # which machine / GPU this is (fresh boxes per call: compare sessions)
           { echo "boot_id $(cat /proc/sys/kernel/random/boot_id)"; timeout 60 rocm-smi --showuniqueid --showserial --showbus 2>&1 | grep -E "GPU|0x|Serial|Unique|PCI" | head -8; } \
             > "$OUT/boxid.txt" 2>&1; cat "$OUT/boxid.txt" ;;
    tests) timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
             > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -40 "$OUT/pytest.log"; exit 1; }
           tail -2 "$OUT/pytest.log" ;;
    xw)    timeout -k 10 300 python3 -u tools/xcd_weight_ab.py > "$OUT/xw.jsonl" 2> "$OUT/xw.err" \
             || { echo "xw rc=$?"; tail -20 "$OUT/xw.err"; exit 1; }
           tail -1 "$OUT/xw.jsonl" ;;
    hdr)   TAG=$TAG bash tools/hdr_spread.sh > "$OUT/hdr.log" 2>&1 || { echo "hdr failed"; tail -20 "$OUT/hdr.log"; exit 1; }
           tail -3 "$OUT/hdr.log" ;;
    box)   # this box's memory system alone: a loads-only row stream (k_flat's schedule) and the
           # same stream ending every task in block-coalesced sc1 result stores (tools/probe)
           PROBE_ARMS=disp_u24_w4_t64,coop_u24_w4_t64 timeout -k 10 120 pip_amd/lib/stream_probe 6.216,5.369 3 \
             > "$OUT/stream_probe.jsonl" 2> "$OUT/stream_probe.err" || { echo "stream_probe rc=$?"; exit 1; }
           PROBE_ARMS=nt_none,nt_block_stsc1,nt_spread timeout -k 10 120 pip_amd/lib/write_probe 6.216 64 44 \
             > "$OUT/write_probe.jsonl" 2> "$OUT/write_probe.err" || { echo "write_probe rc=$?"; exit 1; }
           tail -3 "$OUT/write_probe.jsonl" ;;
    bench) for wl in ${BENCH_WLS:-cfg2 cfg5}; do
             timeout -k 10 300 python3 bench.py --workload $wl --no-cpu > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" \
               || { echo "bench $wl rc=$?"; tail -5 "$OUT/bench_$wl.err"; exit 1; }
           done
           tail -c 300 "$OUT/bench_cfg5.json" ;;
    ab)    timeout -k 10 900 python3 -u tools/ab_scan.py --only ${AB_ONLY:-cfg4b,cfg2,cfg5} --rounds ${ROUNDS:-3} \
             pip_amd/lib/ab/libpipck_r03.so > "$OUT/ab.jsonl" 2> "$OUT/ab.err" \
             || { echo "ab rc=$?"; tail -20 "$OUT/ab.err"; exit 1; }
           cat "$OUT/ab.jsonl" ;;
  esac
done
echo "== session done $(date +%T)"
