#!/usr/bin/env bash
# SQ instruction-mix / stall counters (two passes, counters only) for a bench workload:
#   WL=cfg4 [PKTS=n] bash tools/sq_profile.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
WL="${WL:-cfg4}"
OUT="gpurun_out/sq_${WL}"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
    SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d "$OUT/pmc" -o run --output-format csv -- \
    python3 bench.py --workload "$WL" ${PKTS:+--packets-per-gpu $PKTS} --no-cpu --steps 2 --warmup 1 > "$OUT/bench.json" 2> "$OUT/err.log" || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
    SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD -d "$OUT/pmc2" -o run --output-format csv -- \
    python3 bench.py --workload "$WL" ${PKTS:+--packets-per-gpu $PKTS} --no-cpu --steps 2 --warmup 1 > "$OUT/bench2.json" 2> "$OUT/err2.log"
rc=$?
[ $rc = 0 ] && for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d "$OUT/pmc_$c" -o run --output-format csv -- \
    python3 bench.py --workload "$WL" ${PKTS:+--packets-per-gpu $PKTS} --no-cpu --steps 2 --warmup 1 \
    > /dev/null 2> "$OUT/err_$c.log" || { rc=$?; break; }
done
tail -2 "$OUT/err2.log"
exit $rc
