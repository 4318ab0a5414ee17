#!/bin/bash
# Round 6: the ring verifier's default schedule on the final build against the
# round-5 build (pip_amd/lib/ab/libpipck_r05.so, PIPCK_LIB) on one box,
# processes alternating r05 / r06 twice ("no slower than
# r05"). Output: gpurun_out/ring_vs_r05_<build>_<pass>.jsonl
# The round-5 library is git-ignored; rebuild it (sha256 2288e7e3...) with
#   d=$(mktemp -d) && git archive 5b004ec | tar -x -C $d && make -C $d/pip_amd lib/libpipck.so \
#     && mkdir -p pip_amd/lib/ab && cp $d/pip_amd/lib/libpipck.so pip_amd/lib/ab/libpipck_r05.so
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
RINGS=${RINGS:-ring_sparse_9216,ring_dense_1536,ring_dense_9216,ring_short_2048,ring_short_1024}
for pass in 1 2; do
  for build in r05 r06; do
    if [ $build = r05 ]; then lib=pip_amd/lib/ab/libpipck_r05.so; arms=groups; else lib=; arms=groups,kring; fi
    PIPCK_LIB=$lib timeout -k 10 240 python3 -u tools/rx_device_bench.py --skip-packed --rings $RINGS --arms $arms \
      > gpurun_out/ring_vs_r05_${build}_$pass.jsonl 2> gpurun_out/ring_vs_r05_${build}_$pass.err \
      || { tail -20 gpurun_out/ring_vs_r05_${build}_$pass.err; exit 1; }
    echo "== $build pass $pass done $(date +%T)"
  done
done
python3 - <<'EOF'
import json, glob
for f in sorted(glob.glob("gpurun_out/ring_vs_r05_*.jsonl")):
    for l in open(f):
        d = json.loads(l)
        print(f.split("ring_vs_r05_")[1][:-6], d["what"], d["schedule"], d["ms"], d["frac"], d["last_kernel"][-16:])
EOF
