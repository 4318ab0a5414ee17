# result-store cache policy (kStoreSc1 in pipck_device.hpp) A/B over builds in pip_amd/lib/ab/libpipck_polN.so: cfg2 and cfg4 bench lines
set -u
cd "${GRAFT_REPO_ROOT:-.}"
A="cur=pip_amd/lib/libpipck.so pol1=pip_amd/lib/ab/libpipck_pol1.so pol3=pip_amd/lib/ab/libpipck_pol3.so pol17=pip_amd/lib/ab/libpipck_pol17.so pol18=pip_amd/lib/ab/libpipck_pol18.so pol19=pip_amd/lib/ab/libpipck_pol19.so"
ARMS="$A" ROUNDS=3 WL=cfg2 TAG=pol_cfg2 bash tools/bench_ab.sh > /dev/null || exit 1
ARMS="$A" ROUNDS=2 WL=cfg4 TAG=pol_cfg4 bash tools/bench_ab.sh > /dev/null || exit 1
cat gpurun_out/pol_cfg2.jsonl gpurun_out/pol_cfg4.jsonl
