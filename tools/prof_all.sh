#!/usr/bin/env bash
# Every BASELINE config through tools/profile.sh (trace + FETCH + WRITE passes),
# then SQ counters for the configs named in SQ_WLS.  Stops at the first failure.
#   TAG=r02 bash tools/prof_all.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TAG="${TAG:-r02}"
for spec in ${WLS:-cfg1:268435456 cfg1 cfg2 cfg3 cfg4 cfg5}; do
  wl=${spec%%:*}; pk=""; [ "$spec" != "$wl" ] && pk=${spec#*:}
  if [ -n "$pk" ]; then
    WL=$wl PKTS=$pk TAG=${TAG}_${pk} bash tools/profile.sh || exit $?
  else
    WL=$wl bash tools/profile.sh || exit $?
  fi
done
for wl in ${SQ_WLS:-cfg2 cfg4 cfg5}; do
  WL=$wl bash tools/sq_profile.sh || exit $?
done
echo "== prof_all done"
