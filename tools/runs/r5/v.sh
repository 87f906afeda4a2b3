#!/bin/bash
# round 5, lease v: launch floor, eager and hipGraph-replayed (tools/micro/launch_floor)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5v; mkdir -p $O
for w in 800 2883; do
  timeout -k 10 60 ./tools/micro/launch_floor $w 200 >> $O/launch_floor.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "rc=$rc"; cat $O/launch_floor.log; exit $rc; }
done
cat $O/launch_floor.log
exit 0
