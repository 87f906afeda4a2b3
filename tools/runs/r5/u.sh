#!/bin/bash
# round 5, lease u: the per-launch floor of a colour-launch-shaped kernel (tools/micro/launch_floor)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5u; mkdir -p $O
for w in 256 800 1600 3200; do
  timeout -k 10 60 ./tools/micro/launch_floor $w 200 >> $O/launch_floor.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "rc=$rc"; exit $rc; }
done
cat $O/launch_floor.log
exit 0
