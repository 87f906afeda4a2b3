#!/bin/bash
# round 5: leases m and l in one call (m first: the PB A/B and the P_k probe)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
bash tools/runs/r5/m.sh; rc=$?; [ $rc -ne 0 ] && exit $rc
bash tools/runs/r5/l.sh
