#!/bin/bash
# Which AMG ingredient made BiCGSTAB diverge on config-4 systems in round 1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "AMG_COARSE=64 AMG_OMEGA=1.0 AMG_PRE=1" "AMG_COARSE=64 AMG_OMEGA=0.8 AMG_PRE=-1" \
         "AMG_COARSE=1024 AMG_OMEGA=1.0 AMG_PRE=-1" "AMG_COARSE=1024 AMG_OMEGA=0.8 AMG_PRE=1" \
         "AMG_COARSE=64 AMG_OMEGA=1.0 AMG_PRE=-1" "AMG_COARSE=1024 AMG_OMEGA=1.0 AMG_PRE=1"; do
  echo "== $v"
  env $v timeout -k 10 150 python tools/amg_config4_scan.py 3 12 | tail -1 || exit $?
done
