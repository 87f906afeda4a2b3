#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_seq_order.py -x -q -k driver --timeout 250 --timeout-method thread -s > $O/driver_ref_order.log 2>&1; echo "driver test rc=$?"
bash tools/r4g.sh
