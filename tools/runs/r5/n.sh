#!/bin/bash
# round 5, lease n: the rebuilt library (PB sinh/cosh from one exp, P1 and P_k; the slot-store
# probe with the tile-sorted order): PB / P_k GPU tests, the probe at P3 / P2, config 1 rates
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5n; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu.py tests/test_equilibrium.py tests/test_mms.py tests/test_gpu_fans.py tests/test_gpu_pk.py tests/test_gpu_pk_res2.py tests/test_gpu_boundary.py tests/test_gpu_seq_order.py > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
fatal $rc && exit $rc
timeout -k 10 300 python -u tools/probe_pk_stores.py 3 3 64 256 1024 > $O/probe_p3.log 2>&1; rc=$?; echo "probe P3 rc=$rc"; cat $O/probe_p3.log | tail -4
fatal $rc && exit $rc
timeout -k 10 300 python -u tools/probe_pk_stores.py 2 3 64 256 1024 > $O/probe_p2.log 2>&1; rc=$?; echo "probe P2 rc=$rc"; cat $O/probe_p2.log | tail -4
fatal $rc && exit $rc
timeout -k 10 300 python -u tools/bench_configs.py 1 > $O/config1.log 2>&1; rc=$?; echo "config1 rc=$rc"; tail -2 $O/config1.log
fatal $rc && exit $rc
PNP_PK_NO_SOLVE=1 timeout -k 10 300 python -u tools/bench_pk.py 3 2 3 > $O/bench_pk.log 2>&1; rc=$?; echo "bench_pk rc=$rc"; tail -2 $O/bench_pk.log
exit 0
