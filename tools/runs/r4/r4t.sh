#!/bin/bash
# chains by default: natural-SSOR tests (bitwise vs the oracle and vs units only), BCGS_SSORk
# time to solution, and a bench run with the new leg
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4t; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ssor_natural.py tests/test_gpu_seq_order.py -x -q --timeout 200 --timeout-method thread > $O/nat_tests.log 2>&1; rc=$?; echo "nat tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_ssor_chain.py -x -q --timeout 800 --timeout-method thread > $O/chain_tests.log 2>&1; rc=$?; echo "chain tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/newton_ssork.py 4 > $O/newton_ssork.log 2>&1; rc=$?; echo "newton rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1; echo "bench rc=$?"
