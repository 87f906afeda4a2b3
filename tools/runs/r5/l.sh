#!/bin/bash
# round 5, lease l: rehearse the N > 1 bench on the one-GPU box -- two ranks through the
# host-staged transport (gloo), both on device 0 -- and the new partitioned dataflow-SSOR test
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5l; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread "tests/test_gpu_ssor_natural.py::test_ssor_natural_on_two_ranks_is_block_jacobi" tests/test_gpu_dist_host.py > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
fatal $rc && exit $rc
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --transport host --steps 3 --warmup 1 --bicg-iters 5 --no-cpu > $O/bench2.log 2>&1; rc=$?; echo "bench N=2 host rc=$rc"; tail -c 1500 $O/bench2.log
exit 0
