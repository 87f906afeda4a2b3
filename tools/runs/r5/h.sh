#!/bin/bash
# round 5, lease h: two-process host-transport test; then lease g's natural SSOR -- d read at internal positions, gather after; A/B of the
# 32-entry flow head (PNP_NAT_FLOW_KS4)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5h; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 250 --timeout-method thread tests/test_gpu_dist_host.py > $O/dist_host.log 2>&1; rc=$?; echo "dist host rc=$rc"; tail -5 $O/dist_host.log
fatal $rc && exit $rc
for k in 1 0 1 0; do
  PNP_NAT_FLOW_KS4=$k timeout -k 10 200 python -u tools/bench_ssor_natural.py 4 > $O/nat_ks4_$k.log 2>&1; rc=$?; echo "nat ks4=$k rc=$rc"; cat $O/nat_ks4_$k.log
  fatal $rc && exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/bench_ssor_natural.py 4 > $O/trace.log 2>&1; rc=$?; echo "trace rc=$rc"
fatal $rc && exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ssor_natural.py tests/test_gpu_ssor_chain.py tests/test_gpu_seq_order.py tests/test_gpu_rccl.py tests/test_gpu_graph.py tests/test_gpu.py > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
fatal $rc && exit $rc
# the assembly's just-in-time LDS walk (4 waves/SIMD) against the register-gathered one
timeout -k 10 400 python -u -m pytest -x -q --timeout 350 --timeout-method thread tests/test_gpu_asm_lds.py > $O/tests_asm.log 2>&1; rc=$?; echo "asm tests rc=$rc"; tail -2 $O/tests_asm.log
fatal $rc && exit $rc
for i in 1 2; do for j in 1 0; do
  PNP_ASM_JIT=$j timeout -k 10 300 python -u bench.py --no-cpu --no-solve --no-strong --no-ssork --no-per-config --no-amg --steps 20 > $O/asm_jit${j}_$i.log 2>&1; rc=$?; echo "asm jit=$j rc=$rc"
  fatal $rc && exit $rc
  python - $O/asm_jit${j}_$i.log <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print("warm", round(d["roofline"]["avg_launch_us"], 2), "in_situ", round(d["roofline_in_situ"]["avg_launch_us"], 2), "cold", round(d["roofline_cold"]["avg_launch_us"], 2))
PY
done; done
exit 0
