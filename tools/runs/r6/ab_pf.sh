#!/bin/bash
# round 6: ILU(0) sweep prefetch A/B (in-tree ILU_PF=8 against ab/lib_pf0.so), ILU bitwise tests,
# config-5 FETCH_SIZE / WRITE_SIZE passes of the BiCGSTAB kernels
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_ilu_lds.py tests/test_gpu_xdefer.py tests/test_gpu_ilu_flow.py tests/test_gpu_amg.py "tests/test_gpu.py" -k "ilu or ILU or amg or bicgstab" -q --timeout 200 --timeout-method thread -rf > "$OUT/tests.log" 2>&1; rc=$?; echo tests=$rc; fatal $rc && exit 1
: > "$OUT/ab.log"
for i in 1 2 3; do
  for lib in - pf0; do
    if [ "$lib" = "-" ]; then libenv=""; else libenv="PNP_AMD_LIB=dune-pnp_amd/ab/lib_$lib.so"; fi
    env $libenv timeout -k 10 200 python tools/time_bicg.py 3,5 200 >> "$OUT/ab.log" 2>&1; rc=$?; fatal $rc && exit 1
  done
done
echo ab=done
if [ "${2:-}" = "pmc" ]; then
  for set in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/pmc5_$set" -o run -- python3 tools/prof_bicg.py 10 5 > "$OUT/pmc5_$set.log" 2>&1; rc=$?; echo "pmc $set=$rc"; fatal $rc && exit 1
  done
fi
exit 0
