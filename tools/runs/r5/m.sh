#!/bin/bash
# round 5, lease m: A/B of the PB assembly (config 1) with sinh/cosh from one exp + reciprocal
# (ab/lib_pbexp.so) against the in-tree library, interleaved; then the PB-bearing GPU tests on the
# variant; the P_k slot-store probe on ab/lib_probe.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5m; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
for rep in 1 2; do
  for lib in dune-pnp_amd/libpnp_amd.so dune-pnp_amd/ab/lib_pbexp.so; do
    echo "== $lib rep $rep" >> $O/pb.log
    PNP_AMD_LIB=$PWD/$lib timeout -k 10 300 python -u tools/bench_configs.py 1 >> $O/pb.log 2>&1; rc=$?
    echo "config1 $lib rc=$rc"; fatal $rc && exit $rc
  done
done
grep -o '"assemble_us": [0-9.]*' $O/pb.log
PNP_AMD_LIB=$PWD/dune-pnp_amd/ab/lib_pbexp.so timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu.py tests/test_equilibrium.py tests/test_mms.py tests/test_gpu_fans.py > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
fatal $rc && exit $rc
PNP_AMD_LIB=$PWD/dune-pnp_amd/ab/lib_probe.so timeout -k 10 300 python -u tools/probe_pk_stores.py 3 3 64 256 1024 > $O/probe_p3.log 2>&1; rc=$?; echo "probe P3 rc=$rc"; cat $O/probe_p3.log | tail -4
fatal $rc && exit $rc
PNP_AMD_LIB=$PWD/dune-pnp_amd/ab/lib_probe.so timeout -k 10 300 python -u tools/probe_pk_stores.py 2 3 64 256 1024 > $O/probe_p2.log 2>&1; rc=$?; echo "probe P2 rc=$rc"; cat $O/probe_p2.log | tail -4
exit 0
