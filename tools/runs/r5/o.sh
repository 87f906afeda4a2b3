#!/bin/bash
# round 5, lease o: where a BiCGSTAB + AMG(ILU(0)) iteration's time goes at config 3 (kernel trace);
# the PB per-vertex-exp A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/prof_amg.py run 40 > $O/run.log 2>&1; rc=$?; echo "prof rc=$rc"; tail -2 $O/run.log
[ $rc -ne 0 ] && exit $rc
f=$(find $O/prof -name "*kernel_trace.csv" | head -1); echo "trace: $f"
python3 tools/prof_amg.py split "$f" 40 > $O/split.txt 2>&1; head -50 $O/split.txt
s=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$s" $O/kernel_stats.csv
gzip -c "$f" > $O/trace.csv.gz; rm -rf $O/prof
# PB: the quadrature points' e^u from per-vertex e^{u/5} (ab/lib_pbv.so) against HEAD, interleaved
for rep in 1 2; do
  for lib in dune-pnp_amd/libpnp_amd.so dune-pnp_amd/ab/lib_pbv.so; do
    echo "== $lib rep $rep" >> $O/pb.log
    PNP_AMD_LIB=$PWD/$lib timeout -k 10 300 python -u tools/bench_configs.py 1 >> $O/pb.log 2>&1; rc=$?
    echo "config1 $lib rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
grep -o '"assemble_us": [0-9.]*' $O/pb.log
PNP_AMD_LIB=$PWD/dune-pnp_amd/ab/lib_pbv.so timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu -k "not cpp_driver" tests/test_gpu.py tests/test_equilibrium.py tests/test_mms.py tests/test_gpu_fans.py tests/test_gpu_asm_lds.py tests/test_gpu_boundary.py > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
exit 0
