mkdir -p gpurun_out/r4a
timeout -k 10 400 python -u -m pytest tests/test_gpu_ssor_natural.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4a/tests.log 2>&1; rc=$?; echo "nat tests rc=$rc"
[ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_seq_order.py -v --timeout 120 --timeout-method thread > gpurun_out/r4a/seq.log 2>&1; rc=$?; echo "seq tests rc=$rc"
[ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python -u tools/bench_ssor_natural.py 3 4 > gpurun_out/r4a/bench_flow.log 2>&1 || exit $?
PNP_NAT_FLOW=0 timeout -k 10 200 python -u tools/bench_ssor_natural.py 4 > gpurun_out/r4a/bench_levels.log 2>&1
