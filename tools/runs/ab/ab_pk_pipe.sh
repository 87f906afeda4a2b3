set -u
mkdir -p gpurun_out/r2w
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_pk.py > gpurun_out/r2w/pk_tests.log 2>&1 || exit $?
for i in 1 2; do
  PNP_PK_NO_SOLVE=1 timeout -k 10 200 python tools/bench_pk.py 3 2 3 > gpurun_out/r2w/pk_new_$i.log 2>&1 || exit $?
  PNP_PK_NO_SOLVE=1 PNP_AMD_LIB=dune-pnp_amd/ab/lib_pkbase.so timeout -k 10 200 python tools/bench_pk.py 3 2 3 > gpurun_out/r2w/pk_base_$i.log 2>&1 || exit $?
done
