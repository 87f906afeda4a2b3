#!/bin/bash
# chain kernel: higher thresholds, and the pipeline lead D (2 / 4 / 6 / 8) at two thresholds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4p; mkdir -p $O
export TMPDIR=/tmp
for T in 16384 32768 65536 1073741824; do
  echo "== chain $T" >> $O/chain_sweep.log
  PNP_NAT_CHAIN=$T timeout -k 10 200 python tools/bench_ssor_natural.py 4 >> $O/chain_sweep.log 2>&1 || exit $?
done
for lib in - cd2 cd6 cd8; do
  if [ "$lib" = "-" ]; then libenv=""; else libenv="PNP_AMD_LIB=dune-pnp_amd/ab/lib_$lib.so"; fi
  for T in 8192 32768; do
    echo "== $lib chain $T" >> $O/chain_d.log
    env $libenv PNP_NAT_CHAIN=$T timeout -k 10 200 python tools/bench_ssor_natural.py 4 >> $O/chain_d.log 2>&1 || exit $?
  done
done
