#!/bin/bash
# round 5, lease t2 (bf16 factors): counters per ILU(0) colour launch at config 3 (why fwd colour 1 and bwd
# colour 0 take 12-13 us while bwd colour 1 takes 8): four separate --pmc passes over
# tools/prof_bicg.py 20 3, split by kernel and grid (tools/pmc_kernels.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5t2; mkdir -p $O
export TMPDIR=/tmp
run() {  # name, counters...
  local n=$1; shift
  timeout -s KILL 200 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$n -o run -- python3 tools/prof_bicg.py 20 3 > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; [ $rc -ne 0 ] && return $rc
  f=$(find $O/$n -name "*counter_collection.csv" | head -1)
  python3 tools/pmc_kernels.py "$f" "" $O/$n.json > $O/$n.txt 2>&1
  rm -rf $O/$n
  return 0
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU && \
run mem TCC_HIT_sum TCC_MISS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE && \
run fetch FETCH_SIZE && \
run write WRITE_SIZE
grep -h "k_ilu0_solve_lds\|k_update_fwd0" $O/sq.txt $O/mem.txt $O/fetch.txt $O/write.txt | cut -c1-400
exit 0
