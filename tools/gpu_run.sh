#!/bin/bash
# Guarded GPU session: each GPU step under its own time limit; a crash/abort/timeout in any
# step ends the script (no further GPU work), ordinary test failures do not.
# usage: tools/gpu_run.sh <tag> <step>...   steps: tests smoke bench prof
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139|-6|-11) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
for step in "$@"; do
  case $step in
    tests)  timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 600 -rf > "$OUT/tests.log" 2>&1; rc=$? ;;
    smoke)  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$? ;;
    bench)  timeout -k 10 600 python bench.py > "$OUT/bench.log" 2>&1; rc=$? ;;
    benchq) timeout -k 10 600 python bench.py --no-cpu --steps 10 > "$OUT/bench.log" 2>&1; rc=$? ;;
    trace)  timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --no-cpu --no-solve --no-strong --steps 3 --warmup 1 > "$OUT/trace.log" 2>&1; rc=$? ;;
    prof)   timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --no-cpu --no-solve --no-strong --steps 10 > "$OUT/prof.log" 2>&1; rc=$? ;;
    pmcf)   timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 tools/prof_target.py 4 10 10 ilu0 > "$OUT/pmcf.log" 2>&1; rc=$? ;;
    pmcw)   timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run -- python3 tools/prof_target.py 4 10 10 ilu0 > "$OUT/pmcw.log" 2>&1; rc=$? ;;
    pmcsq)  timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_sq" -o run -- python3 tools/prof_target.py 4 10 10 ilu0 > "$OUT/pmcsq.log" 2>&1; rc=$? ;;
    pmcsq2) timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INSTS_VALU --kernel-trace --output-format csv -d "$OUT/pmc_sq2" -o run -- python3 tools/prof_target.py 4 10 10 ilu0 > "$OUT/pmcsq2.log" 2>&1; rc=$? ;;
    pmcmem) rc=0
            for set in "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES" "TCP_PENDING_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES" "TCC_HIT TCC_MISS" "TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM"; do
              tag=$(echo $set | cut -d' ' -f1)
              timeout -k 10 600 rocprofv3 --pmc $set GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_$tag" -o run -- python3 tools/prof_target.py 4 10 10 ilu0 > "$OUT/pmcmem.log" 2>&1; rc=$?
              fatal $rc && break
            done ;;
    calib)  rc=0
            timeout -k 10 120 tools/micro/fetch_calib 2 > "$OUT/calib_stdout.txt" 2> "$OUT/calib.log"; rc=$?
            fatal $rc || [ $rc -ne 0 ] || { timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/calib_fetch" -o run -- tools/micro/fetch_calib 2 >> "$OUT/calib.log" 2>&1; rc=$?; }
            fatal $rc || [ $rc -ne 0 ] || { timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/calib_write" -o run -- tools/micro/fetch_calib 2 >> "$OUT/calib.log" 2>&1; rc=$?; }
            fatal $rc || [ $rc -ne 0 ] || { timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace --output-format csv -d "$OUT/calib_req" -o run -- tools/micro/fetch_calib 2 >> "$OUT/calib.log" 2>&1; rc=$?; } ;;
    ab)     : > "$OUT/ab.log"; rc=0
            for i in 1 2 3; do
              timeout -k 10 120 python tools/runs/ab/ab_asm.py >> "$OUT/ab.log" 2>&1; rc=$?
              fatal $rc && break
            done ;;
    *) echo "unknown step $step"; rc=0 ;;
  esac
  echo "step $step rc=$rc" | tee -a "$OUT/steps.txt"
  tail -5 "$OUT/$step.log" 2>/dev/null
  if fatal $rc; then echo "fatal rc=$rc in $step: stopping"; exit $rc; fi
done
exit 0
