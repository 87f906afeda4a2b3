set -u
mkdir -p gpurun_out/r6d
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/r6d/tests.log 2>&1; rc=$?; echo tests=$rc; fatal $rc && exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6d/prof -o run -- python3 tools/prof_bicg.py 20 3,5 > gpurun_out/r6d/prof_bicg.log 2>&1; rc=$?; echo prof=$rc; fatal $rc && exit 1
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCC_EA0_RDREQ_DRAM_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/r6d/asm_pmc$i -o run -- python3 tools/asm_pmc.py run > gpurun_out/r6d/asm_pmc$i.log 2>&1; rc=$?; echo "pmc$i ($set)=$rc"; fatal $rc && exit 1
done
exit 0
