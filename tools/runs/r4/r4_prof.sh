#!/bin/bash
# round 4 final: rocprofv3 kernel trace + stats of the default bench at HEAD; the regime split of
# the assembly launches from the trace, then the trace itself is dropped (too large to keep)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4_prof; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu > $O/bench_prof.log 2>&1; echo "prof rc=$?"
T=$(ls $O/prof/run_kernel_trace.csv)
python3 tools/asm_regimes.py $T 353561080 $O/asm_regimes_config3_final.json "k_assemble_ga<0, 1, 3, 9, 6" 738048 > $O/asm_regimes.log 2>&1
python3 tools/nat_split.py $T > $O/nat_split.log 2>&1
rm -f $T
