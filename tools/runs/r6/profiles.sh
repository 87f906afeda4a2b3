#!/bin/bash
# round 6: the committed evidence at HEAD -- kernel trace + stats of the bench's timed regions,
# the per-config BiCGSTAB split, the FETCH_SIZE / WRITE_SIZE passes (config 3, bf16 ILU(0))
set -u
O=gpurun_out/$1; mkdir -p "$O"
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/bench_trace" -o run -- python3 bench.py --no-cpu --no-per-config > "$O/bench_traced.json" 2> "$O/bench_traced.err"; rc=$?; echo "bench trace=$rc"; gzip -f "$O"/bench_trace/*kernel_trace.csv; fatal $rc && exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/bicg" -o run -- python3 tools/prof_bicg.py 20 3,5 > "$O/prof_bicg.log" 2>&1; rc=$?; echo "bicg trace=$rc"; fatal $rc && exit 1
bash tools/gpu_run.sh "$1" pmcf pmcw; rc=$?; echo "pmc=$rc"; fatal $rc && exit 1
F=$(ls "$O"/pmc_fetch/*counter_collection.csv | head -1); W=$(ls "$O"/pmc_write/*counter_collection.csv | head -1)
python tools/pmc_summary.py "$F" "$W" "$O/pmc_summary.json" 10 > "$O/pmc_summary.log" 2>&1
python tools/pmc_kernels.py "$F" "" "$O/pmc_fetch.json" > /dev/null 2>&1
python tools/pmc_kernels.py "$W" "" "$O/pmc_write.json" > /dev/null 2>&1
gzip -f "$F" "$W"
# everything under gpurun_out comes back only below 64 MiB: compress the traces on the box
find "$O" -name "*.csv" -size +1M -exec gzip -f {} \;
exit 0
