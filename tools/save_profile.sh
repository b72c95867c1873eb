#!/bin/bash
# Copy the summaries of a tools/gpu_full.sh <tag> run from gpurun_out/ (scratch) into
# profiles/<tag>_M/ (committed) and make its PMC record the one bench.py reads.
# usage: bash tools/save_profile.sh <tag>
set -e
cd "$(dirname "$0")/.."
TAG=$1; SRC=gpurun_out/prof_${TAG}_M; DST=profiles/${TAG}_M
mkdir -p $DST/trace
cp $SRC/summary.txt $SRC/pmc_eval_traffic.json $SRC/bench_*.json $DST/
cp $SRC/trace/run_kernel_stats.csv $SRC/trace/run_domain_stats.csv $DST/trace/
for d in $SRC/pmc_*/; do n=$(basename $d); mkdir -p $DST/$n; cp $d/run_counter_collection.csv $DST/$n/; done
cp gpurun_out/bench_${TAG}.json $DST/bench_default.json
cp $SRC/pmc_eval_traffic.json profiles/pmc_eval_traffic.json
python3 tools/timeline.py $SRC/trace/run_kernel_trace.csv 30 > $DST/iteration_timeline.txt
du -sh $DST
