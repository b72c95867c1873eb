#!/bin/bash
# Copy the summaries of a tools/gpu_profile.sh <tag>_<cfg> run from gpurun_out/ (scratch) into
# profiles/<tag>_<cfg>/ (committed); for config M the PMC record becomes the one bench.py reads.
# usage: bash tools/save_profile.sh <tag> [cfg] [bench-json]
set -e
cd "$(dirname "$0")/.."
TAG=$1; CFG=${2:-M}; SRC=gpurun_out/prof_${TAG}_${CFG}; DST=profiles/${TAG}_${CFG}
mkdir -p $DST/trace
cp $SRC/summary.txt $SRC/pmc_eval_traffic.json $SRC/bench_*.json $DST/
cp $SRC/trace/run_kernel_stats.csv $SRC/trace/run_domain_stats.csv $DST/trace/
for d in $SRC/pmc_*/; do n=$(basename $d); mkdir -p $DST/$n; cp $d/run_counter_collection.csv $DST/$n/; done
[ -n "$3" ] && cp "$3" $DST/bench_default.json
[ "$CFG" = M ] && cp $SRC/pmc_eval_traffic.json profiles/pmc_eval_traffic.json
python3 tools/timeline.py $SRC/trace/run_kernel_trace.csv ${TL_INDEX:-8} > $DST/iteration_timeline.txt
du -sh $DST
