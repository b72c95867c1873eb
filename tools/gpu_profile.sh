#!/bin/bash
# rocprofv3 kernel-trace/stats of the bench + PMC traffic passes for the eval kernel.
# usage: bash tools/gpu_profile.sh <tag> <config> [bench args...]
# Summaries go to gpurun_out/prof_<tag>/ (scratch); copy them into profiles/<tag>/ to commit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r1}; shift
CFG=${1:-M}; shift
ARGS="--config $CFG $@"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --no-cpu-baseline $ARGS > $OUT/bench_traced.json 2> $OUT/bench_traced.err || exit $?
for pmc in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  name=$(echo $pmc | tr ' ' '_')
  timeout -k 10 600 rocprofv3 --pmc $pmc --kernel-include-regex "k_eval" --output-format csv -d $OUT/pmc_$name -o run -- \
      python3 bench.py --no-cpu-baseline $ARGS > $OUT/bench_pmc_$name.json 2> $OUT/bench_pmc_$name.err || exit $?
done
python3 tools/prof_summary.py $OUT $CFG > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
