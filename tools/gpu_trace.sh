#!/bin/bash
# rocprofv3 kernel trace of a short bench run per config + the kernel timeline of one
# graph-replayed iteration.  usage: bash tools/gpu_trace.sh <tag> "M C5 ..." [extra bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1; CFGS=$2; shift 2
for c in $CFGS; do
  OUT=gpurun_out/trace_${TAG}_$c
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
      python3 bench.py --config $c --no-cpu-baseline --steps 20 --warmup 4 --event-iters 0 "$@" \
      > $OUT/bench.json 2> $OUT/bench.err || { echo "trace $c failed"; tail -5 $OUT/bench.err; exit 1; }
  f=$(find $OUT -name "*kernel_trace.csv" | head -1)
  echo "== $c"; python3 tools/timeline.py $f 10 | tee $OUT/timeline.txt
done
