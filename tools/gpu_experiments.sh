#!/bin/bash
# timing-only kernel variants (ALLL_EXPERIMENT): rocprofv3 kernel timeline of one iteration each
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/experiments.txt
: > $OUT
for x in ${EXPERIMENTS:-0 1 2}; do
  echo "=== ALLL_EXPERIMENT=$x" >> $OUT
  rm -rf gpurun_out/exp_$x
  ALLL_EXPERIMENT=$x timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/exp_$x -o run -- \
     python3 bench.py --no-cpu-baseline --steps 20 --warmup 2 --event-iters 0 > /dev/null 2>&1 || { echo "failed" >> $OUT; break; }
  python3 tools/timeline.py $(find gpurun_out/exp_$x -name "*kernel_trace.csv" | head -1) 12 >> $OUT
done
cat $OUT
