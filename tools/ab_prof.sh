#!/bin/bash
# Kernel stats (rocprofv3 --kernel-trace --stats) of bench.py under several builds of liballl.so
# (build/ab/liballl_<v>.so), for per-kernel A/B comparisons.
# usage: VARIANTS="A B" bash tools/ab_prof.sh [bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${VARIANTS:-A B}; do
  ALLL_LIB_AB=build/ab/liballl_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abp_$v -o run \
      -- python3 bench.py --no-cpu-baseline --event-iters 0 "$@" > gpurun_out/abp_$v.log 2>&1 || exit $?
  echo "== $v"
  f=$(find gpurun_out/abp_$v -name 'run_kernel_stats.csv' | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print('%-40s calls %6s avg %9.1f ns' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])))"
done
