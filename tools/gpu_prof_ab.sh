#!/bin/bash
# Kernel-trace A/B of build/ab/liballl_{A,X}.so (tools/build_variant.sh) on one config:
# rocprofv3 --kernel-trace --stats of the bench, then the round-0 kernels' averages.
# usage: bash tools/gpu_prof_ab.sh [config]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
CFG=${1:-C5}
for v in ${VARIANTS:-A X}; do
  ALLL_LIB_AB=build/ab/liballl_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/pab_$v -o run -- python3 bench.py --no-cpu-baseline --no-rr-line --stream-line none --config $CFG \
      > gpurun_out/pab_$v.json 2> gpurun_out/pab_$v.err
  rc=$?; echo "$v rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
  grep -E "bscatter|bresolve|bjoin" gpurun_out/pab_$v/run_kernel_stats.csv | cut -d, -f1-5
done
