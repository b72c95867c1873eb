#!/bin/bash
# Issue counters of the evaluation kernel for several builds (build/ab/liballl_<v>.so), one
# rocprofv3 pass each.  usage: VARIANTS="A B" bash tools/pmc_ab.sh [counters]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
PMC=${1:-"SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_ANY"}
for v in ${VARIANTS:-A B}; do
  ALLL_LIB_AB=build/ab/liballl_$v.so timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-include-regex "k_eval" \
      --output-format csv -d gpurun_out/pmcab/p_$v -o run -- \
      python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --event-iters 0 > /dev/null 2>&1 || { echo "pmc $v failed"; exit 1; }
  echo "== $v"; python3 tools/pmc_table.py gpurun_out/pmcab | grep -v "^k_"; rm -rf gpurun_out/pmcab_done_$v; mv gpurun_out/pmcab/p_$v gpurun_out/pmcab_done_$v
done
