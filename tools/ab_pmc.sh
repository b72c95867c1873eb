#!/bin/bash
# PMC counters of one kernel for several builds (build/ab/liballl_<v>.so), one rocprofv3 pass per
# counter group.  usage: VARIANTS="A B" bash tools/ab_pmc.sh <config> <kernel-regex> [steps]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
CFG=$1; RX=$2; ST=${3:-10}
for v in ${VARIANTS:-A B}; do
  i=0
  for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
             "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM"; do
    i=$((i+1)); OUT=gpurun_out/abpmc_${CFG}_$v/p$i
    mkdir -p $OUT
    ALLL_LIB_AB=build/ab/liballl_$v.so timeout -s KILL 150 rocprofv3 --pmc $pmc --kernel-include-regex "$RX" \
        --output-format csv -d $OUT -o run -- python3 bench.py --config $CFG --no-cpu-baseline --steps $ST --warmup 2 \
        --event-iters 0 > $OUT/b.json 2> $OUT/b.err
    rc=$?; [ $rc -eq 0 ] || { echo "pmc $v pass $i rc=$rc"; tail -3 $OUT/b.err; }
  done
  echo "== $v"; python3 tools/pmc_table.py gpurun_out/abpmc_${CFG}_$v | tee gpurun_out/abpmc_${CFG}_$v/table.txt
done
