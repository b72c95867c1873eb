#!/bin/bash
# Issue/wait/TA counters of the evaluation kernel at config M (one rocprofv3 pass per group).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_eval2
rm -rf $OUT; mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || echo "list rc=$?"
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA" \
           "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "k_eval" --output-format csv -d $OUT/p$i -o run -- \
      python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --event-iters 0 > $OUT/b$i.json 2> $OUT/b$i.err
  rc=$?; [ $rc -eq 0 ] || { echo "pass $i rc=$rc"; tail -3 $OUT/b$i.err; }
done
python3 tools/pmc_table.py $OUT > $OUT/table.txt; cat $OUT/table.txt
