#!/bin/bash
# PMC counters of the LFMIS kernels and the evaluation (one rocprofv3 pass per counter group;
# each pass is its own bounded step, the script stops at the first failure).
# usage: bash tools/gpu_pmc_mis.sh <tag> [config]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r2}; CFG=${2:-M}
OUT=gpurun_out/pmc_mis_${TAG}_${CFG}
mkdir -p $OUT
REGEX="k_eval|k_b|k_claim|k_join|k_w|k_tail|k_resample"
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pmc --kernel-include-regex "$REGEX" --output-format csv -d $OUT/p$i -o run -- \
      python3 bench.py --config $CFG --no-cpu-baseline --steps 10 --warmup 2 --event-iters 0 \
      > $OUT/b$i.json 2> $OUT/b$i.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i ($pmc) failed rc=$rc"; tail -5 $OUT/b$i.err; exit $rc; fi
done
python3 tools/pmc_table.py $OUT > $OUT/table.txt && cat $OUT/table.txt
