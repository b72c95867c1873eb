#!/bin/bash
# Counters of the round robin's evaluation (k_eval_flags) at M, T = 16, steady state, beside the
# T = 1 evaluation's (k_eval_hybrid / k_eval_scatter, the bench).  One rocprofv3 pass per group.
# usage: bash tools/gpu_pmc_evalflags.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA" \
           "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "WRITE_SIZE TCP_TOTAL_CACHE_ACCESSES_sum" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pmc --kernel-include-regex "k_eval_flags" --output-format csv -d $OUT/rr$i -o run -- \
      python3 tools/rr_bench.py --config M --threads 16 --iters 2 --warmup 20 > $OUT/rr$i.log 2>&1 \
      || { echo "rr pass $i rc=$?"; tail -3 $OUT/rr$i.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc $pmc --kernel-include-regex "k_eval" --output-format csv -d $OUT/t1_$i -o run -- \
      python3 bench.py --no-cpu-baseline --stream-line none --no-shard-line --steps 10 --warmup 2 > $OUT/t1_$i.log 2>&1 \
      || { echo "t1 pass $i rc=$?"; tail -3 $OUT/t1_$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, statistics
from collections import defaultdict
d = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[(r["Kernel_Name"].split("(")[0][-32:], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(d.items()):
    print(f"{k:34s} {c:32s} median {statistics.median(v):16.1f} n={len(v)}")
PY
