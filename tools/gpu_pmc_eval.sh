#!/bin/bash
# PMC counters of the evaluation kernel (diagnosis)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_eval
rm -rf $OUT; mkdir -p $OUT
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU" \
           "SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM" "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc --kernel-include-regex "k_eval" --output-format csv -d $OUT/p$i -o run -- \
      python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --event-iters 0 > $OUT/b$i.json 2> $OUT/b$i.err || echo "pass $i failed rc=$?"
done
python3 - <<'PY'
import csv, glob, statistics, collections
res = collections.defaultdict(dict)
for f in glob.glob("gpurun_out/pmc_eval/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void alll::", "")
        res[k].setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, d in res.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:24s} median {statistics.median(v):14.1f}  n={len(v)}")
PY
