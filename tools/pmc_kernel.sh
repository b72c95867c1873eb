#!/bin/bash
# PMC counters (one rocprofv3 pass per group) of the kernels matching a regex, for any command.
# usage: bash tools/pmc_kernel.sh <out-dir> <kernel-regex> -- <command...>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=$1; RX=$2; shift 2; [ "$1" = "--" ] && shift
mkdir -p $OUT
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pmc --kernel-include-regex "$RX" --output-format csv -d $OUT/p$i -o run -- "$@" \
      > $OUT/c$i.log 2>&1 || { echo "pass $i rc=$?"; tail -3 $OUT/c$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, statistics
from collections import defaultdict
d = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[(r["Kernel_Name"].split("(")[0][-40:], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(d.items()):
    print(f"{k:42s} {c:24s} median {statistics.median(v):14.1f} n={len(v)}")
PY
