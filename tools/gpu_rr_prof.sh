#!/bin/bash
# Kernel trace of the round-robin loop at M (T given, default 16): rocprofv3 stats + a per-kernel
# table.  usage: bash tools/gpu_rr_prof.sh <tag> [T]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-rrp}; T=${2:-16}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/trace -o run -- \
    python3 tools/rr_bench.py --config M --threads $T --iters 3 --warmup 1 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/err.log
rc=$?; cat gpurun_out/$TAG/bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/$TAG/err.log; exit $rc; }
f=$(find gpurun_out/$TAG/trace -name '*kernel_stats.csv' | head -1)
python3 - "$f" << 'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:25]:
    print(f"{r['Name'][:60]:60s} calls={int(r['Calls']):7d} avg_us={float(r['AverageNs'])/1e3:9.2f} total_ms={float(r['TotalDurationNs'])/1e6:9.2f} pct={float(r['Percentage']):6.2f}")
PY
