#!/bin/bash
# Round robin on the power-law instance (C5): throughput at T = 16 and 4 with up to 64 passes per
# iteration, and the kernel stats of one iteration.  usage: bash tools/gpu_rr_c5.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-c5}
mkdir -p gpurun_out/$TAG
ALLL_RR_FP_MAX=${FPMAX:-64} timeout -k 10 300 python -u tools/rr_bench.py --config C5 --threads 16,4 --iters 3 --warmup 1 || exit $?
ALLL_RR_FP_MAX=${FPMAX:-64} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/trace -o run -- \
    python3 tools/rr_bench.py --config C5 --threads 16 --iters 1 --warmup 0 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/err.log || exit $?
f=$(find gpurun_out/$TAG/trace -name '*kernel_stats.csv' | head -1)
python3 - "$f" << 'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:12]:
    print(f"{r['Name'][:50]:50s} calls={int(r['Calls']):6d} avg_us={float(r['AverageNs'])/1e3:9.1f} total_ms={float(r['TotalDurationNs'])/1e6:8.2f}")
PY
