#!/bin/bash
# Kernel trace of the multi-GPU exchange path over a one-rank RCCL communicator (M).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/trace_rccl_self
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py --rccl-self --no-cpu-baseline --steps 20 --warmup 3 --event-iters 0 > $O/bench.json 2> $O/bench.err
rc=$?; echo "trace rc=$rc"
python3 -c "
import csv,glob
f=glob.glob('$O/trace/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)): print(r['Name'][:70], r['Calls'], r['AverageNs'])
"
exit $rc
