#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6j
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py --rccl-self --no-cpu-baseline --steps 20 --warmup 3 --event-iters 0 > $O/bench.json 2> $O/bench.err
rc=$?; echo "trace rc=$rc"; tail -2 $O/bench.err; [ $rc -ne 0 ] && exit $rc
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py $f 10 | tee $O/timeline.txt
