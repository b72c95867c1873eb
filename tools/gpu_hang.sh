#!/bin/bash
# the round-robin stall under torch's bundled HIP runtime, with the runtime's API log (see tools/rr_hang.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/hang3
mkdir -p $O
AMD_LOG_LEVEL=3 timeout -k 10 70 python tools/rr_hang.py --torch 2>&1 | tail -c 3000000 > $O/b.log
rc=$?; echo "torch first, logged rc=$rc"; grep -v "^:3:" $O/b.log | tail -12; tail -c 4000 $O/b.log; exit $rc
