#!/bin/bash
# The clause-sharded exchange path: multi-rank GPU tests (host exchange), then the one-rank RCCL
# bench line and its kernel trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/xchg
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "multirank or world or shard or rccl" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --rccl-self --no-cpu-baseline --steps 20 --warmup 3 > $O/bench_rccl_self.json 2> $O/bench_rccl_self.err
rc=$?; echo "rccl-self rc=$rc"; [ $rc -ne 0 ] && exit $rc
python -c "import json; d=json.load(open('$O/bench_rccl_self.json')); print(d['resample_iters_per_s'], d['phase_ms'], d['trajectory_check'])"
exit 0
