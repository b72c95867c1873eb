#!/bin/bash
# C5 A/B of build/ab/liballl_{A,B,C}.so (bench lines, no CPU baseline / round-robin line)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
VARIANTS="A B C" bash tools/ab_bench.sh 2 --config C5 --no-rr-line --event-iters 0
