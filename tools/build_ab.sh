#!/bin/bash
# Build liballl.so of a git revision (or the working tree: "wt") into build/ab/liballl_<name>.so
# for tools/ab_bench.sh.  usage: bash tools/build_ab.sh <name> <rev|wt>
set -e
cd "$(dirname "$0")/.."
NAME=$1; REV=$2
mkdir -p build/ab
if [ "$REV" = wt ]; then
  make -s && cp alllsatisfiabilitysolver_amd/liballl.so build/ab/liballl_$NAME.so
else
  D=$(mktemp -d /tmp/abwt.XXXX)
  git worktree add -q --detach $D $REV
  make -s -C $D && cp $D/alllsatisfiabilitysolver_amd/liballl.so build/ab/liballl_$NAME.so
  git worktree remove --force $D
fi
ls -la build/ab/liballl_$NAME.so
