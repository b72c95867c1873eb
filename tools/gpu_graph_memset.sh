#!/bin/bash
# The graph-replay stall of DESIGN.md §10: tools/microbench/graph_memset under the runtime it
# was built with (ROCm 7.2) and under torch's bundled HIP runtime, with and without memset nodes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TL=$(python3 -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
mkdir -p /tmp/trt
ln -sf $TL/libamdhip64.so /tmp/trt/libamdhip64.so.7
ln -sf $TL/libhsa-runtime64.so /tmp/trt/libhsa-runtime64.so.1
B=tools/microbench/graph_memset
# (args: mode, replays, MiB per cleared buffer, bodies per graph copy)
for args in "memset 20 4 1" "kernels 20 4 1" "memset 30 20 16" "kernels 30 20 16"; do
  echo "== ROCm 7.2 runtime: $args"; timeout -k 5 60 $B $args; echo "rc=$?"
  echo "== torch's runtime: $args"; LD_LIBRARY_PATH=/tmp/trt:$TL timeout -k 5 60 $B $args; echo "rc=$?"
done
exit 0
