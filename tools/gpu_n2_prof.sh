#!/bin/bash
# Kernel trace of the 2-rank path on one GPU (host-staged exchange; kernel durations are
# representative, the exchange is not): two bench.py ranks, each under its own rocprofv3.
# usage: VARIANTS="A B" bash tools/gpu_n2_prof.sh   (ALLL_LIB_AB builds in build/ab/, or "cur")
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 WORLD_SIZE=2 ALLL_BENCH_SAME_DEVICE=1
mkdir -p gpurun_out
port=29541
for v in ${VARIANTS:-cur}; do
  lib=""; [ "$v" != cur ] && lib=build/ab/liballl_$v.so
  rm -rf gpurun_out/n2_${v}_*
  for r in 0 1; do
    ALLL_LIB_AB=$lib MASTER_PORT=$port RANK=$r LOCAL_RANK=$r timeout -k 10 300 rocprofv3 --kernel-trace \
      --output-format csv -d gpurun_out/n2_${v}_$r -o run -- python3 bench.py --gpus 2 --steps 10 --warmup 2 \
      --no-cpu-baseline --event-iters 0 ${CONFIG:+--config $CONFIG} > gpurun_out/n2_${v}_$r.json 2> gpurun_out/n2_${v}_$r.err &
  done
  wait || exit 1
  port=$((port + 1))
  python3 - "$v" <<'PY'
import csv, glob, sys
from collections import defaultdict
v = sys.argv[1]
for r in (0, 1):
    f = glob.glob(f"gpurun_out/n2_{v}_{r}/**/*kernel_trace.csv", recursive=True)
    if not f:
        print(v, r, "no trace"); continue
    d = defaultdict(list)
    for row in csv.DictReader(open(f[0])):
        d[row["Kernel_Name"].split("(")[0].replace("void alll::", "").replace("alll::", "")].append(
            (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1000)
    print(v, "rank", r, " ".join(f"{k} {sum(x)/len(x):.1f}" for k, x in sorted(d.items()) if k.startswith("k_")))
PY
done
