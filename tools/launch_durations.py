"""Per-launch durations of one kernel, in launch order, from a rocprofv3 kernel trace CSV: which
launch is the slow one (the first iteration, an eager replay, a stamp-wrap reduce ...).
usage: python tools/launch_durations.py <run_kernel_trace.csv> <kernel-name-prefix> [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
name, top = sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 8
evals = 0
seq = []
for r in rows:
    k = r["Kernel_Name"].split("(")[0].replace("void alll::", "").replace("alll::", "")
    if k.startswith("k_eval"):
        evals += 1
    if k.startswith(name):
        seq.append((evals, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0))
d = [x for _, x in seq]
if not d:
    sys.exit(f"no launches of {name}")
print(f"{name}: {len(d)} launches, mean {sum(d) / len(d):.2f} us, median {sorted(d)[len(d) // 2]:.2f} us")
for ev, x in sorted(seq, key=lambda t: -t[1])[:top]:
    print(f"   {x:8.2f} us  after evaluation #{ev}")
