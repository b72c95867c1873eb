"""Print the kernel timeline of one loop iteration from a rocprofv3 kernel trace CSV.
usage: python tools/timeline.py <run_kernel_trace.csv> [iteration index]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
it = int(sys.argv[2]) if len(sys.argv) > 2 else 15
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
seq = [(r["Kernel_Name"].split("(")[0].replace("void alll::", "").replace("alll::", ""),
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000, int(r["Start_Timestamp"])) for r in rows]
evals = [i for i, s in enumerate(seq) if s[0].startswith("k_eval")]
i, j = evals[it], evals[it + 1]
t0 = seq[i][2]
for s in seq[i:j + 1]:
    print(f"{s[0]:22s} {s[1]:8.2f}us  start+{(s[2] - t0) / 1000:8.2f}")
