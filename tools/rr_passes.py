"""Per-pass kernel durations of the last traced round-robin iteration (rocprofv3 kernel trace).
usage: python tools/rr_passes.py <trace dir>"""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
seq = [(r["Kernel_Name"].split("(")[0].replace("void ", "").replace("alll::", ""),
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, int(r["Start_Timestamp"])) for r in rows]
starts = [i for i, s in enumerate(seq) if s[0].startswith("k_eval")]
i0 = starts[-1]
line, tot, t_first = [], 0.0, seq[i0][2]
for n, d, t in seq[i0:]:
    if (n.startswith("k_fp_vmin") or n.startswith("k_fp_detect")) and line:
        print(f"{tot:7.1f} | " + " ".join(line))
        line, tot = [], 0.0
    line.append(f"{n.replace('k_fp_', '').replace('<4u>', '')}:{d:.1f}")
    tot += d
print(f"{tot:7.1f} | " + " ".join(line))
print(f"iteration wall (first eval start to last kernel end): {(seq[-1][2] - t_first) / 1e3:.1f} us")
