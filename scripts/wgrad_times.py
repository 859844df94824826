"""Per-launch durations of one kernel family from a rocprofv3 kernel trace (one step).
usage: python scripts/wgrad_times.py trace.csv substring [launches_per_step] [skip_steps]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
sel = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if sys.argv[2] in r["Kernel_Name"]]
per = int(sys.argv[3]) if len(sys.argv) > 3 else 5
skip = int(sys.argv[4]) if len(sys.argv) > 4 else 2
steps = [sel[i:i + per] for i in range(skip * per, len(sel) - per + 1, per)][:5]
for s in steps:
    print(" ".join(f"{d:8.1f}" for d in s), f"| {sum(s):8.1f}")
