"""Summarise rocprofv3 kernel_stats CSVs: per-kernel ms per step, side by side.
usage: python scripts/kstats.py STEPS a.csv [b.csv ...]"""
import csv
import sys

steps = float(sys.argv[1])
tabs = []
for f in sys.argv[2:]:
    t = {}
    for r in csv.DictReader(open(f)):
        t[r["Name"]] = (float(r["TotalDurationNs"]) / 1e6 / steps, int(r["Calls"]) / steps, float(r["AverageNs"]) / 1e3)
    tabs.append(t)
names = sorted(set().union(*tabs), key=lambda n: -max(t.get(n, (0,))[0] for t in tabs))
for n in names[:45]:
    cells = "".join(f"{t[n][0]:8.3f} ms {t[n][2]:8.1f}us x{t[n][1]:5.1f} |" if n in t else " " * 32 + "|" for t in tabs)
    print(cells, n[:110])
print("total ms/step:", " ".join(f"{sum(v[0] for v in t.values()):.2f}" for t in tabs))
