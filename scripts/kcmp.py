#!/usr/bin/env python3
"""Compare rocprofv3 kernel stats of two runs: per-kernel average us and total ms per step.
usage: scripts/kcmp.py <stats A.csv> <stats B.csv> [steps]"""
import csv, sys
def load(p):
    return {r["Name"]: (int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6)
            for r in csv.DictReader(open(p))}
a, b = load(sys.argv[1]), load(sys.argv[2])
steps = float(sys.argv[3]) if len(sys.argv) > 3 else 7.0
rows = []
for k in set(a) | set(b):
    ca, ua, ta = a.get(k, (0, 0, 0)); cb, ub, tb = b.get(k, (0, 0, 0))
    rows.append((tb - ta, k, ca, ua, ta, cb, ub, tb))
rows.sort(key=lambda r: -abs(r[0]))
print(f"{'delta ms':>9} {'A us':>8} {'B us':>8} {'A ms':>8} {'B ms':>8} calls  kernel")
for d, k, ca, ua, ta, cb, ub, tb in rows[:30]:
    print(f"{d:9.2f} {ua:8.1f} {ub:8.1f} {ta:8.2f} {tb:8.2f} {ca:4d}/{cb:<4d} {k[:110]}")
print("total ms A %.2f B %.2f" % (sum(v[2] for v in a.values()), sum(v[2] for v in b.values())))
