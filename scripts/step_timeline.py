#!/usr/bin/env python3
"""Per-stream view of one training step from a rocprofv3 kernel trace: for the last step
(from the last k_den_fb backwards to the previous one), per stream the busy time (union
of its kernels), and per phase (forward / chain / backward) the wall time and the busy
time of each stream. usage: scripts/step_timeline.py <run_kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Stream_Id"]), r["Kernel_Name"])
             for r in rows), key=lambda k: k[0])
den = [i for i, k in enumerate(ks) if "k_den_fb" in k[3]]
if len(den) < 2:
    sys.exit("need two steps")
# a step: from the kernel after the previous step's SGD to this step's SGD (k_sgd_flat)
sgd = [i for i, k in enumerate(ks) if "k_sgd" in k[3]]
s1 = max(i for i in sgd if i < den[-1])
s2 = min(i for i in sgd if i > den[-1])
step = ks[s1 + 1:s2 + 1]
t0, t1 = step[0][0], max(k[1] for k in step)
print(f"step wall {(t1 - t0) / 1e6:.3f} ms, {len(step)} kernels")


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


d = [k for k in step if "k_den_fb" in k[3]][0]
dp = [k for k in step if "k_den_post" in k[3]][0]
phases = [("forward", t0, d[0]), ("den", d[0], dp[1]), ("backward", dp[1], t1)]
streams = sorted({k[2] for k in step})
for name, a, b in phases:
    ins = [k for k in step if k[0] >= a and k[0] < b]
    line = f"{name:9s} wall {(b - a) / 1e6:7.3f} ms  all-streams busy {union([(k[0], min(k[1], b)) for k in ins]) / 1e6:7.3f}"
    for s in streams:
        iv = [(k[0], min(k[1], b)) for k in ins if k[2] == s]
        if iv:
            line += f"  s{s}: {len(iv)} k {union(iv) / 1e6:.3f} ms"
    print(line)
# top kernels of the backward by stream
bw = [k for k in step if k[0] >= dp[1]]
agg = defaultdict(lambda: [0, 0.0])
for k in bw:
    a = agg[(k[2], k[3][:70])]
    a[0] += 1
    a[1] += (k[1] - k[0]) / 1e3
for (s, n), (c, us) in sorted(agg.items(), key=lambda x: -x[1][1])[:16]:
    print(f"  s{s} {c:3d} x {us / c:7.1f} us = {us / 1e3:6.2f} ms  {n}")
