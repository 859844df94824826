#!/usr/bin/env python3
"""Per-kernel median / mean duration (us) from rocprofv3 kernel traces.
usage: scripts/kmed.py <pattern> <run dir> [<run dir> ...]   (run dir holds run_kernel_trace.csv)"""
import csv
import re
import sys

import numpy as np

pat = re.compile(sys.argv[1])
for d in sys.argv[2:]:
    rows = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
    by = {}
    for r in rows:
        if pat.search(r["Kernel_Name"]):
            by.setdefault(r["Kernel_Name"][:60], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(d, " | ".join(f"{k[:40]} n={len(v)} med={np.median(v):.1f} mean={np.mean(v):.1f}" for k, v in sorted(by.items())))
