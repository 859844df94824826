#!/usr/bin/env python3
"""Table of bench.py A/B logs: one row per log with the JSON line's median / mean ms per step,
how the inputs arrived (resident / in-step upload on the step's stream / upload overlapped on
a copy stream), whether the weight gradients ran on their own stream, whether per-launch
profiling events were on, and the box's HBM copy probe.
usage: scripts/ab_table.py <log> [<log> ...]   (a log's label = its path)"""
import json
import sys


def h2d_mode(cfg):
    if not cfg.get("h2d_in_step"):
        return "resident"
    return "inline" if "first on the step's stream" in cfg.get("inputs", "") else "overlap"


print(f"{'log':28s} {'med ms':>7s} {'mean ms':>8s} {'inputs':>9s} {'wgrad':>6s} {'prof':>5s} {'box GB/s':>9s}")
for path in sys.argv[1:]:
    d = None
    for line in open(path):
        if line.startswith("{") and '"metric"' in line:
            d = json.loads(line)
    if d is None:
        print(f"{path:28s} (no bench line)")
        continue
    c = d["config"]
    ws = d.get("wgrad_stream")
    print(f"{path:28s} {d['ms_per_step']:7.2f} {d.get('ms_per_step_mean') or 0:8.2f} {h2d_mode(c):>9s} "
          f"{'2 str' if ws else ('1 str' if ws is False else '-'):>6s} {'on' if d.get('roofline') else 'off':>5s} "
          f"{d.get('box', {}).get('copy_GBps') or 0:9.0f}")
