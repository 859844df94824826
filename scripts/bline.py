#!/usr/bin/env python3
"""One-line summary of a bench.py log's JSON line: median / mean ms per step, frames/s,
the box's HBM probe. usage: scripts/bline.py <log>"""
import json
import sys

for line in open(sys.argv[1]):
    line = line.strip()
    if line.startswith("{") and '"metric"' in line:
        d = json.loads(line)
        print(f"med {d['ms_per_step']} mean {d.get('ms_per_step_mean')} value {d['value']:.0f} "
              f"box {d.get('box', {}).get('copy_GBps')} GB/s wgrad_stream {d.get('wgrad_stream')} steps {d.get('step_ms')} issue {d.get('cpu_issue_ms')}")
