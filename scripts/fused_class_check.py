"""Fused-class (gemm_kernel with WGRAD false + conv_halo_kernel) average launch duration
over the headline's timed steps, from a rocprofv3 kernel trace of the default
`python3 bench.py` command, for comparison with the bench line's roofline timing.
usage: python3 scripts/fused_class_check.py <run_kernel_trace.csv> <bench log> [warmup] [steps]"""
import csv
import json
import sys

trace, log = sys.argv[1], sys.argv[2]
warm = int(sys.argv[3]) if len(sys.argv) > 3 else 3
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
line = next(json.loads(l) for l in open(log) if l.startswith('{"metric"'))
per_step = line["roofline"]["launches"] // line["steps"]
rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))


def fused(n):
    return ("gemm_kernel<" in n and n.split("<")[1].split(",")[6].strip() == "false") or "conv_halo_kernel<" in n


d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if fused(r["Kernel_Name"])]
skip = line["roofline"].get("priming_launches", 0) + warm * per_step
timed = d[skip:skip + steps * per_step]
bench_us = line["roofline"]["kernel_ms_per_step"] * 1e3 / per_step
print(json.dumps({"launches_timed": len(timed), "rocprof_avg_us": round(sum(timed) / len(timed), 1),
                  "bench_hip_event_avg_us": round(bench_us, 1),
                  "rocprof_class_ms_per_step": round(sum(timed) / 1e3 / steps, 3),
                  "bench_class_ms_per_step": line["roofline"]["kernel_ms_per_step"]}))
