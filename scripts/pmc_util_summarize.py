"""Per kernel class from one rocprofv3 PMC pass (scripts/pmc_util.sh):
  mfma_busy   SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): the fraction
              of SIMD cycles the matrix cores were busy while the kernel ran (one
              v_mfma_f32_16x16x32_f16 = 16 busy cycles = 16,384 FLOP, so this is also the
              fraction of the dense fp16 peak at the clock the chip held);
  wait / issue_stall / active  SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over
              SQ_WAVE_CYCLES (disjoint, MI355X_MICROARCH.md §rocprofv3 PMC slots): waves
              parked on s_waitcnt / barriers, waves stalled at issue, waves issuing;
  lds_conflict SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles per LDS cycle);
  clock_GHz   GRBM_GUI_ACTIVE / 8 / kernel duration.
Counters are summed over launches of the class (per-dispatch rows of the CSV)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summarize import kclass  # noqa: E402

root = sys.argv[1]


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0][:120]


def collect(keyf):
    vals = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    dur = defaultdict(float)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = keyf(row.get("Kernel_Name", ""))
            vals[k][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[k].add(row.get("Dispatch_Id") or row.get("Correlation_Id"))
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = keyf(row.get("Kernel_Name", ""))
            dur[k] += (float(row["End_Timestamp"]) - float(row["Start_Timestamp"])) * 1e-9
    return vals, disp, dur


def summary(vals, disp, dur, raw=True):
    out = {}
    for k, v in sorted(vals.items(), key=lambda kv: -dur.get(kv[0], 0.0)):
        gui = v.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        wc = v.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        out[k] = {
            "launches": len(disp[k]),
            "kernel_s": dur.get(k),
            "mfma_busy": v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024.0 * gui) if gui else None,
            "wait": v.get("SQ_WAIT_ANY", 0.0) / wc,
            "issue_stall": v.get("SQ_WAIT_INST_ANY", 0.0) / wc,
            "active": v.get("SQ_ACTIVE_INST_ANY", 0.0) / wc,
            "lds_conflict": v.get("SQ_LDS_BANK_CONFLICT", 0.0) / (v.get("SQ_LDS_IDX_ACTIVE", 0.0) or 1.0),
            "clock_GHz": gui / dur[k] * 1e-9 if dur.get(k) else None,
        }
        if raw:
            out[k]["raw"] = dict(v)
    return out


by_class = summary(*collect(kclass))
by_kernel = summary(*collect(short), raw=False)
print(json.dumps({"by_class": by_class, "by_kernel": dict(list(by_kernel.items())[:25])}, indent=1))
