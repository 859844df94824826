"""Print one training step's kernel sequence from a rocprofv3 kernel trace.

usage: python scripts/step_trace.py <run_kernel_trace.csv | run_results.db> [step_index_from_end]
Steps are delimited by k_sgd_flat (the last kernel of a step).
"""
import csv
import re
import sys

if sys.argv[1].endswith(".db"):  # rocprofv3's default rocpd (SQLite) output
    import sqlite3
    cur = sqlite3.connect(sys.argv[1]).execute(
        "select start, end, name, queue_id, grid_x, grid_y, workgroup_x, vgpr_count, accum_vgpr_count from kernels")
    keys = ["Start_Timestamp", "End_Timestamp", "Kernel_Name", "Queue_Id", "Grid_Size_X", "Grid_Size_Y",
            "Workgroup_Size_X", "VGPR_Count", "Accum_VGPR_Count"]
    rows = [dict(zip(keys, map(str, r))) for r in cur]
else:
    rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "k_sgd_flat" in r["Kernel_Name"]]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 1
lo = ends[-back - 1] + 1 if len(ends) > back else 0
hi = ends[-back]
seg = rows[lo:hi + 1]
t0 = int(seg[0]["Start_Timestamp"])
tot = 0.0
groups = {}
for r in seg:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    name = r["Kernel_Name"]
    m = re.match(r"void (\w+)<([^>]*)>", name)
    short = (m.group(1) + "<" + m.group(2) + ">") if m else re.sub(r"\(.*", "", name)[:60]
    groups[short] = groups.get(short, 0) + d
    grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) // int(r["Workgroup_Size_X"])
    print(f"{(int(r['Start_Timestamp'])-t0)/1e3:9.1f} {d:8.1f}us  q{r['Queue_Id']} wg={grid:6d} vgpr={r['VGPR_Count']:>3}+{r['Accum_VGPR_Count']:>3} {short}")
wall = (int(seg[-1]["End_Timestamp"]) - t0) / 1e3
print(f"kernels {len(seg)}  sum {tot/1e3:.2f} ms  wall {wall/1e3:.2f} ms")
for k, v in sorted(groups.items(), key=lambda x: -x[1])[:25]:
    print(f"{v/1e3:8.2f} ms  {k}")
