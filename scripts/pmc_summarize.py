"""Summarise the two PMC passes of scripts/pmc_traffic.sh into HBM bytes per
launch for each kernel class (gemm_fused, gemm_wgrad, chain kernels, ...).
FETCH_SIZE / WRITE_SIZE are KiB; FETCH_SIZE is doubled (gfx950 reports half of a
wide coalesced read, MI355X_MICROARCH.md §HBM)."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def kclass(name):
    m = re.search(r"gemm_kernel<([^>]*)>", name)
    if m:
        args = [a.strip() for a in m.group(1).split(",")]
        return "gemm_wgrad" if len(args) > 6 and args[6] == "true" else "gemm_fused"
    if "conv_wgrad_halo_kernel" in name:  # conv weight gradients (kf_prof class 1)
        return "gemm_wgrad"
    if "conv_halo_kernel" in name or "panel_kernel" in name:  # fused GEMMs too (kf_prof class 0)
        return "gemm_fused"
    for k in ("k_den_fb", "k_den_fwd", "k_den_bwd", "k_den_post", "k_num_fb", "k_conv_c1_wgrad", "k_conv_c1_fwd",
              "k_slab_reduce", "k_sgd_flat"):
        if k in name:
            return k
    return "other"


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                per[kclass(row.get("Kernel_Name", ""))].append(float(row["Counter_Value"]))
    return per


def main():
    root = sys.argv[1]
    fetch = load(os.path.join(root, "fetch"), "FETCH_SIZE")
    write = load(os.path.join(root, "write"), "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        n = max(len(f), len(w))
        if not n:
            continue
        fb = 2.0 * 1024 * sum(f) / max(len(f), 1)
        wb = 1024.0 * sum(w) / max(len(w), 1)
        out[k] = {"launches": n, "read_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                  "hbm_bytes_per_launch": fb + wb}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
