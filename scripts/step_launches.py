"""Per-launch times of one train step's GEMM / conv launches (kf_prof_records), in issue
order, on the bench model at 64 egs: forward, backward from a fixed output gradient, SGD.
Prints one line per launch (class, ms, TF/s, M N K, tile) and per-class sums.

  python scripts/step_launches.py [--xconfig X] [--egs 64] [--one-stream] [--steps 3]
"""
import argparse
import json
import os
import sys

import torch  # noqa: F401  (the HIP runtime first, as bench.py)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kaldi-fp16_amd", "python"))
import numpy as np  # noqa: E402
import kfp16  # noqa: E402
from kfp16 import synth  # noqa: E402

CLS = {0: "fused", 1: "wgrad", 2: "num", 3: "den", 4: "halo", 5: "cwgrad", 6: "reduce"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--xconfig", default="cnn_tdnn_17f.xconfig")
    p.add_argument("--egs", type=int, default=64)
    p.add_argument("--one-stream", action="store_true")
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--json", default="")
    p.add_argument("--variants", default="default",
                   help="comma list of labels run in turn in this process (same-box repeats)")
    p.add_argument("--quiet", action="store_true", help="per-class sums only")
    p.add_argument("--rsub", action="store_true", help="row-subsampled step (nnet_set_row_subsampling 3)")
    a = p.parse_args()
    kfp16.check(kfp16.core.bridge_gpu_init(0))
    T = a.egs * 1500
    net = kfp16.Network(synth.load_xconfig(a.xconfig), max_frames=T)
    synth.init_network(net, seed=42)
    if a.one_stream:
        net.set_wgrad_stream(False)
    fb = kfp16.upload_fp16(synth.make_features(T, 40))
    P = net.layers[-1][3]
    rows = T
    if a.rsub:
        net.set_row_subsampling(3)
        net.forward(fb.ptr, T)
        rows = net.row_set()[0] or T
    og = kfp16.upload_fp16((np.random.default_rng(11).standard_normal((rows, P)) * 0.01).astype(np.float16))
    kfp16.core.kf_prof_reserve(512)
    for v in a.variants.split(","):
        print(f"== variant {v}")
        run(a, net, fb, og, T)
    net.close()


def run(a, net, fb, og, T):
    recs = []
    for s in range(a.steps):
        last = s == a.steps - 1
        if last:
            kfp16.core.kf_prof_reset()
            kfp16.core.kf_prof_enable(1)
        net.forward(fb.ptr, T)
        net.backward(og.ptr)
        net.sgd(1e-9, 0.9)
        if last:
            torch.cuda.synchronize()
            kfp16.core.kf_prof_enable(0)
            recs = kfp16.prof_records()
    tot = {}
    for r in recs:
        name = CLS.get(r["cls"], str(r["cls"]))
        tf = r["flops"] / (r["ms"] * 1e-3) / 1e12 if r["ms"] > 0 else 0
        t = r["tile"]
        if not a.quiet:
            print(f"{name:7s} {r['ms'] * 1e3:9.1f} us {tf:7.1f} TF/s  M={r['M']:8d} N={r['N']:5d} K={r['K']:5d} "
                  f"tile={t // 10000}x{t % 10000}")
        c = tot.setdefault(name, [0, 0.0, 0.0])
        c[0] += 1
        c[1] += r["ms"]
        c[2] += r["flops"]
    for k, (n, ms, fl) in tot.items():
        print(f"# {k:7s} launches {n:3d}  {ms:8.3f} ms  {fl / (ms * 1e-3) / 1e12 if ms else 0:7.1f} TF/s")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(recs, fh)


if __name__ == "__main__":
    main()
