"""Tile timeline of gemm_kernel launches in the benchmark network's forward + backward
(kf_gemm_trace): per launch the shape, the tile duration distribution, how many tiles a CU
runs at once, and block `blk`'s phase stamps (K-step waits, epilogue).
usage: python scripts/gemm_trace.py [launch ids, default 0-7] [--egs 64] [--blk 3000]"""
import argparse
import os
import sys
from collections import defaultdict

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kaldi-fp16_amd", "python"))
import kfp16  # noqa: E402
from kfp16 import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("ids", nargs="*", type=int)
ap.add_argument("--egs", type=int, default=64)
ap.add_argument("--blk", type=int, default=3000)
args = ap.parse_args()
ids = args.ids or list(range(8))

torch.cuda.set_device(0)
kfp16.check(kfp16.core.bridge_gpu_init(0))
kfp16.set_stream(torch.cuda.current_stream().cuda_stream)
T = args.egs * 1500
net = kfp16.Network(synth.load_xconfig("cnn_tdnn_17f.xconfig"), max_frames=T)
synth.init_network(net)
feats = kfp16.upload_fp16(synth.make_features(T, 40))
og = kfp16.upload_fp16((np.random.default_rng(1).standard_normal((T, 3080)) * 1e-3).astype(np.float16))
NW = 64 + 3 * 40000
tb = torch.zeros(NW, dtype=torch.int64, device="cuda")


def step():
    net.forward(feats.ptr, T)
    net.backward(og.ptr)


step()
torch.cuda.synchronize()
for at in ids:
    tb.zero_()
    kfp16.core.kf_gemm_trace(tb.data_ptr(), at, args.blk)
    step()
    torch.cuda.synchronize()
    kfp16.core.kf_gemm_trace(None, -1, 0)
    a = tb.cpu().numpy().astype(np.uint64)
    if a[60] == 0 and a[61] == 0:
        print(f"launch {at}: not reached")
        continue
    M, N, K = int(a[60] & 0xFFFFF), int((a[60] >> 20) & 0xFFFFF), int(a[60] >> 40)
    BM, BN, gx, gy = int(a[61] & 0xFFFF), int((a[61] >> 16) & 0xFFFF), int(a[61] >> 32), int(a[62])
    nb = gx * gy
    rec = a[64:64 + 3 * nb].reshape(nb, 3)
    st = rec[:, 0].astype(np.float64) * 0.01
    en = rec[:, 1].astype(np.float64) * 0.01
    ok = (rec[:, 0] > 0) & (rec[:, 1] > 0)
    t0 = st[ok].min()
    dur = (en - st)[ok]
    hw = rec[:, 2]
    # CU key: xcc, se, sh, cu of HW_ID (gfx9 layout: cu 11:8, sh 12, se 15:13)
    cu = ((hw >> np.uint64(32)) << np.uint64(8)) | ((hw >> np.uint64(8)) & np.uint64(0xFF))
    span = en[ok].max() - t0
    # average tiles in flight per CU over the launch
    bycu = defaultdict(float)
    for c, d in zip(cu[ok], dur):
        bycu[int(c)] += d
    ncu = len(bycu)
    conc = np.mean([v / span for v in bycu.values()])
    print(f"launch {at}: M={M} N={N} K={K} tile {BM}x{BN} grid {gx}x{gy}: span {span:.1f} us, {ncu} CUs, "
          f"tile us mean {dur.mean():.2f} p10 {np.percentile(dur, 10):.2f} p90 {np.percentile(dur, 90):.2f}, "
          f"tiles in flight per CU {conc:.2f}, first start spread {np.percentile(st[ok] - t0, 99):.1f} us")
    p = a[:64].astype(np.float64) * 0.01
    if p[0] > 0:
        ks = [i for i in range(40) if a[2 + i] > 0]
        prev = p[1]
        waits = []
        for i in ks:
            waits.append(p[2 + i] - prev)
            prev = p[2 + i]
        epi = p[43] - p[42] if a[42] > 0 else float("nan")
        loop_end = p[42] if a[42] > 0 else p[43]
        print(f"   block {args.blk}: prologue {p[1] - p[0]:.2f}, K-step intervals "
              + " ".join(f"{w:.2f}" for w in waits)
              + f", last step {loop_end - p[2 + ks[-1]]:.2f}, epilogue {epi:.2f}, total {p[43] - p[0]:.2f} us")
