"""Per-step timeline of conv_halo_kernel (block 300, wave 0) for the benchmark network's
forward conv launches: python scripts/halo_trace.py [egs]. Stamps: kf_halo_trace."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kaldi-fp16_amd", "python"))
import kfp16  # noqa: E402
from kfp16 import synth  # noqa: E402

torch.cuda.set_device(0)
kfp16.check(kfp16.core.bridge_gpu_init(0))
kfp16.set_stream(torch.cuda.current_stream().cuda_stream)
kfp16.core.kf_halo_trace.argtypes = [kfp16._vp, kfp16._i]
egs = int(sys.argv[1]) if len(sys.argv) > 1 else 64
T = egs * 1500
net = kfp16.Network(synth.load_xconfig("cnn_tdnn_17f.xconfig"), max_frames=T)
synth.init_network(net)
feats = kfp16.upload_fp16(synth.make_features(T, 40))
tb = torch.zeros(128, dtype=torch.int64, device="cuda")
for at in range(5):
    tb.zero_()
    kfp16.core.kf_halo_trace(tb.data_ptr(), at)
    net.forward(feats.ptr, T)
    torch.cuda.synchronize()
    a = tb.cpu().numpy().astype(np.float64) * 10e-3  # us
    kfp16.core.kf_halo_trace(None, -1)
    if a[0] == 0:
        print(at, "no stamps")
        continue
    steps = [i for i in range(63) if a[1 + 2 * i] > 0]
    w = [a[1 + 2 * s] - (a[2 + 2 * (s - 1)] if s else a[0]) for s in steps]
    c = [a[2 + 2 * s] - a[1 + 2 * s] for s in steps]
    print(f"launch {at}: {len(steps)} steps, total {a[127] - a[0]:.2f} us, first wait {w[0]:.2f}, "
          f"wait/step {np.mean(w[1:]):.3f} (max {np.max(w[1:]):.2f}), mfma/step {np.mean(c):.3f}, "
          f"epilogue {a[127] - a[126]:.2f}")
    print("   waits:", " ".join(f"{x:.2f}" for x in w))
