"""Gradient sensitivity of the 17f + attention model to fp16 rounding: GPU vs the
oracle in F (fused rounding) and NONE (fp32 throughout) modes, all with the GPU's ReLU
decisions replayed. Prints rel-Frobenius errors for the named parameters.
Usage: python scripts/att_precision.py [xconfig] [T]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "kaldi-fp16_amd", "python")]
import torch  # noqa: F401,E402  (bind torch's HIP runtime first)
import kfp16 as kf  # noqa: E402
import oracle  # noqa: E402
from conftest import rel_fro  # noqa: E402
from kfp16 import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cnn_tdnn_17f_att.xconfig"
T = int(sys.argv[2]) if len(sys.argv) > 2 else 240
kf.core.bridge_gpu_init(0)
xcfg = synth.load_xconfig(cfg)
net = kf.Network(xcfg, max_frames=T)
params, bns = synth.init_network(net)
feats = synth.make_features(T, 40)
fb = kf.upload_fp16(feats)
net.forward(fb.ptr, T)
masks = net.relu_masks()
P = [d for n, _, _, d in net.layers if n == "output"][0]
og = (np.random.default_rng(7).standard_normal((T, P)) * 0.05).astype(np.float16)
gb = kf.upload_fp16(og)
net.backward(gb.ptr)
got = net.read_grads()
tp = {k: synth.trunc_fp16(v) for k, v in params.items()}
ref = {}
for mode, name in ((oracle.ROUND_FUSED, "F"), (oracle.ROUND_NONE, "NONE")):
    on = oracle.OracleNet(xcfg, tp, bns, round_mode=mode, threads=16)
    on.forward(feats.astype(np.float32), force_masks=masks)
    on.backward(og.astype(np.float32))
    ref[name] = on.grads()
    on.close()
keys = [k for k in ref["F"] if k.split(".")[0] in ("attention24", "attention3", "tdnnf23", "tdnnf8", "cnn1",
                                                     "prefinal-l", "tdnnf4", "tdnnf2")]
for k in keys:
    print(f"{k:28s} gpu-F {rel_fro(got[k], ref['F'][k]):.2e}  gpu-NONE {rel_fro(got[k], ref['NONE'][k]):.2e}  "
          f"F-NONE {rel_fro(ref['F'][k], ref['NONE'][k]):.2e}", flush=True)
