"""Per-parameter gradient errors of the full-width attention network (tests/test_gpu_attention.py
case cnn_tdnn_17f_att, T=240): GPU vs the fp16-emulating oracle, GPU vs fp32, oracle F vs fp32.
Usage (GPU box): python scripts/att_diag.py [xconfig] [T]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "kaldi-fp16_amd", "python"),
                 os.path.join(ROOT, "oracle"), ROOT]

from conftest import rel_fro  # noqa: E402
import oracle  # noqa: E402
from test_gpu_nnet import _forward_parity, _oracle  # noqa: E402
from kfp16 import synth  # noqa: E402
import kfp16 as kf  # noqa: E402

assert kf.core.bridge_gpu_init(0) == 0

cfg = sys.argv[1] if len(sys.argv) > 1 else "cnn_tdnn_17f_att.xconfig"
T = int(sys.argv[2]) if len(sys.argv) > 2 else 240
xcfg = synth.load_xconfig(cfg)
net = kf.Network(xcfg, max_frames=T)
params, bns = synth.init_network(net)
feats = synth.make_features(T, 40)
fbuf = kf.upload_fp16(feats)
net.forward(fbuf.ptr, T)
on = _oracle(xcfg, params, bns, feats)
masks = _forward_parity(net, on, None)
on.close()
P = [dout for name, ty, din, dout in net.layers if name == "output"][0]
seeds = [int(x) for x in os.environ.get("ATT_SEEDS", "7").split(",")]
for seed in seeds:
    og = (np.random.default_rng(seed).standard_normal((T, P)) * 0.05).astype(np.float16)
    gbuf = kf.upload_fp16(og)
    net.forward(fbuf.ptr, T)
    net.backward(gbuf.ptr)
    got = net.read_grads()
    res = {}
    for nm, mode in (("F", oracle.ROUND_FUSED), ("REF", oracle.ROUND_REF), ("f32", oracle.ROUND_NONE)):
        on = _oracle(xcfg, params, bns, feats, mode=mode)
        on.forward(feats.astype(np.float32), force_masks=masks)
        on.backward(og.astype(np.float32))
        res[nm] = on.grads()
        on.close()
    ref, rr, f32 = res["F"], res["REF"], res["f32"]
    print(f"seed {seed}")
    print(f"{'param':28s} {'gpu-F':>9s} {'gpu-f32':>9s} {'F-f32':>9s} {'REF-f32':>9s} ratioF ratioREF")
    lf, lr = [], []
    for k in ref:
        a, b, c, d = rel_fro(got[k], ref[k]), rel_fro(got[k], f32[k]), rel_fro(ref[k], f32[k]), rel_fro(rr[k], f32[k])
        if c > 0 and d > 0:
            lf.append(np.log(b / c))
            lr.append(np.log(b / d))
        if os.environ.get("ATT_VERBOSE", "1") == "1":
            print(f"{k:28s} {a:9.2e} {b:9.2e} {c:9.2e} {d:9.2e} {b / max(c, 1e-30):5.2f} {b / max(d, 1e-30):5.2f}")
    print(f"seed {seed}: geomean ratio vs F {np.exp(np.mean(lf)):.3f} (max {np.exp(np.max(lf)):.3f}), "
          f"vs REF {np.exp(np.mean(lr)):.3f} (max {np.exp(np.max(lr)):.3f})")
