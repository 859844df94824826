"""Debug: network output statistics and per-sequence chain objective on the bench setup."""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kaldi-fp16_amd", "python"))
import numpy as np
import kfp16
from kfp16 import synth, chain

egs = int(sys.argv[1]) if len(sys.argv) > 1 else 4
torch.cuda.set_device(0)
kfp16.check(kfp16.core.bridge_gpu_init(0))
kfp16.set_stream(torch.cuda.current_stream().cuda_stream)
T = egs * 1500
net = kfp16.Network(synth.load_xconfig("cnn_tdnn_17f.xconfig"), max_frames=T)
synth.init_network(net, seed=42)
feats = synth.make_features(T, 40)
fbuf = kfp16.upload_fp16(feats)
net.forward(fbuf.ptr, T)
P = net.layers[-1][3]
out = net.read_activation("output").astype(np.float32)
print("output", out.shape, "finite", np.isfinite(out).mean(), "absmax", np.nanmax(np.abs(out)), "mean", np.nanmean(out), "std", np.nanstd(out))
for name, ty, din, dout in net.layers:
    a = net.read_activation(name).astype(np.float32)
    print(f"{name:18s} finite={np.isfinite(a).mean():.4f} absmax={np.nanmax(np.abs(a)):.3g} std={np.nanstd(a):.3g}")
g = synth.make_den_graph(num_pdfs=P)
dg = chain.DenGraph(g)
nb = chain.NumBatch([synth.make_num_fst(e, num_pdfs=P) for e in range(egs)])
row0, nfr, stride = synth.chain_layout(egs)
ch = chain.Chain(dg, egs, 490)
og = kfp16.DeviceBuffer(T * P * 2)
ptr = net.activation("output")[0]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
lr = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-6
for it in range(steps):
    if it:
        net.forward(fbuf.ptr, T)
    ch.compute(nb, ptr, P, T, row0, nfr, stride, og.ptr, P)
    r = ch.result()
    print(it, "result", {k: round(getattr(r, k), 3) for k, _ in r._fields_})
    if it == 0:
        print(ch.seq_stats(egs)[:4])
    g = kfp16.read_fp16(og.ptr, (T, P)).astype(np.float32)
    print("   out_grad finite", np.isfinite(g).mean(), "absmax", np.abs(g).max(), "nnz rows", int((np.abs(g).sum(1) > 0).sum()))
    net.backward(og.ptr)
    grads = net.read_grads()
    print("   grad norms", {k: float(np.linalg.norm(v)) for k, v in list(grads.items())[:3]}, "max", max(float(np.abs(v).max()) for v in grads.values()),
          "finite", all(np.isfinite(v).all() for v in grads.values()))
    net.sgd(lr, 0.9)
