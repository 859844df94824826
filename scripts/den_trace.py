"""Phase timeline of the den forward kernel (sequence 0, block 0), frames 16..47."""
import os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kaldi-fp16_amd", "python"))
import numpy as np
import kfp16
from kfp16 import synth, chain
torch.cuda.set_device(0)
kfp16.check(kfp16.core.bridge_gpu_init(0))
kfp16.set_stream(torch.cuda.current_stream().cuda_stream)
kfp16.core.kf_chain_trace.argtypes = [kfp16._vp, kfp16._vp]
egs, P = int(sys.argv[1]) if len(sys.argv) > 1 else 64, 3080
T = egs * 1500
x = torch.from_numpy((np.random.default_rng(0).standard_normal((T, P)) * 2).astype(np.float16).view(np.int16)).cuda()
og = torch.zeros((T, P), dtype=torch.float16, device="cuda")
ch = chain.Chain(chain.DenGraph(synth.make_den_graph(num_pdfs=P)), egs, 490)
nb = chain.NumBatch([synth.make_num_fst(e) for e in range(egs)])
row0, nfr, stride = synth.chain_layout(egs)
tb = torch.zeros(32 * 8 + 32 * 2 * 16, dtype=torch.int64, device="cuda")
kfp16.core.kf_chain_trace(ch.h, tb.data_ptr())
for _ in range(3):
    ch.compute(nb, x.data_ptr(), P, T, row0, nfr, stride, og.data_ptr(), P)
torch.cuda.synchronize()
raw = tb.cpu().numpy().astype(np.float64) * 10e-3  # 100 MHz ticks -> us
a = raw[:256].reshape(32, 8)
w = raw[256:].reshape(32, 2, 16) - a[:, None, :1]  # per-wave arc end relative to the frame start
d = np.diff(a, axis=1)
names = ["arc", "publish", "prefetch", "wait", "psum", "consume", "tail+bar"]
cen = ch.debug_census()
print("G", cen["G"], "units", cen["units"], "XCD-local units", cen["local_fwd"], cen["local_bwd"], "egs", egs)
print("mean us per phase:", {n: round(float(v), 2) for n, v in zip(names, d[1:].mean(0))})
fr = np.diff(a[:, 0])
print("frame period us: mean %.2f min %.2f max %.2f" % (fr.mean(), fr.min(), fr.max()))
wend = w[1:].reshape(31, 32)
print("arc end per wave (us after frame start): mean over waves %.2f, slowest %.2f, wave 0 %.2f" %
      (wend.mean(), wend.max(1).mean(), w[1:, 0, 0].mean()))
print("per-(block,wave) mean arc end:", np.round(w[1:].mean(0), 2).tolist())
