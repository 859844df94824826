"""Times the den forward kernel variants (benchmarking only): 0 product,
1 conflict-free LDS reads, 2 no global arc loads."""
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
kfp16.core.kf_chain_debug_variant.argtypes = [kfp16._i]
egs, P = 64, 3080
T = egs * 1500
x = torch.from_numpy((np.random.default_rng(0).standard_normal((T, P)) * 2).astype(np.float16).view(np.int16)).cuda()
og = torch.zeros((T, P), dtype=torch.float16, device="cuda")
g = synth.make_den_graph(num_pdfs=P)
ch = chain.Chain(chain.DenGraph(g), egs, 490)
nb = chain.NumBatch([synth.make_num_fst(e) for e in range(egs)])
row0, nfr, stride = synth.chain_layout(egs)
for v in (0, 1, 2):
    kfp16.core.kf_chain_debug_variant(v)
    for _ in range(2):
        ch.compute(nb, x.data_ptr(), P, T, row0, nfr, stride, og.data_ptr(), P)
    torch.cuda.synchronize()
    kfp16.core.kf_prof_reset(); kfp16.core.kf_prof_enable(1)
    t0 = time.perf_counter()
    for _ in range(3):
        ch.compute(nb, x.data_ptr(), P, T, row0, nfr, stride, og.data_ptr(), P)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 3
    kfp16.core.kf_prof_enable(0)
    n, ms, _ = kfp16.prof_collect(3)
    print(f"variant {v}: chain {dt*1e3:.2f} ms/call, den bracket {ms/3:.2f} ms", flush=True)
kfp16.core.kf_chain_debug_variant(0)
