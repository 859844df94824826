"""Times the batched chain objective (num || den fwd -> den bwd) for each G
(blocks per sequence) on the bench shape: 64 egs x 490 frames."""
import os, sys, time, subprocess
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "child":
    import torch
    sys.path.insert(0, os.path.join(ROOT, "kaldi-fp16_amd", "python"))
    import numpy as np
    import kfp16
    from kfp16 import synth, chain
    torch.cuda.set_device(0)
    kfp16.check(kfp16.core.bridge_gpu_init(0))
    kfp16.set_stream(torch.cuda.current_stream().cuda_stream)
    egs, P = 64, 3080
    T = egs * 1500
    x = torch.from_numpy((np.random.default_rng(0).standard_normal((T, P)) * 2).astype(np.float16).view(np.int16)).cuda()
    og = torch.zeros((T, P), dtype=torch.float16, device="cuda")
    ch = chain.Chain(chain.DenGraph(synth.make_den_graph(num_pdfs=P)), egs, 490)
    nb = chain.NumBatch([synth.make_num_fst(e) for e in range(egs)])
    row0, nfr, stride = synth.chain_layout(egs)
    for _ in range(2):
        ch.compute(nb, x.data_ptr(), P, T, row0, nfr, stride, og.data_ptr(), P)
    torch.cuda.synchronize()
    kfp16.core.kf_prof_reset(); kfp16.core.kf_prof_enable(1)
    t0 = time.perf_counter()
    for _ in range(5):
        ch.compute(nb, x.data_ptr(), P, T, row0, nfr, stride, og.data_ptr(), P)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
    kfp16.core.kf_prof_enable(0)
    _, nms, _ = kfp16.prof_collect(2)
    _, dms, _ = kfp16.prof_collect(3)
    r = ch.result()
    print(f"G={os.environ.get('KF_DEN_G')}: chain {dt*1e3:.2f} ms/call (num {nms/5:.2f}, den path {dms/5:.2f}) ok={r.num_ok}", flush=True)
else:
    for G in sys.argv[1:] or ["1", "2", "4"]:
        env = dict(os.environ, KF_DEN_G=G)
        subprocess.run([sys.executable, __file__, "child"], env=env, check=True, timeout=300)
