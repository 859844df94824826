"""Phase timestamps of the row-panel GEMM (kf_rowpanel_trace): one block's wait / MFMA /
epilogue per 64-column block, on the TDNN-F affine forward at T = 96,000 (full epilogue)
and the linear input gradient. Also the launch time (kf_prof HIP events)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kaldi-fp16_amd", "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import kfp16 as kf  # noqa: E402

kf.check(kf.core.bridge_gpu_init(0))
kf.core.kf_rowpanel_trace.argtypes = [C.c_void_p]
kf.core.kf_gemm_debug_rowpanel.argtypes = [C.c_int]
kf.core.kf_gemm_debug_rowpanel(1)
T, bn, N, s = 96000, 160, 1536, 3
rng = np.random.default_rng(0)
h = lambda a: a.astype(np.float16)
x = kf.upload_fp16(h(rng.standard_normal((T + 1, bn))))
Wt = kf.upload_fp16(h(rng.standard_normal((N, 2 * bn)) / 16))
W = kf.upload_fp16(h(rng.standard_normal((2 * N, bn)) / 16))
bias = kf.upload_fp16(h(rng.uniform(-0.3, 0.3, N)))
sc = kf.upload_f32(np.ones(N, np.float32))
sh = kf.upload_f32(np.zeros(N, np.float32))
res = kf.upload_fp16(h(rng.standard_normal((T, N))))
out = kf.DeviceBuffer(T * N * 2)
out2 = kf.DeviceBuffer(T * N * 2)
mask = kf.DeviceBuffer(T * N // 8 + 64)
tr = torch.zeros(64 * 4, dtype=torch.int64, device="cuda")

cases = {
    "affine_fwd": (kf.operand(x.ptr, bn, T, 2 * bn, 1, nparts=2, part_width=bn, tpolicy=1, dt=(0, s)),
                   kf.operand(Wt.ptr, 2 * bn, N, 2 * bn, 1),
                   kf.KfEpilogue(out=out.ptr, ldo=N, alpha=1.0, bias=bias.ptr, relu=1, mask_out=mask.ptr,
                                 scale=sc.ptr, shift=sh.ptr, resid=res.ptr, ldr=N, resid_alpha=0.66)),
    "linear_dgrad": (kf.operand(x.ptr, bn, T, 2 * bn, 1, nparts=2, part_width=bn, tpolicy=0, dt=(s, 0),
                                edges=[(0, 0, T)]),
                     kf.operand(W.ptr, bn, N, 2 * bn, 1, nparts=2, part_width=bn, T=2 * N, dt=(0, N)),
                     kf.KfEpilogue(out=out.ptr, ldo=N, alpha=1.0, resid=res.ptr, ldr=N, resid_alpha=0.66,
                                   out2=out2.ptr, ldo2=N, scale2=sc.ptr, mask_in=mask.ptr)),
    "affine_no_mask": (kf.operand(x.ptr, bn, T, 2 * bn, 1, nparts=2, part_width=bn, tpolicy=1, dt=(0, s)),
                       kf.operand(Wt.ptr, 2 * bn, N, 2 * bn, 1),
                       kf.KfEpilogue(out=out.ptr, ldo=N, alpha=1.0, bias=bias.ptr, relu=1,
                                     scale=sc.ptr, shift=sh.ptr, resid=res.ptr, ldr=N, resid_alpha=0.66)),
    "affine_no_resid": (kf.operand(x.ptr, bn, T, 2 * bn, 1, nparts=2, part_width=bn, tpolicy=1, dt=(0, s)),
                        kf.operand(Wt.ptr, 2 * bn, N, 2 * bn, 1),
                        kf.KfEpilogue(out=out.ptr, ldo=N, alpha=1.0, bias=bias.ptr, relu=1, mask_out=mask.ptr,
                                      scale=sc.ptr, shift=sh.ptr)),
    "plain_store": (kf.operand(x.ptr, bn, T, 2 * bn, 1, nparts=2, part_width=bn, tpolicy=1, dt=(0, s)),
                    kf.operand(Wt.ptr, 2 * bn, N, 2 * bn, 1),
                    kf.KfEpilogue(out=out.ptr, ldo=N, alpha=1.0)),
}
for name, (a, b, e) in cases.items():
    run = lambda: kf.check(kf.core.kf_gemm_fused(T, N, 2 * bn, C.byref(a), C.byref(b), C.byref(e)))
    run()
    kf.sync()
    kf.core.kf_prof_reset()
    kf.core.kf_prof_enable(1)
    for _ in range(10):
        run()
    kf.sync()
    kf.core.kf_prof_enable(0)
    n, ms, fl = kf.prof_collect(0)
    kf.core.kf_prof_reset()
    kf.core.kf_rowpanel_trace(tr.data_ptr())
    run()
    kf.sync()
    kf.core.kf_rowpanel_trace(None)
    t = tr.cpu().numpy().reshape(64, 4).astype(np.float64) * 10e-3  # 100 MHz -> us
    print(f"{name}: {ms / max(n, 1) * 1e3:.1f} us per launch")
    nbk = N // 32
    for nb in range(0, nbk, nbk // 4):
        w, m, ep = t[nb, 1] - t[nb, 0], t[nb, 2] - t[nb, 1], t[nb, 3] - t[nb, 2]
        nxt = t[nb + 1, 0] - t[nb, 3] if nb + 1 < nbk else 0
        print(f"  block {nb:2d}: wait {w:6.2f}  mfma {m:6.2f}  epilogue {ep:6.2f}  gap {nxt:5.2f} us")
    tot = t[nbk - 1, 3] - t[0, 0]
    print(f"  {nbk} blocks: {tot:.1f} us")
