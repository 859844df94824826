"""Launch time of the persistent fused GEMM (gemm_persist.hip) against the tiled kernel on
the TDNN-F shapes (M = 96,000, N = 1536, K = 2 x 160 splice): the affine forward epilogue
(bias + ReLU + mask + BN + bypass) and the linear input-gradient epilogue (residual + scale
+ input mask). python scripts/persist_time.py"""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kaldi-fp16_amd", "python"))
import kfp16 as kf  # noqa: E402

torch.cuda.set_device(0)
kf.check(kf.core.bridge_gpu_init(0))
kf.set_stream(torch.cuda.current_stream().cuda_stream)
M, N, K, S = 96000, 1536, 320, 3
pw = K // 2
rng = np.random.default_rng(0)
x = kf.upload_fp16(rng.standard_normal((M + 2, pw), dtype=np.float32).astype(np.float16))
wt = kf.upload_fp16((rng.standard_normal((N, K), dtype=np.float32) / 18).astype(np.float16))
resid = kf.upload_fp16(rng.standard_normal((M, N), dtype=np.float32).astype(np.float16))
out, out2 = kf.DeviceBuffer(M * N * 2), kf.DeviceBuffer(M * N * 2)
mo, mi = kf.DeviceBuffer(M * N // 8), kf.DeviceBuffer(M * N // 8)
bias = kf.upload_fp16(np.zeros(N, np.float16))
sc, sh = kf.upload_f32(np.ones(N, np.float32)), kf.upload_f32(np.zeros(N, np.float32))
a = kf.operand(x.ptr, pw, M, K, 1, nparts=2, part_width=pw, tpolicy=1, dt=(0, S), edges=[(1, M - 1, M)])
b = kf.operand(wt.ptr, K, N, K, 1)


def epilogue(epi):
    if epi == "forward":
        return kf.KfEpilogue(out=out.ptr, ldo=N, alpha=1.0, bias=bias.ptr, relu=1, mask_out=mo.ptr, scale=sc.ptr,
                             shift=sh.ptr, resid=resid.ptr, ldr=N, resid_alpha=0.66)
    return kf.KfEpilogue(out=out.ptr, ldo=N, alpha=1.0, resid=resid.ptr, ldr=N, resid_alpha=0.66, out2=out2.ptr,
                         ldo2=N, scale2=sc.ptr, mask_in=mi.ptr)


for epi in ("forward", "dgrad"):
    e = epilogue(epi)
    for persist in (1, 0):
        kf.core.kf_gemm_debug_persist(persist)
        run = lambda: kf.check(kf.core.kf_gemm_fused(M, N, K, C.byref(a), C.byref(b), C.byref(e)), "fused")
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            run()
        torch.cuda.synchronize()
        print(f"{epi} persist={persist}: {(time.perf_counter() - t0) / 20 * 1e6:.1f} us per launch", flush=True)
kf.core.kf_gemm_debug_persist(0)
