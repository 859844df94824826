"""Timeline of the persistent fused GEMM (gemm_persist.hip) on the TDNN-F affine forward
shape (M = 96,000, N = 1536, K = 2 x 160 splice, bias + ReLU + mask + BN + bypass):
block 0's MFMA wave 0 and store wave 0 stamps (kf_gemm_persist_trace), plus the launch
time of the persistent and the tiled kernel. python scripts/persist_trace.py [epi]"""
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
kf.core.kf_gemm_persist_trace.argtypes = [kf._vp]
epi = sys.argv[1] if len(sys.argv) > 1 else "forward"
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
if epi == "forward":
    e = kf.KfEpilogue(out=out.ptr, ldo=N, alpha=1.0, bias=bias.ptr, relu=1, mask_out=mo.ptr, scale=sc.ptr,
                      shift=sh.ptr, resid=resid.ptr, ldr=N, resid_alpha=0.66)
else:
    e = kf.KfEpilogue(out=out.ptr, ldo=N, alpha=1.0, resid=resid.ptr, ldr=N, resid_alpha=0.66, out2=out2.ptr,
                      ldo2=N, scale2=sc.ptr, mask_in=mi.ptr)


def run():
    kf.check(kf.core.kf_gemm_fused(M, N, K, C.byref(a), C.byref(b), C.byref(e)), "fused")


for persist in (1, 0):
    kf.core.kf_gemm_debug_persist(persist)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        run()
    torch.cuda.synchronize()
    print(f"persist={persist}: {(time.perf_counter() - t0) / 20 * 1e6:.1f} us per launch")
kf.core.kf_gemm_debug_persist(1)
tb = torch.zeros(256, dtype=torch.int64, device="cuda")
kf.core.kf_gemm_persist_trace(tb.data_ptr())
run()
torch.cuda.synchronize()
t = tb.cpu().numpy().astype(np.float64) * 10e-3  # 100 MHz ticks -> us
t0 = t[0]
for i in range(6):
    m = t[i * 16:i * 16 + 11] - t0
    s = t[128 + i * 16:128 + i * 16 + 14] - t0
    print(f"tile {i}: MFMA steps landed " + " ".join(f"{v:6.2f}" for v in m[:5]) +
          f" | K done {m[8]:6.2f} half0 read {m[9]:6.2f} handoff {m[10]:6.2f}")
    print(f"        store steps " + " ".join(f"{v:6.2f}" for v in s[:5]) +
          f" | loads landed {s[8]:6.2f} passes " + " ".join(f"{v:6.2f}" for v in s[9:13]))
