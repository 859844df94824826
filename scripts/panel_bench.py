"""Micro-benchmark of the TDNN-F short-K fused GEMMs (T = 96,000, K = 2 x 160,
N = 1536): panel kernel vs tiled kernel, plain store vs full epilogue.
HIP-event timing via kf_prof_*. KF_PANEL_DBG=1/2 isolates B loads / epilogue."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kaldi-fp16_amd", "python"))
import numpy as np  # noqa: E402
import kfp16 as kf  # noqa: E402

kf.check(kf.core.bridge_gpu_init(0))
kf.core.kf_gemm_debug_panel.argtypes = [C.c_int]
rng = np.random.default_rng(0)
T, bn, N = 96000, 160, 1536
K = 2 * bn
X = kf.upload_fp16((rng.standard_normal((T + 2, bn)) * 0.1).astype(np.float16))
Wt = kf.upload_fp16((rng.standard_normal((N, K)) * 0.05).astype(np.float16))
W = kf.upload_fp16((rng.standard_normal((K, N)) * 0.05).astype(np.float16))
R = kf.upload_fp16((rng.standard_normal((T, N)) * 0.1).astype(np.float16))
Y = kf.DeviceBuffer(T * N * 2)
Y2 = kf.DeviceBuffer(T * N * 2)
mask = kf.DeviceBuffer(T * N // 8 + 64)
bias = kf.upload_fp16(np.zeros(N, np.float16))
sc = kf.upload_f32(np.ones(N, np.float32))
sh = kf.upload_f32(np.zeros(N, np.float32))


def timeit(fn, reps=20):
    fn()
    kf.sync()
    kf.core.kf_prof_reset()
    kf.core.kf_prof_enable(1)
    for _ in range(reps):
        fn()
    kf.sync()
    kf.core.kf_prof_enable(0)
    n, ms, fl, by = kf.prof_collect2(0)
    kf.core.kf_prof_reset()
    return ms / reps * 1e3, by / n


a = kf.operand(X.ptr, bn, T, K, 1, nparts=2, part_width=bn, tpolicy=1, dt=(0, 3))
bkc = kf.operand(Wt.ptr, K, N, K, 1)
bmn = kf.operand(W.ptr, N, K, N, 0)
# linear dX: zero policy + edge row, op_wrows B, out + out2 + resid + mask_in
Wl = kf.upload_fp16((rng.standard_normal((2 * N, bn)) * 0.05).astype(np.float16))
ad = kf.operand(X.ptr, bn, T, K, 1, nparts=2, part_width=bn, tpolicy=0, dt=(3, 0), edges=[(0, 0, T)])
bw = kf.operand(Wl.ptr, bn, N, K, 1, nparts=2, part_width=bn, T=2 * N, dt=(0, N))
epis = {
    "plain": kf.KfEpilogue(out=Y.ptr, ldo=N, alpha=1.0),
    "affine": kf.KfEpilogue(out=Y.ptr, ldo=N, alpha=1.0, bias=bias.ptr, relu=1, mask_out=mask.ptr,
                            scale=sc.ptr, shift=sh.ptr, resid=R.ptr, ldr=N, resid_alpha=0.66),
    "dgrad": kf.KfEpilogue(out=Y.ptr, ldo=N, alpha=1.0, resid=R.ptr, ldr=N, resid_alpha=0.66, out2=Y2.ptr,
                           ldo2=N, scale2=sc.ptr, mask_in=mask.ptr),
}
for name, e in epis.items():
    for mode in (1, 0):
        kf.core.kf_gemm_debug_panel(mode)
        A_, B_ = (ad, bw) if name == "dgrad" else (a, bkc if mode else bmn)
        us, by = timeit(lambda: kf.check(kf.core.kf_gemm_fused(T, N, K, C.byref(A_), C.byref(B_), C.byref(e))))
        print(f"{name:8s} {'panel' if mode else 'tiled':6s} {us:8.1f} us  {by / 1e6:7.1f} MB  "
              f"{by / (us * 1e-6) / 1e9:7.1f} GB/s", flush=True)
kf.core.kf_gemm_debug_panel(-1)
# the tiled kernel on the affine forward with the transposed (k-contiguous) weights
kf.core.kf_gemm_debug_panel(0)
for name in ("plain", "affine"):
    e = epis[name]
    us, by = timeit(lambda: kf.check(kf.core.kf_gemm_fused(T, N, K, C.byref(a), C.byref(bkc), C.byref(e))))
    print(f"{name:8s} tiledKC {us:8.1f} us  {by / 1e6:7.1f} MB  {by / (us * 1e-6) / 1e9:7.1f} GB/s", flush=True)
kf.core.kf_gemm_debug_panel(-1)
