"""Micro-benchmark of kf_gemm_fused / kf_gemm_wgrad on the CNN-TDNN shapes,
isolating the core loop (plain operands, plain store) from the implicit
addressing and the fused epilogue. HIP-event timing via kf_prof_*."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kaldi-fp16_amd", "python"))
import numpy as np  # noqa: E402
import kfp16 as kf  # noqa: E402

kf.check(kf.core.bridge_gpu_init(0))
rng = np.random.default_rng(0)
bufs = {}


sizes = {}


def buf(name, nbytes):
    if name not in bufs or bufs[name].nbytes < nbytes:
        b = kf.DeviceBuffer(nbytes)
        kf.core.bridge_gpu_memset(b.ptr, 0, nbytes)
        bufs[name] = b
        sizes[b.ptr] = nbytes
    return bufs[name].ptr


def need(ptr, elems):
    """refuse to launch an operand that would read past its allocation"""
    assert elems * 2 <= sizes[ptr], (elems * 2, sizes[ptr])


def fill(name, n):
    a = (rng.standard_normal(n) * 0.1).astype(np.float16)
    p = buf(name, a.nbytes + 1024)
    kf.check(kf.core.bridge_transfer_fp16(p, a.ctypes.data, a.size))
    return p


def timeit(fn, flops, reps=10):
    fn()
    kf.sync()
    kf.core.kf_prof_reset()
    kf.core.kf_prof_enable(1)
    for _ in range(reps):
        fn()
    kf.sync()
    kf.core.kf_prof_enable(0)
    tot_ms = 0.0
    for cls in (0, 1):
        n, ms, fl = kf.prof_collect(cls)
        tot_ms += ms
    kf.core.kf_prof_reset()
    us = tot_ms / reps * 1e3
    return us, flops / (us * 1e-6) / 1e12


def fused(M, N, K, a, b, e):
    return lambda: kf.check(kf.core.kf_gemm_fused(M, N, K, C.byref(a), C.byref(b), C.byref(e)))


T = 96000
X = fill("X", T * 3072)
W = fill("W", 8192 * 8192)
Y = buf("Y", T * 3080 * 2)
R = fill("R", T * 2560)
mask = buf("mask", T * 3080 // 8 + 64)
scale = kf.upload_f32(np.ones(3080, np.float32))
shift = kf.upload_f32(np.zeros(3080, np.float32))
rows = []
for (label, M, N, K) in [("sq8192", 8192, 8192, 8192), ("tdnnf_lin_fwd", T, 160, 3072),
                         ("tdnnf_aff_fwd", T, 1536, 320), ("output_fwd", T, 3080, 256)]:
    if label == "sq8192":
        Xp = fill("Xsq", 8192 * 8192)
    else:
        Xp = X
    need(Xp, M * K), need(W, K * N), need(Y, M * N)
    a = kf.operand(Xp, K, M, K, 1)
    b = kf.operand(W, N, K, N, 0)
    e = kf.KfEpilogue(out=Y, ldo=N, alpha=1.0)
    us, tf = timeit(fused(M, N, K, a, b, e), 2.0 * M * N * K)
    rows.append((label + " plain/MN", us, tf))
    b2 = kf.operand(W, K, N, K, 1)
    us, tf = timeit(fused(M, N, K, a, b2, e), 2.0 * M * N * K)
    rows.append((label + " plain/KC", us, tf))
# conv6 forward through the implicit im2col operand (x = [T x 10*256])
offs = [(a_, b_) for a_ in (-1, 0, 1) for b_ in (-1, 0, 1)]
need(X, T * 2560), need(W, 2304 * 256), need(Y, T * 10 * 256)
a = kf.operand(X, 2560, T * 10, 2304, 1, nparts=9, part_width=256, T=T, hout=10, hsrc=10, hmul=1,
               dt=[o[0] for o in offs], dh=[o[1] for o in offs])
b = kf.operand(W, 256, 2304, 256, 0)
e = kf.KfEpilogue(out=Y, ldo=256, alpha=1.0)
rows.append(("conv6_fwd im2col", *timeit(fused(T * 10, 256, 2304, a, b, e), 2.0 * T * 10 * 256 * 2304)))
# implicit splice + full epilogue on the TDNN-F shapes
for (label, M, N, d) in [("tdnnf_lin_fwd splice", T, 160, 1536), ("tdnnf_aff_fwd splice", T, 1536, 160)]:
    K = 2 * d
    need(X, T * d), need(W, K * N), need(Y, M * N), need(R, M * N)
    a = kf.operand(X, d, M, K, 1, nparts=2, part_width=d, tpolicy=1, dt=(-3, 0))
    b = kf.operand(W, N, K, N, 0)
    e = kf.KfEpilogue(out=Y, ldo=N, alpha=1.0)
    rows.append((label, *timeit(fused(M, N, K, a, b, e), 2.0 * M * N * K)))
    e = kf.KfEpilogue(out=Y, ldo=N, alpha=1.0, bias=W, relu=1, mask_out=mask, scale=scale.ptr,
                      shift=shift.ptr, resid=R if N == 1536 else None, ldr=N, resid_alpha=0.66)
    rows.append((label + " +epi", *timeit(fused(M, N, K, a, b, e), 2.0 * M * N * K)))
# weight gradients
for (label, M, N) in [("wgrad lin", 3072, 160), ("wgrad aff", 320, 1536), ("wgrad 256x1536", 256, 1536)]:
    Kr = T
    need(X, Kr * M), need(R, Kr * N)
    a = kf.operand(X, M, Kr, M, 0)
    b = kf.operand(R, N, Kr, N, 0)
    g = buf("G", M * N * 4)
    fn = lambda: kf.check(kf.core.kf_gemm_wgrad(M, N, Kr, C.byref(a), C.byref(b), g, N, None, 0))
    rows.append((label, *timeit(fn, 2.0 * M * N * Kr)))
for r in rows:
    print(f"{r[0]:32s} {r[1]:9.1f} us {r[2]:8.1f} TFLOP/s")
