"""The attention backward kernels alone (k_att_bwd_q / k_att_bwd_kv through
kf_attention_backward) on identical fp16 inputs, against the exact gradient.

The network test (test_gpu_attention.py) compares whole backward passes, where the
GPU and the oracle's F mode reach the attention layer with different fp16 roundings
of the upstream gradient, and the softmax backward w (dw - <w, dw>) cancels and
amplifies that difference. Here both sides get the same proj and dz, so a rounding
point that differs from the oracle's (which keeps w, dw and db in fp32 and rounds
dproj once, oracle/kf_oracle.c att_backward) would show directly:

  e_gpu = rel-Frobenius(GPU dproj, float64 exact)
  e_F   = rel-Frobenius(fp16(float32 restatement in the oracle's order), float64)
  e_rnd = rel-Frobenius(fp16(float64 exact), float64)   (one rounding, the floor)

Bar, per part of dproj (query key, query context, key, value), one seed:
e_gpu <= 1.25 * max(e_F, e_rnd). Shapes: the benchmark's attention layer (8 heads,
key 64, value 128, 5 left / 2 right at stride 3) and the tiny one.
Reference semantics: internal/nnet/forward.go:795-909 (forward), DESIGN.md §14."""
import ctypes as C

import numpy as np
import pytest

from conftest import rel_fro

pytestmark = pytest.mark.gpu


class KfAttention(C.Structure):
    _fields_ = [("proj", C.c_void_p), ("ldp", C.c_longlong), ("T", C.c_int), ("num_heads", C.c_int),
                ("key_dim", C.c_int), ("value_dim", C.c_int), ("context", C.c_int), ("num_left", C.c_int),
                ("stride", C.c_int), ("key_scale", C.c_float)]


def att_backward(proj, dz, H, kd, vd, nl, nr, st, s, dt):
    """The exact gradient of the restricted attention (the kernel header's formulas) in
    dtype dt, in the oracle's loop order per (t, h)."""
    T = proj.shape[0]
    ctx, A, od = 1 + nl + nr, 2 * kd + vd + 1 + nl + nr, vd + 1 + nl + nr
    P = proj.astype(dt).reshape(T, H, A)
    G = dz.astype(dt).reshape(T, H, od)
    dP = np.zeros_like(P)
    rows = np.arange(T)[:, None] + (np.arange(ctx)[None, :] - nl) * st          # [T, ctx]
    live = (rows >= 0) & (rows < T)
    rc = np.clip(rows, 0, T - 1)
    for h in range(H):
        key, val = P[:, h, :kd], P[:, h, kd:kd + vd]
        qk, qc = P[:, h, kd + vd:2 * kd + vd], P[:, h, 2 * kd + vd:]
        b = qc + dt(s) * np.where(live, np.einsum("td,tod->to", qk, key[rc]), dt(0))
        e = np.exp((b - b.max(1, keepdims=True)).astype(np.float64)).astype(dt)
        w = e / e.sum(1, keepdims=True, dtype=dt)
        gv, gw = G[:, h, :vd], G[:, h, vd:]
        dw = gw + np.where(live, np.einsum("td,tod->to", gv, val[rc]), dt(0))
        sw = (w * dw).sum(1, keepdims=True, dtype=dt)
        db = w * (dw - sw)
        dP[:, h, 2 * kd + vd:] = db
        dbl = np.where(live, db, dt(0))
        dP[:, h, kd + vd:2 * kd + vd] = dt(s) * np.einsum("to,tod->td", dbl, key[rc])
        for o in range(ctx):  # scatter to the attended rows
            ok = live[:, o]
            np.add.at(dP[:, h, :kd], rc[ok, o], dt(s) * dbl[ok, o, None] * qk[ok])
            np.add.at(dP[:, h, kd:kd + vd], rc[ok, o], w[ok, o, None] * gv[ok])
    return dP.reshape(T, H * A)


@pytest.mark.parametrize("H,kd,vd,T,seed", [(8, 64, 128, 240, 7), (8, 64, 128, 240, 8), (4, 16, 32, 301, 3)])
def test_attention_backward_kernel_rounding(gpu, H, kd, vd, T, seed):
    kf = gpu
    nl, nr, st = 5, 2, 3
    ctx = 1 + nl + nr
    A, od = 2 * kd + vd + ctx, vd + ctx
    rng = np.random.default_rng(seed)
    proj = rng.standard_normal((T, H * A)).astype(np.float16)
    dz = (rng.standard_normal((T, H * od)) * 0.05 * (rng.random((T, H * od)) < 0.6)).astype(np.float16)
    s = 1.0 / np.sqrt(kd)
    dp, dd = kf.upload_fp16(proj), kf.upload_fp16(dz)
    out = kf.DeviceBuffer(T * H * A * 2)
    scratch = kf.DeviceBuffer(2 * T * H * ctx * 4)
    a = KfAttention(dp.ptr, H * A, T, H, kd, vd, ctx, nl, st, s)
    kf.core.kf_attention_backward.argtypes = [C.POINTER(KfAttention), C.c_void_p, C.c_longlong, C.c_void_p,
                                              C.c_void_p]
    kf.check(kf.core.kf_attention_backward(C.byref(a), dd.ptr, H * od, out.ptr, scratch.ptr), "attention bwd")
    got = kf.read_fp16(out.ptr, (T, H * A)).astype(np.float64).reshape(T, H, A)
    r64 = att_backward(proj, dz, H, kd, vd, nl, nr, st, s, np.float64).reshape(T, H, A)
    r32 = att_backward(proj, dz, H, kd, vd, nl, nr, st, s, np.float32).astype(np.float16).astype(np.float64)
    r32 = r32.reshape(T, H, A)
    rnd = r64.astype(np.float16).astype(np.float64)
    parts = {"key": slice(0, kd), "value": slice(kd, kd + vd), "query key": slice(kd + vd, 2 * kd + vd),
             "query context": slice(2 * kd + vd, A)}
    for name, sl in parts.items():
        e_g = rel_fro(got[:, :, sl], r64[:, :, sl])
        e_f = rel_fro(r32[:, :, sl], r64[:, :, sl])
        e_r = rel_fro(rnd[:, :, sl], r64[:, :, sl])
        print(f"{name:14s} gpu {e_g:.2e}  F {e_f:.2e}  one rounding {e_r:.2e}")
        assert e_g <= 1.25 * max(e_f, e_r), (name, e_g, e_f, e_r)


def test_attention_backward_in_network_inputs(gpu):
    """The same bar on the network's own tensors: cnn_tdnn_17f_att at T = 240, the GPU's
    stored affine output (proj) and the gradient its backward hands the attention layer
    (dz, after the three layers above), where the softmax backward cancels. The network's
    dproj must be the kernel's output on those inputs, at the one-rounding floor."""
    kf = gpu
    from kfp16 import synth
    T = 240
    xcfg = synth.load_xconfig("cnn_tdnn_17f_att.xconfig")
    net = kf.Network(xcfg, max_frames=T)
    synth.init_network(net)
    fb = kf.upload_fp16(synth.make_features(T, 40))
    net.forward(fb.ptr, T)
    li = [n for n, *_ in net.layers].index("attention24")
    H, kd, vd, nl, nr, st = 8, 64, 128, 5, 2, 3
    ctx = 1 + nl + nr
    A, od = 2 * kd + vd + ctx, vd + ctx
    P = [d for n, _, _, d in net.layers if n == "output"][0]
    og = kf.upload_fp16((np.random.default_rng(7).standard_normal((T, P)) * 0.05).astype(np.float16))
    kf.check(kf.nnet.nnet_backward_n(net.h, og.ptr, 3), "backward_n")   # output, prefinal-chain, prefinal-l
    dz = kf.read_fp16(kf.nnet.nnet_debug_tensor(net.h, b"dzlast", 0), (T, H * od))
    proj = kf.read_fp16(kf.nnet.nnet_debug_tensor(net.h, b"aux", li), (T, H * A))
    kf.check(kf.nnet.nnet_backward_n(net.h, og.ptr, 4), "backward_n")
    got = kf.read_fp16(kf.nnet.nnet_debug_tensor(net.h, b"dproj", li), (T, H * A)).astype(np.float64)
    r64 = att_backward(proj, dz, H, kd, vd, nl, nr, st, 1.0 / np.sqrt(kd), np.float64)
    r32 = att_backward(proj, dz, H, kd, vd, nl, nr, st, 1.0 / np.sqrt(kd), np.float32)
    e_g = rel_fro(got, r64)
    e_f = rel_fro(r32.astype(np.float16).astype(np.float64), r64)
    e_r = rel_fro(r64.astype(np.float16).astype(np.float64), r64)
    print(f"in-network dproj: gpu {e_g:.2e}  F {e_f:.2e}  one rounding {e_r:.2e}")
    assert np.abs(dz).max() > 0 and e_g <= 1.25 * max(e_f, e_r), (e_g, e_f, e_r)
    net.close()
