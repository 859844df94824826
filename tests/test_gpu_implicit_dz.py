"""Masked GEMM operands (include/kf_ops.h) and the implicit TDNN-F dz they carry
(include/kf_nnet.h nnet_set_implicit_dz, host/network.cpp dx_epilogue / the TDNN-F
backward).

The input-gradient epilogue that produces a TDNN-F layer's output gradient g no longer
stores dz = rne(g * bnscale * relu_mask). The layer's consumers read g through the
forward's ReLU mask instead:
  affine dX   dbott = transpose of the [0, +s] splice of (g . mask) . rne(W2 * bnscale)^T,
              the clamped edge row T = rne(sum of the masked rows) (kf_rows_sum_mask)
  affine dW   bnscale[n] * sum_t splice(bott)[t] (g . mask)[t][n] (kf_gemm_wgrad_scaled,
              the scale applied in the split-K reduce), db the same column-scaled sums
Reference semantics: internal/gpu/backward_ops.go:162-253 (dX / dW / db of the affine),
internal/nnet/network_backward.go:336-463 (backwardTDNNF). References in float64 over the
tensors the GPU consumed (g, the mask bits, the fp16 W2 copy, the edge row); bounds as in
test_gpu_benchsize.py (the fp32 accumulation bound plus one fp16 rounding).
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BN, DOUT, S = 160, 1536, 3
U23 = 2.0 ** -23


def _h(a):
    return np.ascontiguousarray(a, np.float16)


def _within(got, ref, tol, what):
    bad = np.abs(got - ref) > tol
    assert not bad.any(), (what, int(bad.sum()), float(np.max(np.abs(got - ref) - tol)))


def _bits_all(mask_bytes, T, width):
    return np.unpackbits(mask_bytes.reshape(T, width // 8), axis=1, bitorder="little").astype(bool)


@pytest.mark.parametrize("T", [3000, pytest.param(96000, marks=pytest.mark.slow)])
def test_masked_affine_dgrad_and_wgrad(gpu, T):
    kf = gpu
    rng = np.random.default_rng(T + 7)
    g = _h(rng.standard_normal((T + 2, DOUT)) * 0.02)
    bott = _h(rng.standard_normal((T + 2, BN)))
    w2 = _h(rng.standard_normal((2 * BN, DOUT)) / np.sqrt(2 * DOUT))   # [kaff x dout]
    scale = rng.uniform(0.5, 1.5, DOUT).astype(np.float32)
    mask = rng.integers(0, 256, T * DOUT // 8, dtype=np.uint8)
    dg, dbt, dw2 = kf.upload_fp16(g), kf.upload_fp16(bott), kf.upload_fp16(w2)
    dsc = kf.upload_f32(scale)
    dmk = kf.DeviceBuffer(mask.nbytes)
    kf.check(kf.core.bridge_transfer_int32(dmk.ptr, mask.ctypes.data, mask.nbytes // 4), "mask upload")
    dw2s = kf.DeviceBuffer(2 * BN * DOUT * 2)
    dbott = kf.DeviceBuffer((T + 2) * BN * 2)
    gW, gb = kf.DeviceBuffer(2 * BN * DOUT * 4), kf.DeviceBuffer(DOUT * 4)

    kf.check(kf.core.kf_scale_cols(dw2.ptr, DOUT, dsc.ptr, dw2s.ptr, DOUT, 2 * BN, DOUT), "scaled W2")
    edge = dg.ptr + T * DOUT * 2
    kf.check(kf.core.kf_rows_sum_mask(edge, dg.ptr, DOUT, T - 1 - S, T, DOUT, dmk.ptr), "edge")
    a1 = kf.operand(dg.ptr, DOUT, T, 2 * DOUT, 1, nparts=2, part_width=DOUT, tpolicy=0, dt=(0, -S),
                    edges=[(1, T - 1, T)], mask=dmk.ptr, mask_rows=T)
    b1 = kf.operand(dw2s.ptr, DOUT, BN, 2 * DOUT, 1, nparts=2, part_width=DOUT, T=2 * BN, dt=(0, BN))
    e1 = kf.KfEpilogue(out=dbott.ptr, ldo=BN, alpha=1.0)
    kf.check(kf.core.kf_gemm_fused(T, BN, 2 * DOUT, C.byref(a1), C.byref(b1), C.byref(e1)), "masked dgrad")
    aw = kf.operand(dbt.ptr, BN, T, 2 * BN, 0, nparts=2, part_width=BN, tpolicy=1, dt=(0, S))
    bw = kf.operand(dg.ptr, DOUT, T, DOUT, 0, mask=dmk.ptr, mask_rows=T)
    kf.check(kf.core.kf_gemm_wgrad_scaled(2 * BN, DOUT, T, C.byref(aw), C.byref(bw), gW.ptr, DOUT, gb.ptr, 0,
                                          dsc.ptr), "masked wgrad")
    kf.sync()

    g_w2s = kf.read_fp16(dw2s.ptr, (2 * BN, DOUT))
    w2s_ref = _h(w2.astype(np.float32) * scale)
    bad = np.argwhere(g_w2s.view(np.uint16) != w2s_ref.view(np.uint16))
    assert bad.size == 0, ("rne(W2 * scale)", len(bad), [(tuple(i), float(w2[tuple(i)]), float(scale[i[1]]),
                                                          float(g_w2s[tuple(i)]), float(w2s_ref[tuple(i)]))
                                                         for i in bad[:8]])
    bits = _bits_all(mask, T, DOUT)
    gm = g[:T].astype(np.float64) * bits
    g_edge = kf.read_fp16(edge, (DOUT,)).astype(np.float64)
    edge_ref = gm[T - 1 - S:T].sum(0)
    _within(g_edge, edge_ref, np.abs(edge_ref) * 2 ** -10 + 1e-6, "masked edge row")

    rows = np.array(sorted({0, 1, S, S + 1, T - 1, T - 2, T - 1 - S} |
                           set(rng.choice(T, min(T, 4096), replace=False).tolist())))
    p1 = np.where((rows - S >= 0)[:, None], gm[np.clip(rows - S, 0, T - 1)], 0.0)
    p1[rows == T - 1] = g_edge
    A = np.concatenate([gm[rows], p1], 1)
    w2s64 = g_w2s.astype(np.float64)
    Wt = np.concatenate([w2s64[:BN].T, w2s64[BN:].T], 0)
    ref = A @ Wt
    tol = 2 * DOUT * U23 * (np.abs(A) @ np.abs(Wt)) + np.abs(ref) * 2 ** -10 + 2 ** -24
    _within(kf.read_fp16(dbott.ptr, (T + 2, BN))[rows].astype(np.float64), ref, tol, "masked affine dgrad")

    # every element of dW / db
    acc = np.zeros((2 * BN, DOUT))
    mag = np.zeros((2 * BN, DOUT), np.float32)
    allr = np.arange(T)
    for t0 in range(0, T, 12000):
        r = allr[t0:t0 + 12000]
        Ab = np.concatenate([bott[r].astype(np.float64), bott[np.clip(r + S, 0, T - 1)].astype(np.float64)], 1)
        acc += Ab.T @ gm[r]
        mag += np.abs(Ab).astype(np.float32).T @ np.abs(gm[r]).astype(np.float32)
    sc = scale.astype(np.float64)
    g_W = kf.read_f32(gW.ptr, (2 * BN, DOUT)).astype(np.float64)
    _within(g_W, acc * sc, (T * U23 * mag.astype(np.float64) * 1.01 + np.abs(acc) * 2 ** -23) * sc + 1e-30,
            "masked affine dW")
    bref = gm.sum(0)
    _within(kf.read_f32(gb.ptr, (DOUT,)).astype(np.float64), bref * sc,
            (T * U23 * np.abs(gm).sum(0) + np.abs(bref) * 2 ** -23) * sc, "masked affine db")


def test_masked_operand_rejected_where_unsupported(gpu):
    """A masked operand anywhere else fails with an error instead of reading unmasked."""
    kf = gpu
    T = 256
    g, w = kf.upload_fp16(np.zeros((T, DOUT), np.float16)), kf.upload_fp16(np.zeros((DOUT, BN), np.float16))
    mk = kf.DeviceBuffer(T * DOUT // 8)
    out = kf.DeviceBuffer(T * BN * 4)
    a = kf.operand(g.ptr, DOUT, T, DOUT, 1)
    b = kf.operand(w.ptr, BN, DOUT, BN, 0, mask=mk.ptr, mask_rows=DOUT)  # masked B of a fused GEMM
    e = kf.KfEpilogue(out=out.ptr, ldo=BN, alpha=1.0)
    assert kf.core.kf_gemm_fused(T, BN, DOUT, C.byref(a), C.byref(b), C.byref(e)) != 0
    aw = kf.operand(g.ptr, DOUT, T, DOUT, 0, mask=mk.ptr, mask_rows=T)     # masked A of a wgrad
    bw = kf.operand(g.ptr, DOUT, T, DOUT, 0)
    assert kf.core.kf_gemm_wgrad(DOUT, DOUT, T, C.byref(aw), C.byref(bw), out.ptr, DOUT, None, 0) != 0
