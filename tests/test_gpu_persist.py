"""The persistent fused GEMM with store waves (csrc/gemm_persist.hip), which kf_gemm_fused
takes for the short-K wide-N products (TDNN-F affine forward, linear input gradient,
forward.go:589-695, network_backward.go:336-463), against the tiled kernel on the same
operands (kf_gemm_debug_persist(0)) and against float64.

The two kernels run the same K-step and MFMA order per output element, so every output,
mask byte and second output must be bit-identical; the float64 check bounds both (fp32
accumulation K * 2^-23 * sum|ab| plus one fp16 rounding). Shapes: ragged last tiles
(M not a multiple of 128), a two-part clamped splice with its edge rows, K = 192 / 256 /
320 (3 to 5 K-steps: the store waves' step kst = 1 or 2), and the epilogues the network
uses (bias + ReLU + mask + BatchNorm + bypass residual; residual + out + out2 with scale2
x mask_in; plain alpha)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

U23 = 2.0 ** -23


def _h(a):
    return np.ascontiguousarray(a, np.float16)


def _run(kf, persist, M, N, K, a_args, b, e_kw, outs):
    prev = kf.core.kf_gemm_debug_persist(persist)
    for buf, nbytes in outs:
        kf.core.bridge_gpu_memset(buf.ptr, 0x5A, nbytes)
    a = kf.operand(*a_args[0], **a_args[1])
    e = kf.KfEpilogue(**e_kw)
    kf.check(kf.core.kf_gemm_fused(M, N, K, C.byref(a), C.byref(b), C.byref(e)), "fused")
    kf.sync()
    res = [kf.read_fp16(buf.ptr, (nbytes // 2,)).view(np.uint16).copy() for buf, nbytes in outs]
    kf.core.kf_gemm_debug_persist(prev)
    return res


@pytest.mark.parametrize("M,N,K,splice", [(11111, 1536, 320, True), (12000, 1536, 256, False),
                                          (33331, 512, 192, True), (20000, 1536, 320, False)])
@pytest.mark.parametrize("epi", ["forward", "dgrad", "plain"])
def test_persistent_matches_tiled_and_fp64(gpu, M, N, K, splice, epi):
    kf = gpu
    rng = np.random.default_rng(M + N + K)
    S = 3
    pw = K // 2 if splice else K
    x = _h(rng.standard_normal((M + 2, pw), dtype=np.float32))
    wt = _h(rng.standard_normal((N, K), dtype=np.float32) / np.sqrt(K))   # k-contiguous B (W^T rows)
    dx, dw = kf.upload_fp16(x), kf.upload_fp16(wt)
    if splice:  # [x(t) | x(t + S)] clamped, edge row: part 1 of row M - 1 reads spare row M
        a_args = ((dx.ptr, pw, M, K, 1), dict(nparts=2, part_width=pw, tpolicy=1, dt=(0, S), edges=[(1, M - 1, M)]))
    else:
        a_args = ((dx.ptr, pw, M, K, 1), {})
    b = kf.operand(dw.ptr, K, N, K, 1)
    out, out2 = kf.DeviceBuffer(M * N * 2), kf.DeviceBuffer(M * N * 2)
    mo = kf.DeviceBuffer(M * N // 8 + 16)
    resid = _h(rng.standard_normal((M, N), dtype=np.float32) * 0.5)
    dres = kf.upload_fp16(resid)
    bias = _h(rng.standard_normal(N) * 0.1)
    scale = rng.uniform(0.5, 1.5, N).astype(np.float32)
    shift = (rng.standard_normal(N) * 0.1).astype(np.float32)
    mask_in = rng.integers(0, 256, M * N // 8, dtype=np.uint8)
    db, dsc, dsh = kf.upload_fp16(bias), kf.upload_f32(scale), kf.upload_f32(shift)
    dmi = kf.DeviceBuffer(mask_in.nbytes + 16)
    kf.check(kf.core.bridge_transfer_int32(dmi.ptr, mask_in.ctypes.data, mask_in.nbytes // 4), "mask upload")
    if epi == "forward":
        e_kw = dict(out=out.ptr, ldo=N, alpha=1.0, bias=db.ptr, relu=1, mask_out=mo.ptr, scale=dsc.ptr,
                    shift=dsh.ptr, resid=dres.ptr, ldr=N, resid_alpha=0.66)
        outs = [(out, M * N * 2), (mo, M * N // 8)]
    elif epi == "dgrad":
        e_kw = dict(out=out.ptr, ldo=N, alpha=1.0, resid=dres.ptr, ldr=N, resid_alpha=0.66, out2=out2.ptr, ldo2=N,
                    scale2=dsc.ptr, mask_in=dmi.ptr)
        outs = [(out, M * N * 2), (out2, M * N * 2)]
    else:
        e_kw = dict(out=out.ptr, ldo=N, alpha=0.5)
        outs = [(out, M * N * 2)]
    got = _run(kf, 1, M, N, K, a_args, b, e_kw, outs)
    ref = _run(kf, 0, M, N, K, a_args, b, e_kw, outs)
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g, r)
    # float64 on sampled rows (edge rows included)
    rows = np.unique(np.concatenate([rng.choice(M, 2000, replace=False), [0, 1, M - 2, M - 1]]))
    xs = x.astype(np.float64)
    if splice:
        p1 = np.minimum(rows + S, M - 1)
        A = np.concatenate([xs[rows], np.where((rows == M - 1)[:, None], xs[M], xs[p1])], 1)
    else:
        A = xs[rows]
    W = wt.astype(np.float64).T
    acc = A @ W
    bound = K * U23 * (np.abs(A) @ np.abs(W)) + 1e-6 * np.abs(acc)
    g = got[0].view(np.float16).reshape(M, N)[rows].astype(np.float64)
    if epi == "forward":
        pre = acc + bias.astype(np.float64)
        v = np.maximum(pre, 0) * scale + shift + 0.66 * resid[rows].astype(np.float64)
        tol = bound * scale + np.abs(v) * 2 ** -10 + 1e-5 * (1 + np.abs(v)) + 2 ** -24
        assert np.all(np.abs(g - v) <= tol)
        bits = np.unpackbits(got[1].view(np.uint8).reshape(M, N // 8)[rows], axis=1, bitorder="little")
        sure = np.abs(pre) > bound
        assert np.array_equal(bits[sure].astype(bool), (pre > 0)[sure])
    elif epi == "dgrad":
        v = acc + 0.66 * resid[rows].astype(np.float64)
        tol = bound + np.abs(v) * 2 ** -10 + 1e-6 * np.abs(v) + 2 ** -24
        assert np.all(np.abs(g - v) <= tol)
        mb = np.unpackbits(mask_in.reshape(M, N // 8)[rows], axis=1, bitorder="little").astype(bool)
        v2 = v * scale * mb
        g2 = got[1].view(np.float16).reshape(M, N)[rows].astype(np.float64)
        assert np.all(np.abs(g2 - v2) <= tol * scale + np.abs(v2) * 2 ** -10 + 2 ** -24)
    else:
        v = 0.5 * acc
        assert np.all(np.abs(g - v) <= 0.5 * bound + np.abs(v) * 2 ** -10 + 2 ** -24)
