"""kf_gemm_fused / kf_gemm_wgrad operand-addressing modes against numpy
(materialised splice / im2col / col2im, fp64 reference)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _h(a):
    return np.ascontiguousarray(a, np.float16)


def _check(got, ref, K, tol=2e-3):
    err = np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30)
    assert err <= tol, err


def splice(x, dts, policy):
    T = x.shape[0]
    cols = []
    for dt in dts:
        idx = np.arange(T) + dt
        if policy == 1:
            part = x[np.clip(idx, 0, T - 1)]
        else:
            part = np.where(((idx >= 0) & (idx < T))[:, None], x[np.clip(idx, 0, T - 1)], 0)
        cols.append(part)
    return np.concatenate(cols, 1)


def im2col(x, T, hin, fin, hout, sub, offs):
    xr = x.reshape(T, hin, fin)
    out = np.zeros((T, hout, len(offs), fin), x.dtype)
    for o, (dt, dh) in enumerate(offs):
        for t in range(T):
            ts = t + dt
            if ts < 0 or ts >= T:
                continue
            for h in range(hout):
                hs = h * sub + dh
                if 0 <= hs < hin:
                    out[t, h, o] = xr[ts, hs]
    return out.reshape(T * hout, len(offs) * fin)


@pytest.mark.parametrize("kc_b", [0, 1])
@pytest.mark.parametrize("M,N,K", [(300, 160, 320), (257, 64, 96), (128, 200, 64), (64, 1536, 320)])
def test_plain(gpu, kc_b, M, N, K):
    kf = gpu
    rng = np.random.default_rng(M + N + K)
    A = _h(rng.standard_normal((M, K)))
    W = _h(rng.standard_normal((K, N)) / np.sqrt(K))
    dA = kf.upload_fp16(A)
    dW = kf.upload_fp16(W if kc_b == 0 else W.T.copy())
    out = kf.DeviceBuffer(M * N * 2)
    a = kf.operand(dA.ptr, K, M, K, 1)
    b = kf.operand(dW.ptr, N, K, N, 0) if kc_b == 0 else kf.operand(dW.ptr, K, N, K, 1)
    e = kf.KfEpilogue(out=out.ptr, ldo=N, alpha=1.0)
    kf.check(kf.core.kf_gemm_fused(M, N, K, C.byref(a), C.byref(b), C.byref(e)))
    _check(kf.read_fp16(out.ptr, (M, N)).astype(np.float64), A.astype(np.float64) @ W.astype(np.float64), K)


@pytest.mark.parametrize("s,dts,pol", [(3, (-3, 0), 1), (3, (0, 3), 1), (2, (2, 0), 0), (1, (0, -1), 0)])
def test_splice_operand(gpu, s, dts, pol):
    kf = gpu
    rng = np.random.default_rng(s)
    T, d, N = 203, 64, 96
    x = _h(rng.standard_normal((T, d)))
    W = _h(rng.standard_normal((2 * d, N)) / 8)
    dx, dW = kf.upload_fp16(x), kf.upload_fp16(W)
    out = kf.DeviceBuffer(T * N * 2)
    a = kf.operand(dx.ptr, d, T, 2 * d, 1, nparts=2, part_width=d, tpolicy=pol, dt=dts)
    b = kf.operand(dW.ptr, N, 2 * d, N, 0)
    e = kf.KfEpilogue(out=out.ptr, ldo=N, alpha=1.0)
    kf.check(kf.core.kf_gemm_fused(T, N, 2 * d, C.byref(a), C.byref(b), C.byref(e)))
    ref = splice(x.astype(np.float64), dts, pol) @ W.astype(np.float64)
    _check(kf.read_fp16(out.ptr, (T, N)).astype(np.float64), ref, 2 * d)


@pytest.mark.parametrize("hin,fin,hout,sub,fout", [(10, 32, 10, 1, 64), (20, 32, 10, 2, 32), (8, 64, 4, 2, 128)])
def test_im2col_and_col2im(gpu, hin, fin, hout, sub, fout):
    kf = gpu
    rng = np.random.default_rng(hin * fin)
    T = 37
    offs = [(a, b) for a in (-1, 0, 1) for b in (-1, 0, 1)]
    x = _h(rng.standard_normal((T, hin * fin)))
    W = _h(rng.standard_normal((9 * fin, fout)) / 16)
    dx, dW = kf.upload_fp16(x), kf.upload_fp16(W)
    M, K = T * hout, 9 * fin
    out = kf.DeviceBuffer(M * fout * 2)
    a = kf.operand(dx.ptr, hin * fin, M, K, 1, nparts=9, part_width=fin, T=T, hout=hout, hsrc=hin,
                   hmul=sub, hdiv=1, tpolicy=0, dt=[o[0] for o in offs], dh=[o[1] for o in offs])
    b = kf.operand(dW.ptr, fout, K, fout, 0)
    e = kf.KfEpilogue(out=out.ptr, ldo=fout, alpha=1.0)
    kf.check(kf.core.kf_gemm_fused(M, fout, K, C.byref(a), C.byref(b), C.byref(e)))
    P = im2col(x.astype(np.float64), T, hin, fin, hout, sub, offs)
    _check(kf.read_fp16(out.ptr, (M, fout)).astype(np.float64), P @ W.astype(np.float64), K)
    # transpose: dx = col2im(dz . W^T) via the gather operand
    dz = _h(rng.standard_normal((M, fout)))
    ddz = kf.upload_fp16(dz)
    gx = kf.DeviceBuffer(T * hin * fin * 2)
    a2 = kf.operand(ddz.ptr, hout * fout, T * hin, 9 * fout, 1, nparts=9, part_width=fout, T=T, hout=hin,
                    hsrc=hout, hmul=1, hdiv=sub, tpolicy=0, dt=[-o[0] for o in offs], dh=[-o[1] for o in offs])
    b2 = kf.operand(dW.ptr, fout, fin, 9 * fout, 1, nparts=9, part_width=fout, T=9 * fin,
                    dt=[p * fin for p in range(9)])
    e2 = kf.KfEpilogue(out=gx.ptr, ldo=fin, alpha=1.0)
    kf.check(kf.core.kf_gemm_fused(T * hin, fin, 9 * fout, C.byref(a2), C.byref(b2), C.byref(e2)))
    dP = dz.astype(np.float64) @ W.astype(np.float64).T
    ref = np.zeros((T, hin, fin))
    for o, (dt, dh) in enumerate(offs):
        for t in range(T):
            ts = t + dt
            if not 0 <= ts < T:
                continue
            for h in range(hout):
                hs = h * sub + dh
                if 0 <= hs < hin:
                    ref[ts, hs] += dP[t * hout + h, o * fin:(o + 1) * fin]
    _check(kf.read_fp16(gx.ptr, (T * hin, fin)).astype(np.float64), ref.reshape(T * hin, fin), 9 * fout)
    # weight gradient with the im2col operand (reduction-major)
    gW = kf.DeviceBuffer(K * fout * 4)
    gb = kf.DeviceBuffer(fout * 4)
    a3 = kf.operand(dx.ptr, hin * fin, M, K, 0, nparts=9, part_width=fin, T=T, hout=hout, hsrc=hin,
                    hmul=sub, hdiv=1, tpolicy=0, dt=[o[0] for o in offs], dh=[o[1] for o in offs])
    b3 = kf.operand(ddz.ptr, fout, M, fout, 0)
    kf.check(kf.core.kf_gemm_wgrad(K, fout, M, C.byref(a3), C.byref(b3), gW.ptr, fout, gb.ptr, 0))
    _check(kf.read_f32(gW.ptr, (K, fout)), P.T @ dz.astype(np.float64), M)
    _check(kf.read_f32(gb.ptr, (fout,)), dz.astype(np.float64).sum(0), M)


@pytest.mark.parametrize("M,N,T", [(320, 160, 1000), (3072, 160, 777), (288, 32, 6000), (256, 3080, 500)])
def test_wgrad_plain(gpu, M, N, T):
    kf = gpu
    rng = np.random.default_rng(M + N)
    X = _h(rng.standard_normal((T, M)))
    D = _h(rng.standard_normal((T, N)))
    dX, dD = kf.upload_fp16(X), kf.upload_fp16(D)
    gW = kf.DeviceBuffer(M * N * 4)
    gb = kf.DeviceBuffer(N * 4)
    a = kf.operand(dX.ptr, M, T, M, 0)
    b = kf.operand(dD.ptr, N, T, N, 0)
    kf.check(kf.core.kf_gemm_wgrad(M, N, T, C.byref(a), C.byref(b), gW.ptr, N, gb.ptr, 0))
    _check(kf.read_f32(gW.ptr, (M, N)), X.astype(np.float64).T @ D.astype(np.float64), T)
    _check(kf.read_f32(gb.ptr, (N,)), D.astype(np.float64).sum(0), T)
