"""The TDNN-F GEMMs at the benchmark's size (T = 96,000 rows: 64 egs x 1500 frames)
against float64, with the same operands the host layer builds (host/network.cpp
forward :1195-1231, backward :1508-1566).

Tile shapes, split counts, the splice-part XCD pairing of the linear weight gradient
(WgradArgs::pair_ps), the split-K slab reduce with the bias column sums
(k_slab_reduce_both) and the K-step interleave of the wide two-part A are all chosen
by size, so the small parity tests elsewhere do not run the configuration the bench
runs. Here:

  linear forward   aux = splice(x; -s, 0 clamp) . W_lin        K = 2 x 1536 -> N = 160
  affine forward   y = bn(relu(splice(aux; 0, +s clamp) . W_aff + b)) + 0.66 x
                   (W_aff read through its k-contiguous transposed copy, as nl.wt)
  affine dX        dbott = transpose of the [0, +s] splice of dz . W_aff^T (edge row T)
  linear dX        dx = epi(transpose of the [-s, 0] splice of dbott . W_lin^T) with the
                   bypass residual, BN scale and ReLU mask of the layer below
  both dW / db     split-K over T, every element

Fused outputs are checked on 4,096 sampled rows (the clamped edge rows included), the
weight gradients on every element. Bounds: the fp32 accumulation bound
K * 2^-23 * sum|a||b| per element, times the epilogue's per-column scale, plus one
fp16 rounding (|ref| * 2^-10) of the stored result. References replay the stored fp16
tensors the GPU consumed (aux, dbott, the edge rows), i.e. the kernels' rounding points.
Reference semantics: internal/nnet/forward.go:589-695 (TDNN-F), cpp/cuda/ops.cu:381-392
(the GEMM), internal/gpu/backward_ops.go:162-253 (dX / dW / db).
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

T, DIN, BN, DOUT, S, ALPHA = 96000, 1536, 160, 1536, 3, 0.66
U23 = 2.0 ** -23


def _h(a):
    return np.ascontiguousarray(a, np.float16)


def splice(x, rows, dts, clamp=True):
    """rows of [x(t + dts[0]) | x(t + dts[1])] (fp64)"""
    n = x.shape[0]
    parts = []
    for dt in dts:
        idx = rows + dt
        if clamp:
            parts.append(x[np.clip(idx, 0, n - 1)].astype(np.float64))
        else:
            ok = (idx >= 0) & (idx < n)
            parts.append(np.where(ok[:, None], x[np.clip(idx, 0, n - 1)].astype(np.float64), 0.0))
    return np.concatenate(parts, 1)


def _bits(mask_bytes, rows, width):
    m = mask_bytes.reshape(-1, width // 8)[rows]
    return np.unpackbits(m, axis=1, bitorder="little").astype(bool)


def _within(got, ref, tol, what):
    bad = np.abs(got - ref) > tol
    assert not bad.any(), (what, int(bad.sum()), float(np.max(np.abs(got - ref) - tol)))


def _wgrad_ref(a_src, a_dts, b, M, N):
    """splice(a)^T . b over all T rows in fp64, and the bound sum |a||b| (fp32 is enough
    for a bound), blockwise"""
    acc = np.zeros((M, N))
    mag = np.zeros((M, N), np.float32)
    for t0 in range(0, T, 12000):
        rows = np.arange(t0, min(T, t0 + 12000))
        A = splice(a_src, rows, a_dts) if a_dts else a_src[rows].astype(np.float64)
        B = b[rows].astype(np.float64)
        acc += A.T @ B
        mag += np.abs(A).astype(np.float32).T @ np.abs(B).astype(np.float32)
    return acc, mag.astype(np.float64) * 1.01


def test_tdnnf_layer_gemms_at_bench_size(gpu):
    kf = gpu
    rng = np.random.default_rng(96000)
    # ---- inputs (fp16 as the network stores them; +2 spare rows like its buffers)
    x = _h(np.maximum(rng.standard_normal((T + 2, DIN)), -0.5))
    w_lin = _h(rng.standard_normal((2 * DIN, BN)) / np.sqrt(2 * DIN))
    w_aff = _h(rng.standard_normal((2 * BN, DOUT)) / np.sqrt(2 * BN))
    w_aff_t = _h(w_aff.T)
    bias = _h(rng.standard_normal(DOUT) * 0.1)
    scale = (rng.uniform(0.5, 1.5, DOUT)).astype(np.float32)
    shift = (rng.standard_normal(DOUT) * 0.1).astype(np.float32)
    dz = _h(rng.standard_normal((T + 2, DOUT)) * 0.02)        # gradient at the affine pre-activation
    gcur = _h(rng.standard_normal((T + 2, DOUT)) * 0.02)      # layer output gradient (bypass)
    scale2 = (rng.uniform(0.5, 1.5, DIN)).astype(np.float32)  # BN scale of the layer below
    mask_in = rng.integers(0, 256, T * DIN // 8, dtype=np.uint8)

    dx_ = kf.upload_fp16(x)
    dwl, dwa, dwat, db_ = kf.upload_fp16(w_lin), kf.upload_fp16(w_aff), kf.upload_fp16(w_aff_t), kf.upload_fp16(bias)
    dsc, dsh, dsc2 = kf.upload_f32(scale), kf.upload_f32(shift), kf.upload_f32(scale2)
    ddz, dg = kf.upload_fp16(dz), kf.upload_fp16(gcur)
    dmi = kf.DeviceBuffer(mask_in.nbytes)
    kf.check(kf.core.bridge_transfer_int32(dmi.ptr, mask_in.ctypes.data, mask_in.nbytes // 4), "mask upload")
    aux = kf.DeviceBuffer((T + 2) * BN * 2)
    y = kf.DeviceBuffer(T * DOUT * 2)
    ymask = kf.DeviceBuffer(T * DOUT // 8)
    dbott = kf.DeviceBuffer((T + 2) * BN * 2)
    dxo = kf.DeviceBuffer(T * DIN * 2)
    dzn = kf.DeviceBuffer(T * DIN * 2)
    gWl, gWa, gba = kf.DeviceBuffer(2 * DIN * BN * 4), kf.DeviceBuffer(2 * BN * DOUT * 4), kf.DeviceBuffer(DOUT * 4)

    def fused(M, N, K, a, b, e, what):
        kf.check(kf.core.kf_gemm_fused(M, N, K, C.byref(a), C.byref(b), C.byref(e)), what)

    # ---- forward: linear, then affine with bias / ReLU + mask / BN / bypass
    a = kf.operand(dx_.ptr, DIN, T, 2 * DIN, 1, nparts=2, part_width=DIN, tpolicy=1, dt=(-S, 0))
    b = kf.operand(dwl.ptr, BN, 2 * DIN, BN, 0)
    fused(T, BN, 2 * DIN, a, b, kf.KfEpilogue(out=aux.ptr, ldo=BN, alpha=1.0), "tdnnf linear")
    a2 = kf.operand(aux.ptr, BN, T, 2 * BN, 1, nparts=2, part_width=BN, tpolicy=1, dt=(0, S))
    b2 = kf.operand(dwat.ptr, 2 * BN, DOUT, 2 * BN, 1)
    e2 = kf.KfEpilogue(out=y.ptr, ldo=DOUT, alpha=1.0, bias=db_.ptr, relu=1, mask_out=ymask.ptr, scale=dsc.ptr,
                       shift=dsh.ptr, resid=dx_.ptr, ldr=DIN, resid_alpha=ALPHA)
    fused(T, DOUT, 2 * BN, a2, b2, e2, "tdnnf affine")

    # ---- backward: affine dW / db, affine dX (dbott), linear dW, linear dX
    aw = kf.operand(aux.ptr, BN, T, 2 * BN, 0, nparts=2, part_width=BN, tpolicy=1, dt=(0, S))
    bw = kf.operand(ddz.ptr, DOUT, T, DOUT, 0)
    kf.check(kf.core.kf_gemm_wgrad(2 * BN, DOUT, T, C.byref(aw), C.byref(bw), gWa.ptr, DOUT, gba.ptr, 0),
             "affine wgrad")
    edge_dz = ddz.ptr + T * DOUT * 2
    kf.check(kf.core.kf_rows_sum(edge_dz, ddz.ptr, DOUT, T - 1 - S, T, DOUT), "edge")
    a1 = kf.operand(ddz.ptr, DOUT, T, 2 * DOUT, 1, nparts=2, part_width=DOUT, tpolicy=0, dt=(0, -S),
                    edges=[(1, T - 1, T)])
    b1 = kf.operand(dwa.ptr, DOUT, BN, 2 * DOUT, 1, nparts=2, part_width=DOUT, T=2 * BN, dt=(0, BN))
    fused(T, BN, 2 * DOUT, a1, b1, kf.KfEpilogue(out=dbott.ptr, ldo=BN, alpha=1.0), "affine dgrad")
    al = kf.operand(dx_.ptr, DIN, T, 2 * DIN, 0, nparts=2, part_width=DIN, tpolicy=1, dt=(-S, 0))
    bl = kf.operand(dbott.ptr, BN, T, BN, 0)
    kf.check(kf.core.kf_gemm_wgrad(2 * DIN, BN, T, C.byref(al), C.byref(bl), gWl.ptr, BN, None, 0),
             "linear wgrad")
    edge_db = dbott.ptr + T * BN * 2
    kf.check(kf.core.kf_rows_sum(edge_db, dbott.ptr, BN, 0, S + 1, BN), "edge")
    a3 = kf.operand(dbott.ptr, BN, T, 2 * BN, 1, nparts=2, part_width=BN, tpolicy=0, dt=(S, 0),
                    edges=[(0, 0, T)])
    b3 = kf.operand(dwl.ptr, BN, DIN, 2 * BN, 1, nparts=2, part_width=BN, T=2 * DIN, dt=(0, DIN))
    e3 = kf.KfEpilogue(out=dxo.ptr, ldo=DIN, alpha=1.0, out2=dzn.ptr, ldo2=DIN, scale2=dsc2.ptr,
                       mask_in=dmi.ptr, resid=dg.ptr, ldr=DOUT, resid_alpha=ALPHA)
    fused(T, DIN, 2 * BN, a3, b3, e3, "linear dgrad")
    kf.sync()

    # ---- read back
    g_aux = kf.read_fp16(aux.ptr, (T + 2, BN))[:T]
    g_y = kf.read_fp16(y.ptr, (T, DOUT)).astype(np.float64)
    g_ym = kf.read_fp16(ymask.ptr, (T * DOUT // 16,)).view(np.uint8)
    g_dzfull = kf.read_fp16(ddz.ptr, (T + 2, DOUT))
    g_db = kf.read_fp16(dbott.ptr, (T + 2, BN))
    g_dx = kf.read_fp16(dxo.ptr, (T, DIN)).astype(np.float64)
    g_dzn = kf.read_fp16(dzn.ptr, (T, DIN)).astype(np.float64)
    g_wa = kf.read_f32(gWa.ptr, (2 * BN, DOUT)).astype(np.float64)
    g_ba = kf.read_f32(gba.ptr, (DOUT,)).astype(np.float64)
    g_wl = kf.read_f32(gWl.ptr, (2 * DIN, BN)).astype(np.float64)

    edge = {0, 1, 2, S, S + 1, T - 1, T - 2, T - 1 - S, T - 2 - S}
    rows = np.array(sorted(edge | set(rng.choice(T, 4096, replace=False).tolist())))
    x64 = x[:T]

    # linear forward
    A = splice(x64, rows, (-S, 0))
    ref = A @ w_lin.astype(np.float64)
    tol = 2 * DIN * U23 * (np.abs(A) @ np.abs(w_lin.astype(np.float64))) + np.abs(ref) * 2 ** -10 + 2 ** -24
    _within(g_aux[rows].astype(np.float64), ref, tol, "linear forward")

    # affine forward on the GPU's aux
    A = splice(g_aux, rows, (0, S))
    acc = A @ w_aff.astype(np.float64) + bias.astype(np.float64)
    bound = 2 * BN * U23 * (np.abs(A) @ np.abs(w_aff.astype(np.float64))) + 1e-6 * np.abs(acc)
    pre = np.maximum(acc, 0) * scale + shift
    ref = pre + ALPHA * x64[rows].astype(np.float64)
    tol = bound * scale + np.abs(ref) * 2 ** -10 + 1e-6 * (np.abs(pre) + ALPHA * np.abs(x64[rows])) + 2 ** -24
    _within(g_y[rows], ref, tol, "affine forward")
    bits = _bits(g_ym, rows, DOUT)
    sure = np.abs(acc) > bound
    assert np.array_equal(bits[sure], (acc > 0)[sure]), "affine ReLU mask"

    # affine dX: dbott[r] = dz[r] . W_aff[:BN]^T + (the clamped +S part's transpose)
    dz64 = g_dzfull[:T].astype(np.float64)
    edge_ref = dz64[T - 1 - S:T].sum(0)
    assert np.all(np.abs(g_dzfull[T].astype(np.float64) - edge_ref) <= np.abs(edge_ref) * 2 ** -10 + 1e-6), "dz edge row"
    dzs = np.where((rows - S >= 0)[:, None], dz64[np.clip(rows - S, 0, T - 1)], 0.0)
    dzs[rows == T - 1] = g_dzfull[T].astype(np.float64)
    A = np.concatenate([dz64[rows], dzs], 1)
    Wt = np.concatenate([w_aff[:BN].astype(np.float64).T, w_aff[BN:].astype(np.float64).T], 0)
    ref = A @ Wt
    tol = 2 * DOUT * U23 * (np.abs(A) @ np.abs(Wt)) + np.abs(ref) * 2 ** -10 + 2 ** -24
    _within(g_db[rows].astype(np.float64), ref, tol, "affine dgrad")

    # linear dX with the layer below's epilogue: out = v, out2 = v * scale2 * mask_in
    db64 = g_db[:T].astype(np.float64)
    edge_ref = db64[:S + 1].sum(0)
    assert np.all(np.abs(g_db[T].astype(np.float64) - edge_ref) <= np.abs(edge_ref) * 2 ** -10 + 1e-6), "dbott edge row"
    part0 = np.where((rows + S < T)[:, None], db64[np.clip(rows + S, 0, T - 1)], 0.0)
    part0[rows == 0] = g_db[T].astype(np.float64)
    A = np.concatenate([part0, db64[rows]], 1)
    Wt = np.concatenate([w_lin[:DIN].astype(np.float64).T, w_lin[DIN:].astype(np.float64).T], 0)
    accd = A @ Wt
    bound = 2 * BN * U23 * (np.abs(A) @ np.abs(Wt)) + 1e-6 * np.abs(accd)
    v = accd + ALPHA * gcur[rows].astype(np.float64)
    tol = bound + np.abs(v) * 2 ** -10 + 1e-6 * np.abs(v) + 2 ** -24
    _within(g_dx[rows], v, tol, "linear dgrad out")
    mb = _bits(mask_in, rows, DIN)
    v2 = v * scale2 * mb
    tol2 = (bound + 1e-6 * np.abs(v)) * scale2 + np.abs(v2) * 2 ** -10 + 2 ** -24
    _within(g_dzn[rows], v2, tol2, "linear dgrad out2")

    # weight gradients, every element (split-K, slab reduce, bias sums, part pairing)
    ref, mag = _wgrad_ref(g_aux, (0, S), g_dzfull[:T], 2 * BN, DOUT)
    _within(g_wa, ref, T * U23 * mag + 1e-30, "affine dW")
    bref = dz64.sum(0)
    _within(g_ba, bref, T * U23 * np.abs(dz64).sum(0), "affine db")
    ref, mag = _wgrad_ref(x64, (-S, 0), g_db[:T], 2 * DIN, BN)
    _within(g_wl, ref, T * U23 * mag + 1e-30, "linear dW")


def test_kstep_interleave_matches_part_order(gpu):
    """The K-step interleave (default) and part order give the same product within fp32
    re-association, and both match float64 (kf_gemm_debug_kil)."""
    kf = gpu
    rng = np.random.default_rng(5)
    Tn, d, N, s = 3000, 1536, 160, 3
    x = _h(rng.standard_normal((Tn, d)))
    w = _h(rng.standard_normal((2 * d, N)) / np.sqrt(2 * d))
    dx_, dw = kf.upload_fp16(x), kf.upload_fp16(w)
    outs = []
    for kil in (1, 0):
        kf.core.kf_gemm_debug_kil(kil)
        out = kf.DeviceBuffer(Tn * N * 2)
        a = kf.operand(dx_.ptr, d, Tn, 2 * d, 1, nparts=2, part_width=d, tpolicy=1, dt=(-s, 0))
        b = kf.operand(dw.ptr, N, 2 * d, N, 0)
        e = kf.KfEpilogue(out=out.ptr, ldo=N, alpha=1.0)
        kf.check(kf.core.kf_gemm_fused(Tn, N, 2 * d, C.byref(a), C.byref(b), C.byref(e)), "fused")
        outs.append(kf.read_fp16(out.ptr, (Tn, N)).astype(np.float64))
    kf.core.kf_gemm_debug_kil(1)
    A = splice(x, np.arange(Tn), (-s, 0))
    ref = A @ w.astype(np.float64)
    tol = 2 * d * U23 * (np.abs(A) @ np.abs(w.astype(np.float64))) + np.abs(ref) * 2 ** -10 + 2 ** -24
    for o in outs:
        _within(o, ref, tol, "kil")
    # the two orders differ at most by two fp16 roundings of the same value
    assert np.all(np.abs(outs[0] - outs[1]) <= 2 * tol)


# ---------------------------------------------------------------------------------------
# 3x3 convolutions at the bench's size (conv_halo_kernel forward / input gradient,
# conv_wgrad_halo_kernel with the split count chosen for T = 96,000), operands built as
# host/network.cpp builds them (op_im2col / op_col2im / op_wrows, :1160-1192, :1608-1658),
# with the network's epilogues: forward bias + ReLU + mask + BN scale / shift, input
# gradient into the layer below's dz (BN scale x ReLU mask). Reference semantics:
# internal/nnet/forward.go:418-524 (host im2col + GEMM), network_backward.go:468-537.
OFFS = [(a, b) for a in (-1, 0, 1) for b in (-1, 0, 1)]
# (name, hin, fin, hout, sub, fout): cnn2 (one 64-channel chunk, 512-split wgrad), cnn3
# (height stride 2, per-residue input gradient), cnn5 (two chunks, stride 2)
CONV = [("cnn2", 40, 64, 40, 1, 64), ("cnn3", 40, 64, 20, 2, 128), ("cnn5", 20, 128, 10, 2, 256)]


def _im2col_rows(x3, t, h, sub):
    """[n x 9 fin] im2col rows (t, h) of x3 [T, hin, fin] (zero outside), fp64"""
    Tn, hin, _ = x3.shape
    parts = []
    for dt, dh in OFFS:
        ts, hs = t + dt, h * sub + dh
        ok = (ts >= 0) & (ts < Tn) & (hs >= 0) & (hs < hin)
        parts.append(np.where(ok[:, None], x3[np.clip(ts, 0, Tn - 1), np.clip(hs, 0, hin - 1)].astype(np.float64), 0))
    return np.concatenate(parts, 1)


def _col2im_rows(dz3, W, t, h, sub, fin):
    """input-gradient rows (t, h): sum over taps of dz[t - dt, h'] . W_tap^T, h = h' sub + dh;
    also the bound sum |dz||W|"""
    Tn, hout, _ = dz3.shape
    acc = np.zeros((t.size, fin))
    mag = np.zeros((t.size, fin))
    for o, (dt, dh) in enumerate(OFFS):
        ts, r = t - dt, h - dh
        hp = r // sub
        ok = (ts >= 0) & (ts < Tn) & (r % sub == 0) & (hp >= 0) & (hp < hout)
        d = np.where(ok[:, None], dz3[np.clip(ts, 0, Tn - 1), np.clip(hp, 0, hout - 1)].astype(np.float64), 0)
        Wo = W[o * fin:(o + 1) * fin].astype(np.float64)
        acc += d @ Wo.T
        mag += np.abs(d) @ np.abs(Wo).T
    return acc, mag


@pytest.mark.parametrize("name,hin,fin,hout,sub,fout", CONV)
def test_conv_at_bench_size(gpu, name, hin, fin, hout, sub, fout):
    kf = gpu
    rng = np.random.default_rng(hin * fout)
    K, M = 9 * fin, T * hout
    x = _h(np.maximum(rng.standard_normal((T, hin * fin), dtype=np.float32), -0.5))
    W = _h(rng.standard_normal((K, fout), dtype=np.float32) / np.sqrt(K))
    bias = _h(rng.standard_normal(fout) * 0.1)
    scale = rng.uniform(0.5, 1.5, fout).astype(np.float32)
    shift = (rng.standard_normal(fout) * 0.1).astype(np.float32)
    dz = _h(rng.standard_normal((M, fout), dtype=np.float32) * 0.05)
    scale2 = rng.uniform(0.5, 1.5, fin).astype(np.float32)      # BN scale of the layer below
    mask_in = rng.integers(0, 256, T * hin * fin // 8, dtype=np.uint8)
    dx_, dW, db_, ddz = kf.upload_fp16(x), kf.upload_fp16(W), kf.upload_fp16(bias), kf.upload_fp16(dz)
    dsc, dsh, dsc2 = kf.upload_f32(scale), kf.upload_f32(shift), kf.upload_f32(scale2)
    dmi = kf.DeviceBuffer(mask_in.nbytes)
    kf.check(kf.core.bridge_transfer_int32(dmi.ptr, mask_in.ctypes.data, mask_in.nbytes // 4), "mask upload")
    y, ymask = kf.DeviceBuffer(M * fout * 2), kf.DeviceBuffer(M * fout // 8)
    gx = kf.DeviceBuffer(T * hin * fin * 2)
    gW, gb = kf.DeviceBuffer(K * fout * 4), kf.DeviceBuffer(fout * 4)

    # forward: op_im2col (k-contiguous), plain weights, the conv layer's epilogue
    a = kf.operand(dx_.ptr, hin * fin, M, K, 1, nparts=9, part_width=fin, T=T, hout=hout, hsrc=hin,
                   hmul=sub, hdiv=1, tpolicy=0, dt=[o[0] for o in OFFS], dh=[o[1] for o in OFFS])
    b = kf.operand(dW.ptr, fout, K, fout, 0)
    e = kf.KfEpilogue(out=y.ptr, ldo=fout, alpha=1.0, bias=db_.ptr, relu=1, mask_out=ymask.ptr, scale=dsc.ptr,
                      shift=dsh.ptr)
    kf.check(kf.core.kf_gemm_fused(M, fout, K, C.byref(a), C.byref(b), C.byref(e)), name + " forward")
    # input gradient: op_col2im with op_wrows, out2 = v * scale2 * mask (the layer below's dz)
    if sub == 1:
        a2 = kf.operand(ddz.ptr, hout * fout, T * hin, 9 * fout, 1, nparts=9, part_width=fout, T=T, hout=hin,
                        hsrc=hout, hmul=1, hdiv=1, tpolicy=0, dt=[-o[0] for o in OFFS], dh=[-o[1] for o in OFFS])
        b2 = kf.operand(dW.ptr, fout, fin, 9 * fout, 1, nparts=9, part_width=fout, T=K,
                        dt=[p * fin for p in range(9)])
        e2 = kf.KfEpilogue(out2=gx.ptr, ldo2=fin, scale2=dsc2.ptr, mask_in=dmi.ptr, alpha=1.0)
        kf.check(kf.core.kf_gemm_fused(T * hin, fin, 9 * fout, C.byref(a2), C.byref(b2), C.byref(e2)),
                 name + " dgrad")
    else:
        for pi in range(sub):   # one GEMM per input-height residue (network.cpp:1620-1650)
            taps = [(o, dt, (pi - dh) // sub) for o, (dt, dh) in enumerate(OFFS) if (pi - dh) % sub == 0]
            n = len(taps)
            a2 = kf.operand(ddz.ptr, hout * fout, T * (hin // sub), n * fout, 1, nparts=n, part_width=fout, T=T,
                            hout=hin // sub, hsrc=hout, hmul=1, hdiv=1, tpolicy=0,
                            dt=[-tp[1] for tp in taps], dh=[tp[2] for tp in taps])
            b2 = kf.operand(dW.ptr, fout, fin, n * fout, 1, nparts=n, part_width=fout, T=K,
                            dt=[tp[0] * fin for tp in taps])
            e2 = kf.KfEpilogue(out2=gx.ptr + pi * fin * 2, ldo2=sub * fin, scale2=dsc2.ptr,
                               mask_in=dmi.ptr + pi * fin // 8, alpha=1.0)
            kf.check(kf.core.kf_gemm_fused(T * (hin // sub), fin, n * fout, C.byref(a2), C.byref(b2), C.byref(e2)),
                     name + " dgrad residue %d" % pi)
    # weight gradient: op_im2col reduction-major, split-K over the 3.84 M / 1.92 M / 0.96 M rows
    aw = kf.operand(dx_.ptr, hin * fin, M, K, 0, nparts=9, part_width=fin, T=T, hout=hout, hsrc=hin,
                    hmul=sub, hdiv=1, tpolicy=0, dt=[o[0] for o in OFFS], dh=[o[1] for o in OFFS])
    bw = kf.operand(ddz.ptr, fout, M, fout, 0)
    kf.check(kf.core.kf_gemm_wgrad(K, fout, M, C.byref(aw), C.byref(bw), gW.ptr, fout, gb.ptr, 0), name + " wgrad")
    kf.sync()

    x3 = x.reshape(T, hin, fin)
    edge_t = [0, 1, T - 2, T - 1, 1499, 1500]
    # forward on 4,096 sampled output rows plus the edge frames / heights
    ts = np.concatenate([rng.integers(0, T, 4096), np.repeat(edge_t, 2)])
    hs = np.concatenate([rng.integers(0, hout, 4096), np.tile([0, hout - 1], len(edge_t))])
    P = _im2col_rows(x3, ts, hs, sub)
    acc = P @ W.astype(np.float64) + bias.astype(np.float64)
    bound = K * U23 * (np.abs(P) @ np.abs(W.astype(np.float64))) + 1e-6 * np.abs(acc)
    ref = np.maximum(acc, 0) * scale + shift
    rows = ts * hout + hs
    g_y = kf.read_fp16(y.ptr, (M, fout))[rows].astype(np.float64)
    _within(g_y, ref, bound * scale + np.abs(ref) * 2 ** -10 + 1e-6 * np.abs(ref) + 2 ** -24, name + " forward")
    mbits = _bits(kf.read_fp16(ymask.ptr, (M * fout // 16,)).view(np.uint8), rows, fout)
    sure = np.abs(acc) > bound
    assert np.array_equal(mbits[sure], (acc > 0)[sure]), name + " ReLU mask"
    # input gradient on 4,096 sampled input rows plus the edges
    ts = np.concatenate([rng.integers(0, T, 4096), np.repeat(edge_t, 2)])
    hs = np.concatenate([rng.integers(0, hin, 4096), np.tile([0, hin - 1], len(edge_t))])
    v, mag = _col2im_rows(dz.reshape(T, hout, fout), W, ts, hs, sub, fin)
    rows = ts * hin + hs
    mb = _bits(mask_in, rows, fin)
    v2 = v * scale2 * mb
    tol2 = (9 * fout * U23 * mag + 1e-6 * np.abs(v)) * scale2 + np.abs(v2) * 2 ** -10 + 2 ** -24
    g_x = kf.read_fp16(gx.ptr, (T * hin, fin))[rows].astype(np.float64)
    _within(g_x, v2, tol2, name + " dgrad")
    # weight gradient and bias sums, every element, blockwise fp64 P^T dZ
    refw = np.zeros((K, fout))
    magw = np.zeros((K, fout))
    dz3 = dz.reshape(T, hout, fout)
    for t0 in range(0, T, 2000):
        tt = np.repeat(np.arange(t0, min(T, t0 + 2000)), hout)
        hh = np.tile(np.arange(hout), tt.size // hout)
        Pb = _im2col_rows(x3, tt, hh, sub)
        Db = dz3[tt, hh].astype(np.float64)
        refw += Pb.T @ Db
        magw += np.abs(Pb).T @ np.abs(Db)
    _within(kf.read_f32(gW.ptr, (K, fout)).astype(np.float64), refw, M * U23 * magw * 1.01 + 1e-30, name + " dW")
    dz64 = dz.astype(np.float64)
    _within(kf.read_f32(gb.ptr, (fout,)).astype(np.float64), dz64.sum(0), M * U23 * np.abs(dz64).sum(0) * 1.01,
            name + " db")
