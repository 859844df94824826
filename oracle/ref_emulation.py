"""Reference-emulation mode of the oracle: the reference's OWN formulation of the
conv-relu-batchnorm layer, internal/nnet/forward.go:418-524, restated literally.

TEST INFRASTRUCTURE ONLY (same rule as kf_oracle.h): only tests/ load this.

The MI355X build (and the C oracle, kf_oracle.c) implement Kaldi's conv semantics:
the time x height cross product of offsets and a height-major output [t][h*F + f].
The reference differs in two places, and this module reproduces both so the
difference can be measured instead of asserted:

1. zipped offsets (forward.go:438-446): offset i is the PAIR (time_offsets[i],
   height_offsets[i]), numOffsets = len(time_offsets); patch column off*nfIn + f;
   weights W [nfIn*numOffsets x nfOut];
2. filter-major reorder (forward.go:495-509): after GEMM, bias and ReLU, output
   column f*heightOut + h (Kaldi: h*nfOut + f); BatchNorm (ops.cu:171-204) then runs
   on those columns.

The input is read height-major (forward.go:443-448: tSrc*(heightIn*nfIn) +
hSrc*nfIn + f) whatever layout the producing layer wrote; out-of-range taps
(time or height) contribute zero. Arithmetic is fp32 with fp32 accumulation
(GEMMSimple -> cublasGemmEx, ops.cu:381-392) and the reference's rounding points
when round16 is set: the patches are uploaded as fp16 (TensorFromFP32), the GEMM
output, the bias add, the ReLU and the BN each store fp16.
"""
import numpy as np


def _r16(a, on):
    return a.astype(np.float16).astype(np.float32) if on else a.astype(np.float32)


def zipped_offsets(time_offsets, height_offsets):
    """forward.go:438-446 pairs offset i of each list"""
    assert len(time_offsets) == len(height_offsets)
    return list(zip(time_offsets, height_offsets))


def im2col_ref(x, T, height_in, nf_in, height_out, subsample, offsets):
    """forward.go:435-456: patches [T*heightOut x numOffsets*nfIn]"""
    x = np.asarray(x, np.float32).reshape(T, height_in * nf_in)
    n = len(offsets)
    p = np.zeros((T * height_out, n * nf_in), np.float32)
    for t in range(T):
        for h in range(height_out):
            row = t * height_out + h
            for off, (to, ho) in enumerate(offsets):
                ts, hs = t + to, h * subsample + ho
                if 0 <= ts < T and 0 <= hs < height_in:
                    p[row, off * nf_in:(off + 1) * nf_in] = x[ts, hs * nf_in:(hs + 1) * nf_in]
    return p


def conv_relu_bn_ref(x, T, height_in, nf_in, height_out, subsample, time_offsets, height_offsets,
                     W, bias, bn=None, round16=True):
    """forward.go:418-524 end to end. W [nfIn*numOffsets x nfOut]; bn = (mean, var,
    gamma, beta, eps) indexed by OUTPUT COLUMN of the filter-major layout (the
    reference's BN params have heightOut*nfOut entries, allocWeights)."""
    offs = zipped_offsets(time_offsets, height_offsets)
    p = _r16(im2col_ref(x, T, height_in, nf_in, height_out, subsample, offs), round16)
    # GEMM(h, A.Rows, B.Cols, A.Cols, ...) (internal/gpu/ops.go:72) contracts over
    # K = patchDim = numOffsets*nfIn and reads W row-major with ldb = nfOut, so a W with
    # more rows (a Kaldi cross-product matrix from weight_loader.go:129-163) contributes
    # its first patchDim rows only
    Wf = np.asarray(W, np.float32)[:p.shape[1]]
    y = _r16(p.astype(np.float64) @ Wf.astype(np.float64), round16)
    nf_out = Wf.shape[1]
    if bias is not None:
        y = _r16(y + np.asarray(bias, np.float32)[None, :], round16)
    y = _r16(np.maximum(y, 0), round16)
    # filter-major reorder: dst[t][f*heightOut + h] = src[t*heightOut + h][f]
    out = y.reshape(T, height_out, nf_out).transpose(0, 2, 1).reshape(T, nf_out * height_out)
    if bn is not None:
        mean, var, gamma, beta, eps = bn
        out = (out - mean) / np.sqrt(np.asarray(var, np.float32) + np.float32(eps)) * gamma + beta
        out = _r16(out, round16)
    return out


def cross_weights_from_zipped(W_zip, nf_in, time_offsets, height_offsets):
    """Kaldi-layout (cross-product) weights [nt*nh*nfIn x nfOut] that compute the
    reference's zipped conv: tap (time_offsets[i], height_offsets[i]) carries W_zip's
    block i, every other tap is zero. Cross-product tap order is time-major
    (tests' oracle.py / host/xconfig.cpp: o = ti*nh + hi)."""
    nt, nh = len(time_offsets), len(height_offsets)
    W_zip = np.asarray(W_zip, np.float32)
    out = np.zeros((nt * nh * nf_in, W_zip.shape[1]), np.float32)
    for i in range(len(time_offsets)):
        o = i * nh + i
        out[o * nf_in:(o + 1) * nf_in] = W_zip[i * nf_in:(i + 1) * nf_in]
    return out


def filter_major_to_height_major(y, T, height, nf):
    """column f*H + h -> h*F + f"""
    return np.asarray(y).reshape(T, nf, height).transpose(0, 2, 1).reshape(T, height * nf)


def height_major_to_filter_major(y, T, height, nf):
    return np.asarray(y).reshape(T, height, nf).transpose(0, 2, 1).reshape(T, nf * height)
