"""The fused epilogue's edge-row sum (KfEpilogue.edge_out, include/kf_ops.h): the row tile
holding rows [edge_r0, edge_r1) writes their column sums (of the stored out or out2 values)
into edge_out, bit-identical to kf_rows_sum over the stored tensor, which it replaces in the
TDNN-F backward (host/network.cpp: the clamped-splice edge rows of dz and of the bottleneck
gradient, internal/nnet/forward.go:699-790 spliceBackward). A range that spans two row tiles
takes the launch's kf_rows_sum fallback."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _h(a):
    return np.ascontiguousarray(a, np.float16)


@pytest.mark.parametrize("T,N,K,r0,r1,src", [
    (3000, 1536, 320, 2996, 3000, 1),   # dz edge: last tile, out2 (BN scale x mask applied)
    (3000, 160, 3072, 0, 4, 0),         # dbott edge: first tile, out
    (3000, 1536, 320, 120, 136, 1),     # spans the 128-row tiles: the kf_rows_sum fallback
    (517, 256, 128, 513, 517, 0),
])
def test_epilogue_edge_matches_rows_sum(gpu, T, N, K, r0, r1, src):
    kf = gpu
    rng = np.random.default_rng(T + N + r0)
    a = _h(rng.standard_normal((T + 2, K)) * 0.5)
    w = _h(rng.standard_normal((N, K)) / np.sqrt(K))
    sc = rng.uniform(0.5, 1.5, N).astype(np.float32)
    mk = rng.integers(0, 256, T * N // 8, dtype=np.uint8)
    da, dw, dsc = kf.upload_fp16(a), kf.upload_fp16(w), kf.upload_f32(sc)
    dmk = kf.DeviceBuffer(mk.nbytes)
    kf.check(kf.core.bridge_transfer_int32(dmk.ptr, mk.ctypes.data, mk.nbytes // 4), "mask")
    out, out2 = kf.DeviceBuffer((T + 2) * N * 2), kf.DeviceBuffer((T + 2) * N * 2)
    ref_edge = kf.DeviceBuffer(N * 2)
    A = kf.operand(da.ptr, K, T, K, 1)
    B = kf.operand(dw.ptr, K, N, K, 1)
    tgt = (out if src == 0 else out2).ptr
    E = kf.KfEpilogue(out=out.ptr, ldo=N, alpha=1.0, out2=out2.ptr, ldo2=N, scale2=dsc.ptr, mask_in=dmk.ptr,
                      edge_out=tgt + T * N * 2, edge_r0=r0, edge_r1=r1, edge_src=src)
    kf.check(kf.core.kf_gemm_fused(T, N, K, C.byref(A), C.byref(B), C.byref(E)), "gemm + edge")
    kf.check(kf.core.kf_rows_sum(ref_edge.ptr, tgt, N, r0, r1, N), "rows_sum")
    kf.sync()
    got = kf.read_fp16(tgt + T * N * 2, (N,))
    ref = kf.read_fp16(ref_edge.ptr, (N,))
    assert np.array_equal(got.view(np.uint16), ref.view(np.uint16))
