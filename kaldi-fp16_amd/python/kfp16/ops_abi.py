"""ctypes signatures of the reference's per-op C-ABI as the Go ``internal/gpu``
package binds it (internal/gpu/ops.go:21-366, backward_ops.go, bridge.go):

- ``ops_*``       include/ops.h   (cpp/include/ops.h:16-188; ops.cu, backward_wrappers.cu)
- ``bridge_batch_*`` / ``bridge_host_*`` include/bridge.h (cpp/include/bridge.h:13-60)
- ``chain_*_det`` / ``chain_workspace_bytes`` include/chain.h (chain_det.cu:293-477)

Only signatures live here; every call runs the HIP kernels in libkaldi_fp16.so.
"""
import ctypes as C

from . import core
from .chain import ChainFstGPU

_vp, _i, _f, _sz, _i64 = C.c_void_p, C.c_int, C.c_float, C.c_size_t, C.c_int64
_fp = C.POINTER(C.c_float)


class GPUBatchPtrs(C.Structure):
    """bridge.h:34-50 (byte-identical to the reference's struct)."""
    _fields_ = [("d_features", _vp), ("d_ivectors", _vp), ("d_csr_row_ptr", _vp),
                ("d_csr_col_idx", _vp), ("d_csr_labels", _vp), ("d_csr_weights", _vp),
                ("d_buffer", _vp), ("total_bytes", _sz),
                ("features_bytes", _sz), ("ivectors_bytes", _sz), ("csr_rowptr_bytes", _sz),
                ("csr_colidx_bytes", _sz), ("csr_labels_bytes", _sz), ("csr_weights_bytes", _sz)]


def _sig(name, res, *args):
    fn = getattr(core, name)
    fn.restype = res
    fn.argtypes = list(args)
    return fn


_pfst = C.POINTER(ChainFstGPU)
for _name, _res, _args in [
    # ops.h: activations, softmax, batchnorm, element-wise, layout
    ("ops_relu", _i, (_vp, _i)),
    ("ops_sigmoid", _i, (_vp, _i)),
    ("ops_tanh_act", _i, (_vp, _i)),
    ("ops_clipped_relu", _i, (_vp, _i, _f)),
    ("ops_softmax", _i, (_vp, _i, _i)),
    ("ops_log_softmax", _i, (_vp, _i, _i)),
    ("ops_batchnorm_forward", _i, (_vp, _i, _i, _vp, _vp, _vp, _vp, _f)),
    ("ops_batchnorm_forward_rms", _i, (_vp, _i, _i, _vp, _vp, _f, _f)),
    ("ops_add_scaled", _i, (_vp, _vp, _i, _f, _f)),
    ("ops_add", _i, (_vp, _vp, _i)),
    ("ops_copy", _i, (_vp, _vp, _i)),
    ("ops_fill", _i, (_vp, _i, _f)),
    ("ops_concat_cols", _i, (_vp, _i, _i, _vp, _i, _i)),
    ("ops_slice_cols", _i, (_vp, _i, _i, _vp, _i, _i)),
    ("ops_combine_feature_maps", _i, (_vp, _i, _i, _i, _i, _i)),
    ("ops_subsample_rows", None, (_vp, _vp, _i, _i, _i, _i)),
    ("ops_gemm_strided", _i, (_vp, _i, _i, _i, _f, _vp, _i, _i64, _vp, _i, _i64, _f, _vp, _i,
                              _i64, _i)),
    ("ops_clear_error", None, ()),
    # ops.h: backward element-wise and optimiser pieces
    ("ops_relu_backward", _i, (_vp, _vp, _i)),
    ("ops_sigmoid_backward", _i, (_vp, _vp, _i)),
    ("ops_tanh_backward", _i, (_vp, _vp, _i)),
    ("ops_transpose", _i, (_vp, _vp, _i, _i)),
    ("ops_batchnorm_backward", _i, (_vp, _vp, _vp, _vp, _f, _i, _i)),
    ("ops_fp16_to_fp32", _i, (_vp, _vp, _i)),
    ("ops_sgd_update", _i, (_vp, _vp, _vp, _vp, _f, _f, _i)),
    # bridge.h: pinned host memory and the one-allocation minibatch buffer
    ("bridge_host_alloc", _vp, (_sz,)),
    ("bridge_host_free", None, (_vp,)),
    ("bridge_batch_alloc", _i, (_i, _i, _i, _i, _i, _i, C.POINTER(GPUBatchPtrs))),
    ("bridge_batch_transfer", _i, (C.POINTER(GPUBatchPtrs), _vp, _sz)),
    ("bridge_batch_free", None, (C.POINTER(GPUBatchPtrs),)),
    # chain.h: deterministic entry points
    ("chain_forward_backward_det", _i, (_vp, _pfst, _i, _i, _vp, _vp, _fp)),
    ("chain_compute_posteriors_det", _i, (_vp, _pfst, _i, _i, _vp, _vp, _f, _vp)),
    ("chain_num_forward_backward_det", _f, (_vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp, _vp,
                                            _i, _i, _vp)),
    ("chain_workspace_bytes", _sz, (_i, _i)),
]:
    _sig(_name, _res, *_args)
