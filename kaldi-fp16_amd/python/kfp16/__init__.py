"""kfp16 — Python binding of the MI355X kaldi-fp16 core.

Thin ctypes layer over the C-ABI libraries built in ``kaldi-fp16_amd/lib``:
``libkaldi_fp16.so`` (bridge_* / ops_* / chain_* / den_* / kf_* kernels) and
``libkaldi_fp16_nnet.so`` (the C++ host layer restating internal/nnet).
Tests and bench.py drive the product through this module; nothing here
computes anything itself. If the HIP libraries are missing, importing this
module raises — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# KFP16_LIBDIR: load another in-tree build (A/B timing of kernel variants)
LIBDIR = os.environ.get("KFP16_LIBDIR") or os.path.normpath(os.path.join(_HERE, "..", "..", "lib"))
INCDIR = os.path.normpath(os.path.join(_HERE, "..", "..", "..", "include"))


class KfError(RuntimeError):
    pass


def _load(name):
    path = os.path.join(LIBDIR, name)
    if not os.path.exists(path):
        raise ImportError(
            f"kfp16: {path} is missing — build the HIP libraries first "
            "(python -c 'import __graft_entry__ as g; g.build()'); there is no CPU fallback")
    if os.environ.get("KF_ERR_TRACE", "0") not in ("", "0"):
        return _TracedCDLL(path, mode=C.RTLD_GLOBAL)
    return C.CDLL(path, mode=C.RTLD_GLOBAL)


# KF_ERR_TRACE=1: origin of a HIP error left pending. Every call through the
# libraries peeks at HIP's pending error (kf_peek_error, not consumed) before and after it:
# one pending before the call was raised by HIP calls the process made outside kfp16 since
# its previous call (torch, ctypes users); one pending after it by the call itself. Notes
# go to stderr and to trace_notes; the libraries' own kf_take_pending checks are unchanged.
trace_notes: list = []


def _trace_note(msg):
    import sys
    import traceback
    where = "".join(traceback.format_stack(limit=5)[:-2]).rstrip()
    trace_notes.append(msg + "\n" + where)
    print(f"kfp16 KF_ERR_TRACE: {msg}\n{where}", file=sys.stderr, flush=True)


class _TracedCDLL(C.CDLL):
    def __init__(self, path, mode):
        super().__init__(path, mode=mode)
        peek = C.CDLL(os.path.join(LIBDIR, "libkaldi_fp16.so"), mode=mode).kf_peek_error
        peek.restype, peek.argtypes = C.c_int, []
        base = self._FuncPtr

        class _Traced(base):
            _flags_ = base._flags_
            _restype_ = base._restype_

            def __call__(self, *args):
                pre = peek()
                if pre:
                    _trace_note(f"HIP error {pre} pending before {self.__name__} "
                                "(raised outside kfp16 since its previous call)")
                r = base.__call__(self, *args)
                post = peek()
                if post and post != pre:
                    _trace_note(f"HIP error {post} pending after {self.__name__}")
                return r

        self._FuncPtr = _Traced


core = _load("libkaldi_fp16.so")
nnet = _load("libkaldi_fp16_nnet.so")

_vp, _i, _f, _ll, _sz = C.c_void_p, C.c_int, C.c_float, C.c_longlong, C.c_size_t


def _sig(lib, name, res, *args):
    if os.environ.get("KFP16_LIBDIR") and not hasattr(lib, name):
        return None  # A/B against an older build that lacks this entry point
    fn = getattr(lib, name)
    fn.restype = res
    fn.argtypes = list(args)
    return fn


# ---------------------------------------------------------------- bridge_*
for _n in ("bridge_last_error", "ops_last_error", "kf_last_error", "nnet_last_error"):
    _sig(core if not _n.startswith("nnet") else nnet, _n, C.c_char_p)
_sig(core, "bridge_clear_error", None)
_sig(core, "kf_take_pending", _i, C.c_char_p)
_sig(core, "kf_pending_log", C.c_char_p)
_sig(core, "kf_pending_clear", None)
_sig(core, "kf_peek_error", _i)
_sig(core, "bridge_gpu_init", _i, _i)
_sig(core, "bridge_gpu_sync", _i)
_sig(core, "bridge_gpu_get_free_memory", _i, C.POINTER(_sz), C.POINTER(_sz))
_sig(core, "bridge_gpu_malloc", _vp, _sz)
_sig(core, "bridge_gpu_free", None, _vp)
_sig(core, "bridge_transfer_fp16", _i, _vp, _vp, _sz)
_sig(core, "bridge_read_fp16", _i, _vp, _vp, _sz)
_sig(core, "bridge_transfer_int32", _i, _vp, _vp, _sz)
_sig(core, "bridge_transfer_float32", _i, _vp, _vp, _sz)
_sig(core, "bridge_read_float32", _i, _vp, _vp, _sz)
_sig(core, "bridge_gpu_memset", None, _vp, _i, _sz)
_sig(core, "bridge_fp16_to_fp32_gpu", _i, _vp, _vp, _sz)
_sig(core, "bridge_fp32_to_fp16_gpu", _i, _vp, _vp, _sz)
_sig(core, "kf_set_stream", None, _vp)
_sig(core, "kf_get_stream", _vp)
_sig(core, "ops_gemm", _i, _vp, _i, _i, _i, _f, _vp, _i, _vp, _i, _f, _vp, _i)
_sig(core, "ops_cublas_create", _vp)
_sig(core, "ops_cublas_destroy", None, _vp)
_sig(core, "ops_log_softmax", _i, _vp, _i, _i)

# ---------------------------------------------------------------- nnet_*
_sig(nnet, "nnet_create", _vp, C.c_char_p, _i)
_sig(nnet, "nnet_free", None, _vp)
_sig(nnet, "nnet_parse_summary", _i, C.c_char_p, C.c_char_p, _i)
_sig(nnet, "nnet_num_layers", _i, _vp)
_sig(nnet, "nnet_layer_info", _i, _vp, _i, C.c_char_p, _i, C.POINTER(_i), C.POINTER(_i), C.POINTER(_i))
_sig(nnet, "nnet_num_params", _ll, _vp)
_sig(nnet, "nnet_num_param_tensors", _i, _vp)
_sig(nnet, "nnet_param_info", _i, _vp, _i, C.c_char_p, _i, C.POINTER(_i), C.POINTER(_i), C.POINTER(_ll))
_sig(nnet, "nnet_set_params", _i, _vp, _vp)
_sig(nnet, "nnet_get_params", _i, _vp, _vp)
_sig(nnet, "nnet_set_bn", _i, _vp, C.c_char_p, _i, _vp, _vp, _vp, _vp, _f, _f)
_sig(nnet, "nnet_forward", _i, _vp, _vp, _i)
_sig(nnet, "nnet_forward_ivector", _i, _vp, _vp, _i, _vp, _i, _vp)
_sig(nnet, "nnet_activation", _vp, _vp, C.c_char_p, C.POINTER(_i), C.POINTER(_i))
_sig(nnet, "nnet_backward", _i, _vp, _vp)
_sig(nnet, "nnet_grad_buffer", _vp, _vp)
_sig(nnet, "nnet_master_buffer", _vp, _vp)
_sig(nnet, "nnet_weight_buffer", _vp, _vp)
_sig(nnet, "nnet_sgd", _i, _vp, _f, _f)
_sig(nnet, "nnet_set_fp8", _i, _vp, _i)
_sig(nnet, "nnet_bind_grad_buffer", _i, _vp, _vp)
_sig(nnet, "nnet_backward_n", _i, _vp, _vp, _i)
_sig(nnet, "nnet_debug_tensor", _vp, _vp, C.c_char_p, _i)
_sig(nnet, "nnet_create_layout", _vp, C.c_char_p, _i)
_sig(nnet, "nnet_bind_dp", _i, _vp, _vp, _ll)
_sig(nnet, "nnet_dp_plan", _i, _vp, _ll, _i, C.POINTER(_i), C.POINTER(_ll), C.POINTER(_ll))
_sig(nnet, "nnet_dp_debug_early", _i, _vp, _i)
_sig(nnet, "nnet_set_wgrad_stream", _i, _vp, _i)
_sig(nnet, "nnet_set_implicit_dz", _i, _vp, _i)
_sig(nnet, "nnet_set_row_subsampling", _i, _vp, _i)
_sig(nnet, "nnet_row_set", _i, _vp, C.POINTER(_i), C.POINTER(_i))
_sig(nnet, "nnet_debug_backward", _i, _vp, _i, _ll)
_sig(core, "kf_debug_spin", _i, _vp, _ll)
_sig(nnet, "nnet_weights_changed", _i, _vp)
# kf_dp.h (RCCL data parallel)
_sig(core, "kf_dp_last_error", C.c_char_p)
_sig(core, "kf_dp_unique_id", _i, C.c_char_p)
_sig(core, "kf_dp_create", _vp, _i, _i, C.c_char_p, _i)
_sig(core, "kf_dp_free", None, _vp)
_sig(core, "kf_dp_rank", _i, _vp)
_sig(core, "kf_dp_world", _i, _vp)
_sig(core, "kf_dp_allreduce_mean_async", _i, _vp, _vp, _sz)
_sig(core, "kf_dp_join", _i, _vp)
_sig(core, "kf_dp_allreduce_mean", _i, _vp, _vp, _sz)
_sig(core, "kf_dp_allreduce_sum_f64", _i, _vp, _vp, _sz)
_sig(core, "kf_dp_stats", _i, _vp, C.POINTER(_ll), C.POINTER(_ll))
_sig(core, "kf_dp_debug", _i, _vp, _i, _vp, _vp, C.c_size_t)
_sig(core, "kf_dp_plan", _i, _i, C.POINTER(_ll), C.POINTER(_ll), _ll, _ll, _i, C.POINTER(_i),
     C.POINTER(_ll), C.POINTER(_ll))
_sig(core, "kf_prof_enable", None, _i)
_sig(core, "kf_prof_reserve", _i, _i)
_sig(core, "kf_prof_collect", _i, _i, C.POINTER(_ll), C.POINTER(C.c_double), C.POINTER(C.c_double))
_sig(core, "kf_prof_reset", None)
_sig(core, "kf_prof_records", _i, _i, C.POINTER(_i), C.POINTER(C.c_float), C.POINTER(C.c_double), C.POINTER(_i))
_sig(core, "kf_prof_collect2", _i, _i, C.POINTER(_ll), C.POINTER(C.c_double), C.POINTER(C.c_double),
     C.POINTER(C.c_double))


def _err(lib_fn):
    s = lib_fn()
    return s.decode() if s else "unknown error"


def check(rc, what="kfp16"):
    if rc != 0:
        msgs = [m for m in (core.kf_last_error(), core.ops_last_error(), core.bridge_last_error(),
                            nnet.nnet_last_error()) if m]
        stale = core.kf_pending_log()
        if stale:   # errors other HIP calls left pending, consumed by the library's entry checks
            msgs.append(b"[" + stale + b"]")
        raise KfError(f"{what}: " + "; ".join(m.decode() for m in msgs))


def pending_log():
    """kf_pending_log(): errors earlier HIP calls left pending, consumed and logged by the
    library's entry points (kf_take_pending), or None."""
    s = core.kf_pending_log()
    return s.decode() if s else None


# ---------------------------------------------------------------- device buffers
class DeviceBuffer:
    """Owning device allocation made through bridge_gpu_malloc."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        self.ptr = core.bridge_gpu_malloc(max(self.nbytes, 16))
        if not self.ptr:
            raise KfError("bridge_gpu_malloc: " + _err(core.bridge_last_error))

    def free(self):
        if self.ptr:
            core.bridge_gpu_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def upload_fp16(arr: np.ndarray) -> DeviceBuffer:
    a = np.ascontiguousarray(arr, dtype=np.float16)
    buf = DeviceBuffer(a.nbytes)
    check(core.bridge_transfer_fp16(buf.ptr, a.ctypes.data, a.size), "upload_fp16")
    buf.shape = a.shape
    return buf


def upload_f32(arr: np.ndarray) -> DeviceBuffer:
    a = np.ascontiguousarray(arr, dtype=np.float32)
    buf = DeviceBuffer(a.nbytes)
    check(core.bridge_transfer_float32(buf.ptr, a.ctypes.data, a.size), "upload_f32")
    buf.shape = a.shape
    return buf


def read_fp16(ptr, shape) -> np.ndarray:
    out = np.empty(shape, dtype=np.float16)
    check(core.bridge_read_fp16(out.ctypes.data, ptr, out.size), "read_fp16")
    return out


def read_f32(ptr, shape) -> np.ndarray:
    out = np.empty(shape, dtype=np.float32)
    check(core.bridge_read_float32(out.ctypes.data, ptr, out.size), "read_f32")
    return out


def hip_runtimes():
    """Paths of every HIP runtime mapped into this process (must be exactly one:
    import torch BEFORE kfp16 when both are used, so both bind torch's copy)."""
    with open("/proc/self/maps") as f:
        return sorted({l.split()[-1] for l in f if "libamdhip64" in l})


def assert_single_hip_runtime():
    libs = hip_runtimes()
    if len(libs) > 1:
        raise KfError(f"two HIP runtimes loaded {libs}: import torch before kfp16")


def prof_collect(cls: int):
    n, ms, fl = _ll(), C.c_double(), C.c_double()
    core.kf_prof_collect(cls, C.byref(n), C.byref(ms), C.byref(fl))
    return n.value, ms.value, fl.value


def prof_collect2(cls: int):
    """(launches, ms, algorithmic flops, algorithmic HBM bytes) of a kernel class"""
    n, ms, fl, by = _ll(), C.c_double(), C.c_double(), C.c_double()
    core.kf_prof_collect2(cls, C.byref(n), C.byref(ms), C.byref(fl), C.byref(by))
    return n.value, ms.value, fl.value, by.value


def prof_records(max_n: int = 4096):
    """every kf_prof record since the last reset, in issue order: dicts of class, ms,
    flops, M, N, K and tile (BM * 10000 + BN; 0 for brackets that are not one GEMM)"""
    cls = (C.c_int * max_n)()
    ms = (C.c_float * max_n)()
    fl = (C.c_double * max_n)()
    mnkt = (C.c_int * (4 * max_n))()
    n = core.kf_prof_records(max_n, cls, ms, fl, mnkt)
    return [dict(cls=cls[i], ms=ms[i], flops=fl[i], M=mnkt[4 * i], N=mnkt[4 * i + 1], K=mnkt[4 * i + 2],
                 tile=mnkt[4 * i + 3]) for i in range(n)]


def set_stream(stream_handle) -> None:
    core.kf_set_stream(C.c_void_p(stream_handle) if stream_handle else None)


def sync() -> None:
    check(core.bridge_gpu_sync(), "sync")


# ---------------------------------------------------------------- network
class Network:
    """internal/nnet Network (forward.go:15-21) behind the nnet_* C-ABI."""

    def __init__(self, xconfig: str, max_frames: int, layout_only: bool = False):
        """layout_only: nnet_create_layout — no device storage, no GPU needed (layer,
        parameter and data-parallel bucket queries only)."""
        create = nnet.nnet_create_layout if layout_only else nnet.nnet_create
        self.h = create(xconfig.encode(), int(max_frames))
        if not self.h:
            raise KfError("nnet_create: " + _err(nnet.nnet_last_error))
        self.max_frames = int(max_frames)
        self.layers = []
        name = C.create_string_buffer(256)
        ty, di, do = _i(), _i(), _i()
        for i in range(nnet.nnet_num_layers(self.h)):
            nnet.nnet_layer_info(self.h, i, name, 256, C.byref(ty), C.byref(di), C.byref(do))
            self.layers.append((name.value.decode(), ty.value, di.value, do.value))
        self.num_params = nnet.nnet_num_params(self.h)
        self.params = {}
        r, c, off = _i(), _i(), _ll()
        for i in range(nnet.nnet_num_param_tensors(self.h)):
            nnet.nnet_param_info(self.h, i, name, 256, C.byref(r), C.byref(c), C.byref(off))
            self.params[name.value.decode()] = (r.value, c.value, off.value)
        self.T = 0

    def close(self):
        if getattr(self, "h", None):
            nnet.nnet_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # parameters --------------------------------------------------------
    def flat_params(self, named: dict) -> np.ndarray:
        flat = np.zeros(self.num_params, dtype=np.float32)
        for k, (r, c, off) in self.params.items():
            flat[off:off + r * c] = np.asarray(named[k], dtype=np.float32).reshape(-1)
        return flat

    def unflatten(self, flat: np.ndarray) -> dict:
        return {k: flat[off:off + r * c].reshape(r, c) for k, (r, c, off) in self.params.items()}

    def set_params(self, named: dict):
        flat = self.flat_params(named)
        check(nnet.nnet_set_params(self.h, flat.ctypes.data), "nnet_set_params")

    def get_params(self) -> dict:
        flat = np.empty(self.num_params, dtype=np.float32)
        check(nnet.nnet_get_params(self.h, flat.ctypes.data), "nnet_get_params")
        return self.unflatten(flat)

    def set_bn(self, layer, which, mean, var, gamma, beta, eps=1e-3, target_rms=None):
        """target_rms None: the layer's configured target-rms (1 unless a batchnorm-component
        sets one)."""
        target_rms = 0.0 if target_rms is None else target_rms
        arrs = [np.ascontiguousarray(a, dtype=np.float32) for a in (mean, var, gamma, beta)]
        check(nnet.nnet_set_bn(self.h, layer.encode(), which, *[a.ctypes.data for a in arrs],
                               float(eps), float(target_rms)), "nnet_set_bn")

    # compute -----------------------------------------------------------
    def forward(self, features_ptr, T: int):
        check(nnet.nnet_forward(self.h, features_ptr, int(T)), "nnet_forward")
        self.T = int(T)

    def forward_ivector(self, features_ptr, T: int, ivectors_ptr, seq_row0):
        """Forward with the ivector input: ivectors fp16 [B x dim] on the device, seq_row0
        int[B+1] frame offsets of the sequences (0 ... T)."""
        so = np.ascontiguousarray(seq_row0, dtype=np.int32)
        check(nnet.nnet_forward_ivector(self.h, features_ptr, int(T), ivectors_ptr, len(so) - 1,
                                        so.ctypes.data), "nnet_forward_ivector")
        self.T = int(T)

    def activation(self, layer: str):
        r, c = _i(), _i()
        p = nnet.nnet_activation(self.h, layer.encode(), C.byref(r), C.byref(c))
        if not p:
            raise KfError("nnet_activation: " + _err(nnet.nnet_last_error))
        return p, r.value, c.value

    def read_activation(self, layer: str) -> np.ndarray:
        p, r, c = self.activation(layer)
        return read_fp16(p, (r, c))

    def backward(self, out_grad_ptr):
        check(nnet.nnet_backward(self.h, out_grad_ptr), "nnet_backward")

    @property
    def grad_ptr(self):
        return nnet.nnet_grad_buffer(self.h)

    @property
    def master_ptr(self):
        return nnet.nnet_master_buffer(self.h)

    def relu_masks(self) -> dict:
        """Every layer's ReLU decisions (bit-packed on device) as uint8 per element."""
        out = {}
        for i, (name, ty, din, dout) in enumerate(self.layers):
            width = {6: dout, 7: dout, 9: None}.get(ty, 0)
            if width is None:
                width = self.params[name + ".BigW"][1]
            if not width:
                continue
            p = nnet.nnet_debug_tensor(self.h, b"mask", i)
            n = self.T * width
            raw = read_fp16(p, ((n + 15) // 16,)).view(np.uint8)
            out[name] = np.unpackbits(raw, bitorder="little")[:n]
        return out

    def read_grads(self) -> dict:
        return self.unflatten(read_f32(self.grad_ptr, (self.num_params,)))

    def bind_grad_buffer(self, ptr):
        check(nnet.nnet_bind_grad_buffer(self.h, ptr), "nnet_bind_grad_buffer")

    def set_fp8(self, on: bool = True):
        """MXFP8 forward GEMMs (kf_nnet.h nnet_set_fp8)"""
        check(nnet.nnet_set_fp8(self.h, int(on)), "nnet_set_fp8")

    def sgd(self, lr: float, momentum: float):
        check(nnet.nnet_sgd(self.h, float(lr), float(momentum)), "nnet_sgd")

    def dp_plan(self, bucket_bytes: int, max_buckets: int = 256):
        """[(after_step, begin, end)]: the gradient buckets nnet_backward exchanges
        (kf_nnet.h nnet_dp_plan), in issue order."""
        a, b, e = (_i * max_buckets)(), (_ll * max_buckets)(), (_ll * max_buckets)()
        n = nnet.nnet_dp_plan(self.h, int(bucket_bytes), max_buckets, a, b, e)
        if n < 0:
            raise KfError("nnet_dp_plan: " + _err(nnet.nnet_last_error))
        return [(a[i], b[i], e[i]) for i in range(n)]

    def weights_changed(self):
        """The fp16 weights were written through nnet_weight_buffer (kf_nnet.h)."""
        check(nnet.nnet_weights_changed(self.h), "nnet_weights_changed")

    def set_wgrad_stream(self, on: bool):
        """Weight gradients on their own stream, overlapping the input gradients (default
        on; kf_nnet.h nnet_set_wgrad_stream)."""
        check(nnet.nnet_set_wgrad_stream(self.h, int(on)), "nnet_set_wgrad_stream")

    def debug_backward(self, main_aff: int = -1, stall_cycles: int = 0):
        """Test hook of the two-stream backward (kf_nnet.h nnet_debug_backward): where the
        TDNN-F affine weight gradients run, and a spin of `stall_cycles` GPU cycles on the
        weight-gradient stream before each of its batches of work."""
        check(nnet.nnet_debug_backward(self.h, int(main_aff), int(stall_cycles)), "nnet_debug_backward")

    def set_row_subsampling(self, stride: int):
        """Row-subsampled train step (kf_nnet.h nnet_set_row_subsampling): 3 = the layers above
        the conv stack run on the rows the chain objective's output rows 0 (mod 3) depend on;
        0 = off (full rows)."""
        check(nnet.nnet_set_row_subsampling(self.h, int(stride)), "nnet_set_row_subsampling")

    def row_set(self):
        """(tc, tc0, rows) of the last forward: tc compact rows (0: full rows), compact row c is
        source row rows[c] (3c for c < tc0, then the tail (T-1) - 3(tc-1-c))."""
        tc, tc0 = _i(), _i()
        check(nnet.nnet_row_set(self.h, C.byref(tc), C.byref(tc0)), "nnet_row_set")
        n, n0 = tc.value, tc0.value
        T = self.T
        rows = np.array([3 * c if c < n0 else (T - 1) - 3 * (n - 1 - c) for c in range(n)], np.int64)
        return n, n0, rows

    def set_implicit_dz(self, on: bool):
        """TDNN-F input gradients without the stored dz: consumers read g through the ReLU
        mask (default off; kf_nnet.h nnet_set_implicit_dz)."""
        check(nnet.nnet_set_implicit_dz(self.h, int(on)), "nnet_set_implicit_dz")

    def dp_debug_early(self, on: bool):
        """Test hook: issue every gradient bucket before the backward runs (the
        negative control of the overlap tests)."""
        check(nnet.nnet_dp_debug_early(self.h, int(on)), "nnet_dp_debug_early")

    def bind_dp(self, comm, bucket_bytes: int):
        """Exchange the gradient over `comm` (kfp16.dp.Communicator) in buckets during
        nnet_backward; comm None unbinds."""
        check(nnet.nnet_bind_dp(self.h, comm.h if comm is not None else None, int(bucket_bytes)),
              "nnet_bind_dp")


def parse_summary(xconfig: str):
    """Host-layer xconfig resolution without touching the device."""
    n = nnet.nnet_parse_summary(xconfig.encode(), None, 0)
    if n < 0:
        raise KfError("nnet_parse_summary: " + _err(nnet.nnet_last_error))
    buf = C.create_string_buffer(n)
    nnet.nnet_parse_summary(xconfig.encode(), buf, n)
    lines = buf.value.decode().strip().splitlines()
    layers = [(a, int(b), int(c), int(d)) for a, b, c, d in (l.split() for l in lines[:-1])]
    return layers, int(lines[-1].split()[1])


def read_header_symbols(header: str):
    """Function names declared in include/<header> (for the ABI export test)."""
    import re
    text = open(os.path.join(INCDIR, header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    names = re.findall(r"\b([a-z][a-z0-9_]*)\s*\([^;{]*\)\s*;", text)
    return sorted(set(n for n in names if not n.startswith(("sizeof", "typedef"))))


# ---------------------------------------------------------------- kf_ops structs
MAXP = 9


class KfOperand(C.Structure):
    _fields_ = [("base", _vp), ("ld", _ll), ("nrows", _i), ("ncols", _i), ("kcontig", _i),
                ("nparts", _i), ("part_width", _i), ("T", _i), ("hout", _i), ("hsrc", _i),
                ("hmul", _i), ("hdiv", _i), ("tpolicy", _i), ("dt", _i * MAXP), ("dh", _i * MAXP),
                ("edge_t", _i * MAXP), ("edge_row", _i * MAXP), ("fmt", _i), ("scales", _vp),
                ("lds", _ll), ("mask", _vp), ("mask_rows", _i), ("tmul", _i), ("t0", _i)]


FMT_FP16, FMT_MXFP8 = 0, 1


class KfEpilogue(C.Structure):
    _fields_ = [("out", _vp), ("ldo", _ll), ("alpha", _f), ("beta", _f), ("bias", _vp), ("relu", _i),
                ("mask_out", _vp), ("scale", _vp), ("shift", _vp), ("resid", _vp), ("ldr", _ll),
                ("resid_alpha", _f), ("out2", _vp), ("ldo2", _ll), ("scale2", _vp), ("mask_in", _vp),
                ("out8", _vp), ("ldo8", _ll), ("scale8", _vp), ("out8_src", _i), ("edge_out", _vp),
                ("edge_r0", _i), ("edge_r1", _i), ("edge_src", _i),
                ("row_group", _i), ("row_stride", _i)]


def operand(base, ld, rows, cols, kcontig, nparts=1, part_width=None, T=None, hout=1, hsrc=1,
            hmul=0, hdiv=1, tpolicy=0, dt=(), dh=(), edges=(), scales=None, lds=0, mask=None, mask_rows=0):
    """scales != None makes an MXFP8 operand (base: e4m3 bytes, scales: E8M0, lds bytes/row);
    mask != None a masked fp16 operand (kf_ops.h: bit i of mask gates source element i of the
    first mask_rows source rows)"""
    o = KfOperand()
    if mask is not None:
        o.mask, o.mask_rows = mask, mask_rows
    if scales is not None:
        o.fmt, o.scales, o.lds = FMT_MXFP8, scales, lds
    o.base, o.ld, o.nrows, o.ncols, o.kcontig = base, ld, rows, cols, kcontig
    o.nparts, o.part_width = nparts, part_width if part_width is not None else cols
    o.T = T if T is not None else rows
    o.hout, o.hsrc, o.hmul, o.hdiv, o.tpolicy = hout, hsrc, hmul, hdiv, tpolicy
    for i in range(MAXP):
        o.edge_t[i] = -1
    for i, v in enumerate(dt):
        o.dt[i] = v
    for i, v in enumerate(dh):
        o.dh[i] = v
    for p, t, row in edges:
        o.edge_t[p] = t
        o.edge_row[p] = row
    return o


_sig(core, "kf_gemm_fused", _i, _i, _i, _i, C.POINTER(KfOperand), C.POINTER(KfOperand), C.POINTER(KfEpilogue))
_sig(core, "kf_gemm_wgrad", _i, _i, _i, _i, C.POINTER(KfOperand), C.POINTER(KfOperand), _vp, _ll, _vp, _i)
_sig(core, "kf_rows_sum", _i, _vp, _vp, _ll, _i, _i, _i)
_sig(core, "kf_rows_sum_mask", _i, _vp, _vp, _ll, _i, _i, _i, _vp)
_sig(core, "kf_dot2_rows", _i, _vp, _vp, _vp, _vp, _i, _i)
_sig(core, "kf_gemm_fused_edge", _i, _i, _i, _i, C.POINTER(KfOperand), C.POINTER(KfOperand), C.POINTER(KfEpilogue),
     _vp, _vp, _vp, _vp, _i)
_sig(core, "kf_scale_cols", _i, _vp, _ll, _vp, _vp, _ll, _i, _i)
_sig(core, "kf_gemm_wgrad_scaled", _i, _i, _i, _i, C.POINTER(KfOperand), C.POINTER(KfOperand), _vp, _ll, _vp, _i,
     _vp)
_sig(core, "kf_gemm_debug_kil", None, _i)
_sig(core, "kf_gemm_trace", None, _vp, _i, _i)
_sig(core, "kf_quant_mxfp8", _i, _vp, _ll, _i, _i, _i, _vp, _ll, _vp, _ll)
