"""kfp16.chain — ctypes binding of the batched chain objective (include/kf_chain.h)
and of the reference's chain / den ABI (include/chain.h, chain_den.h,
chain_backward_api.h). Device work only; the CPU restatement lives in oracle/."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import KfError, core

_vp, _i, _f, _ll = C.c_void_p, C.c_int, C.c_float, C.c_longlong
_ip = C.POINTER(C.c_int32)
_fp = C.POINTER(C.c_float)


class KfChainOpts(C.Structure):
    """ChainTrainingOpts, backward.go:114-140 (DefaultChainTrainingOpts :132-140)."""
    _fields_ = [("l2_regularize", C.c_float), ("out_of_range_regularize", C.c_float),
                ("leaky_hmm_coefficient", C.c_float), ("xent_regularize", C.c_float),
                ("supervision_weight", C.c_float)]

    @classmethod
    def default(cls):
        return cls(0.0, 0.01, 1e-5, 0.0, 1.0)


class KfChainResult(C.Structure):
    _fields_ = [("objf", C.c_double), ("l2_term", C.c_double), ("total_weight", C.c_double),
                ("num_logprob", C.c_double), ("den_logprob", C.c_double), ("frames", C.c_int),
                ("out_of_range", C.c_int), ("num_ok", C.c_int), ("num_seqs", C.c_int)]


class ChainFstGPU(C.Structure):
    _fields_ = [("row_ptr", _vp), ("col_idx", _vp), ("labels", _vp), ("weights", _vp),
                ("final_states", _vp), ("final_weights", _vp), ("num_states", C.c_int),
                ("num_arcs", C.c_int), ("num_final", C.c_int), ("start_state", C.c_int)]


class ChainLossResult(C.Structure):
    _fields_ = [("num_logprob", C.c_float), ("den_logprob", C.c_float), ("loss", C.c_float)]


class DenFstGPU(C.Structure):
    _fields_ = [("src_states", _vp), ("dst_states", _vp), ("pdf_ids", _vp),
                ("transition_probs", _vp), ("num_transitions", C.c_int), ("num_states", C.c_int),
                ("num_pdfs", C.c_int)]


def _sig(name, res, *args):
    fn = getattr(core, name)
    fn.restype = res
    fn.argtypes = list(args)


for _n in ("kf_chain_last_error", "chain_last_error", "den_last_error"):
    _sig(_n, C.c_char_p)
_sig("kf_den_graph_create", _vp, _i, _i, _i, _vp, _vp, _vp, _vp, _i, _vp)
_sig("kf_den_graph_initial_probs", _i, _vp, _vp)
_sig("kf_den_graph_free", None, _vp)
_sig("kf_num_batch_create", _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp)
_sig("kf_num_batch_refill", _i, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp)
_sig("kf_num_batch_free", None, _vp)
_sig("kf_chain_create", _vp, _vp, _i, _i)
_sig("kf_chain_free", None, _vp)
_sig("kf_chain_compute", _i, _vp, _vp, C.POINTER(KfChainOpts), _vp, _ll, _ll, _i, _vp, _vp, _i, _vp, _ll)
_sig("kf_chain_seq_stats", _vp, _vp)
_sig("kf_chain_result", _i, _vp, C.POINTER(KfChainResult))
_sig("kf_chain_debug_spin_limit", None, _vp, C.c_uint)
_sig("kf_chain_debug_exchange_sys", None, _vp, C.c_int)
_sig("kf_chain_debug_den_pairs", None, _vp, C.c_int)
_sig("kf_chain_debug_census", C.c_int, _vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int),
     C.POINTER(C.c_int), C.POINTER(C.c_int))
_sig("chain_forward_backward", _i, _vp, C.POINTER(ChainFstGPU), _i, _i, _vp, _vp, _fp)
_sig("chain_compute_posteriors", _i, _vp, C.POINTER(ChainFstGPU), _i, _i, _vp, _vp, _f, _vp)
_sig("chain_compute_loss", _i, _vp, C.POINTER(ChainFstGPU), C.POINTER(ChainFstGPU), _i, _i, _vp,
     C.POINTER(ChainLossResult))
_sig("chain_num_forward_backward", _f, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp, _vp, _i, _i, _vp)
_sig("chain_penalize_out_of_range", _i, _vp, _vp, _f, _f, _i, _i)
_sig("chain_l2_regularize", _f, _vp, _vp, _f, _i)
_sig("chain_add_posterior_gradient", _i, _vp, _vp, _vp, _f, _i)
_sig("chain_combine_gradient", _i, _vp, _vp, _f, _i, _i, _vp)
_sig("chain_grad_fp32_to_fp16", _i, _vp, _vp, _i)
_sig("den_fst_upload", _i, C.POINTER(DenFstGPU), _vp, _vp, _vp, _vp, _i, _i, _i)
_sig("den_fst_free", None, C.POINTER(DenFstGPU))
_sig("den_forward", _f, C.POINTER(DenFstGPU), _vp, _vp, _i, _f)
_sig("den_forward_backward", _f, C.POINTER(DenFstGPU), _vp, _vp, _i, _f, _vp)


def _raise(what):
    s = core.kf_chain_last_error()
    raise KfError(f"{what}: {s.decode() if s else 'unknown error'}")


def _a(x, dt):
    return np.ascontiguousarray(x, dtype=dt)


class DenGraph:
    """kf_den_graph_create over a dict from synth.make_den_graph."""

    def __init__(self, g: dict, initial_probs=None):
        self.S, self.P, self.A = int(g["S"]), int(g["P"]), int(g["A"])
        self._keep = [_a(g["src"], np.int32), _a(g["dst"], np.int32), _a(g["pdf0"], np.int32),
                      _a(g["tp"], np.float32)]
        ip = None if initial_probs is None else _a(initial_probs, np.float32)
        self.h = core.kf_den_graph_create(self.S, self.P, self.A,
                                          *[k.ctypes.data for k in self._keep], int(g["start"]),
                                          None if ip is None else ip.ctypes.data)
        if not self.h:
            _raise("kf_den_graph_create")

    def initial_probs(self) -> np.ndarray:
        out = np.empty(self.S, np.float32)
        core.kf_den_graph_initial_probs(self.h, out.ctypes.data)
        return out

    def close(self):
        if self.h:
            core.kf_den_graph_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def pack_num_fsts(fsts) -> dict:
    """Concatenate per-eg CSR FSTs into the kf_num_batch_create arrays."""
    so, ao, fo = [0], [0], [0]
    rp, dst, pdf, w, fs, fw = [], [], [], [], [], []
    for f in fsts:
        so.append(so[-1] + f["S"])
        ao.append(ao[-1] + f["A"])
        fo.append(fo[-1] + len(f["final_state"]))
        rp.append(f["row_ptr"])
        dst.append(f["dst"])
        pdf.append(f["pdf1"])
        w.append(f["logw"])
        fs.append(f["final_state"])
        fw.append(f["final_w"])
    return dict(nseq=len(fsts), state_off=_a(so, np.int32), arc_off=_a(ao, np.int32),
                row_ptr=_a(np.concatenate(rp), np.int32), dst=_a(np.concatenate(dst), np.int32),
                pdf1=_a(np.concatenate(pdf), np.int32), logw=_a(np.concatenate(w), np.float32),
                final_off=_a(fo, np.int32), final_state=_a(np.concatenate(fs), np.int32),
                final_w=_a(np.concatenate(fw), np.float32))


_NUM_KEYS = ("state_off", "arc_off", "row_ptr", "dst", "pdf1", "logw", "final_off", "final_state", "final_w")


class NumBatch:
    """Numerator FSTs of one minibatch on the device. `fsts`: per-eg CSR dicts, or the
    arrays of pack_num_fsts."""

    def __init__(self, fsts):
        p = fsts if isinstance(fsts, dict) else pack_num_fsts(fsts)
        self.nseq = p["nseq"]
        self._keep = p
        self.h = core.kf_num_batch_create(self.nseq, *[p[k].ctypes.data for k in _NUM_KEYS])
        if not self.h:
            _raise("kf_num_batch_create")

    def refill(self, fsts, stream=None):
        """The next minibatch's FSTs into this batch (kf_num_batch_refill): asynchronous on
        `stream` (a HIP stream handle, None: the library stream), no device-wide stall."""
        p = fsts if isinstance(fsts, dict) else pack_num_fsts(fsts)
        if core.kf_num_batch_refill(self.h, p["nseq"], *[p[k].ctypes.data for k in _NUM_KEYS], stream) != 0:
            _raise("kf_num_batch_refill")
        self.nseq = p["nseq"]
        self._keep = p   # the host arrays were staged (pinned copy) before the call returned

    def close(self):
        if self.h:
            core.kf_num_batch_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Chain:
    """Batched objective: compute() is asynchronous on the library stream."""

    def __init__(self, den: DenGraph, max_seqs: int, max_frames: int):
        self.den = den
        self.h = core.kf_chain_create(den.h, max_seqs, max_frames)
        if not self.h:
            _raise("kf_chain_create")

    def compute(self, num: NumBatch, nnet_ptr, ld, num_rows, seq_row0, seq_frames, stride,
                out_grad_ptr, ldg, opts: KfChainOpts | None = None):
        opts = opts or KfChainOpts.default()
        self._r0 = _a(seq_row0, np.int32)
        self._fr = _a(seq_frames, np.int32)
        rc = core.kf_chain_compute(self.h, num.h, C.byref(opts), nnet_ptr, ld, num_rows, len(self._r0),
                                   self._r0.ctypes.data, self._fr.ctypes.data, stride,
                                   out_grad_ptr, ldg)
        if rc != 0:
            _raise("kf_chain_compute")

    def result(self) -> KfChainResult:
        r = KfChainResult()
        if core.kf_chain_result(self.h, C.byref(r)) != 0:
            _raise("kf_chain_result")
        return r

    def debug_spin_limit(self, polls: int | None):
        """Test knob: polls before a den exchange wait gives up (None: default)."""
        core.kf_chain_debug_spin_limit(self.h, 0xFFFFFFFF if polls is None else int(polls))

    def debug_exchange_sys(self, force: bool):
        """Test knob: den exchange through memory (agent scope) even on one XCD."""
        core.kf_chain_debug_exchange_sys(self.h, 1 if force else 0)

    def debug_den_pairs(self, pairs: bool):
        """Test knob: den recursions on sequence pairs (default) or one sequence per unit."""
        core.kf_chain_debug_den_pairs(self.h, 1 if pairs else 0)

    def debug_census(self) -> dict:
        """The XCD census of the last compute's den launch: exchange units per direction,
        units whose workgroups all shared one XCD (L2-local exchange unless forced)."""
        v = [C.c_int() for _ in range(5)]
        if core.kf_chain_debug_census(self.h, *(C.byref(x) for x in v)) != 0:
            _raise("kf_chain_debug_census")
        return {"units": v[0].value, "local_fwd": v[1].value, "local_bwd": v[2].value, "forced": bool(v[3].value),
                "G": v[4].value}

    def seq_stats(self, nseq: int) -> np.ndarray:
        from . import read_f32, sync
        sync()
        return read_f32(core.kf_chain_seq_stats(self.h), (nseq, 8))

    def close(self):
        if self.h:
            core.kf_chain_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def den_graph_from_fst(path_or_bytes, num_pdfs: int) -> dict:
    """NewNativeDenominator's transition extraction (denominator.go:68-117): read den.fst
    (OpenFst vector or compact acceptor, through the egs FST reader kf_egs_parse_fst),
    drop epsilon arcs, pdf0 = label - 1, tp = float32(exp(-weight)) computed in float64.
    Returns the dict DenGraph takes; initial probabilities are left to
    kf_den_graph_create's 100-iteration rule (denominator.go:131-171)."""
    from . import egs
    data = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else open(path_or_bytes, "rb").read()
    f = egs.parse_fst(bytes(data))
    if f is None:
        raise KfError("failed to parse den.fst (unsupported format?)")
    src = np.repeat(np.arange(f.num_states, dtype=np.int32), np.diff(f.arc_off))
    keep = f.label - 1 >= 0
    tp = np.exp(-f.weight.astype(np.float64)).astype(np.float32)
    return dict(S=int(f.num_states), P=int(num_pdfs), A=int(keep.sum()), src=src[keep].astype(np.int32),
                dst=f.next_state[keep].astype(np.int32), pdf0=(f.label[keep] - 1).astype(np.int32),
                tp=tp[keep], start=int(f.start))
