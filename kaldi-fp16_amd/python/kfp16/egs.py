"""kfp16.egs — ctypes binding of the Kaldi chain egs reader / loader (include/kf_egs.h,
libkaldi_fp16_egs.so).

Mirrors the reference's Go surface (internal/parser, internal/sparse, internal/loader,
internal/batch): Reader / read_example, parse_index_vector, parse_fst, parse_sparse_matrix,
fst_to_csr, DataLoader.next_batch, TrainingBatch. Parsing, merging and the CSR build
run in the C++ library; the minibatch features go to the GPU still compressed and are
expanded there (TrainingBatch.features_to_device). Nothing here computes itself.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field

import numpy as np

from . import KfError, LIBDIR

_path = os.path.join(LIBDIR, "libkaldi_fp16_egs.so")
if not os.path.exists(_path):
    raise ImportError(f"kfp16.egs: {_path} is missing — build the libraries first (make -C kaldi-fp16_amd)")
lib = C.CDLL(_path, mode=C.RTLD_GLOBAL)

_vp, _i, _f, _sz = C.c_void_p, C.c_int, C.c_float, C.c_size_t
_i32p = C.POINTER(C.c_int32)
_fp = C.POINTER(C.c_float)

MAT_NONE, MAT_CM, MAT_CM2, MAT_CM3, MAT_FM = range(5)
MAT_NAMES = {MAT_CM: "CM", MAT_CM2: "CM2", MAT_CM3: "CM3", MAT_FM: "FM"}


class KfEgsIo(C.Structure):
    _fields_ = [("name", C.c_char_p), ("num_indexes", _i), ("indexes", _i32p), ("format", _i),
                ("rows", _i), ("cols", _i), ("min_value", _f), ("range", _f),
                ("payload", C.POINTER(C.c_uint8)), ("payload_bytes", _sz)]


class KfEgsFst(C.Structure):
    _fields_ = [("start", C.c_int64), ("num_states", C.c_int64), ("num_arcs", C.c_int64),
                ("properties", C.c_uint64), ("arc_off", _i32p), ("label", _i32p),
                ("weight", _fp), ("next_state", _i32p), ("final_weight", _fp)]


class KfEgsExample(C.Structure):
    _fields_ = [("key", C.c_char_p), ("num_inputs", _i), ("num_outputs", _i), ("num_io", _i),
                ("io", C.POINTER(KfEgsIo)), ("sup_name", C.c_char_p), ("sup_num_indexes", _i),
                ("sup_indexes", _i32p), ("weight", _f), ("num_sequences", _i),
                ("frames_per_seq", _i), ("label_dim", _i), ("end2end", _i), ("has_fst", _i),
                ("fst", KfEgsFst), ("num_deriv_weights", _i), ("deriv_weights", _fp)]


class KfEgsBatchInfo(C.Structure):
    _fields_ = [("batch_size", _i), ("total_frames", _i), ("feat_dim", _i), ("ivector_dim", _i),
                ("label_dim", _i), ("num_sequences", _i), ("weight", _f),
                ("frame_offsets", _i32p), ("num_frames", _i32p), ("frames_per_seq", _i32p),
                ("state_offsets", _i32p), ("num_states", _i), ("num_arcs", _i), ("num_finals", _i),
                ("row_ptr", _i32p), ("col", _i32p), ("label", _i32p), ("logw", _fp),
                ("final_state", _i32p), ("final_logw", _fp), ("state_off", _i32p),
                ("arc_off", _i32p), ("final_off", _i32p), ("per_row_ptr", _i32p),
                ("per_col", _i32p), ("per_final_state", _i32p)]


def _sig(name, res, *args):
    fn = getattr(lib, name)
    fn.restype = res
    fn.argtypes = list(args)
    return fn


_sig("kf_egs_last_error", C.c_char_p)
_sig("kf_egs_clear_error", None)
_sig("kf_egs_detect_format", _i, C.c_char_p)
_sig("kf_egs_open", _vp, C.c_char_p)
_sig("kf_egs_next", _i, _vp, C.POINTER(C.POINTER(KfEgsExample)))
_sig("kf_egs_close", None, _vp)
_sig("kf_egs_example_valid", _i, C.POINTER(KfEgsExample))
_sig("kf_egs_example_usable", _i, C.POINTER(KfEgsExample))
_sig("kf_egs_io_to_float", _i, C.POINTER(KfEgsIo), _vp)
_sig("kf_egs_parse_index_vector", _i, _vp, _sz, _i, _vp, C.POINTER(_i), C.POINTER(_sz))
_sig("kf_egs_parse_fst", C.POINTER(KfEgsFst), _vp, _sz, C.POINTER(_sz))
_sig("kf_egs_fst_free", None, C.POINTER(KfEgsFst))
_sig("kf_egs_parse_sparse_matrix", _i, _vp, _sz, _vp, _vp, _vp, _vp, C.POINTER(_i), C.POINTER(_sz))
_sig("kf_egs_fst_to_csr", _i, C.POINTER(KfEgsFst), _vp, _vp, _vp, _vp, _vp, _vp, C.POINTER(_i))
_sig("kf_egs_loader_create", _vp, C.c_char_p, _i, _i, C.c_ulonglong, _i)
_sig("kf_egs_loader_next", _i, _vp, C.POINTER(_vp))
_sig("kf_egs_loader_reset", None, _vp)
_sig("kf_egs_loader_stats", None, _vp, C.POINTER(_i), C.POINTER(_i), C.POINTER(C.c_double))
_sig("kf_egs_loader_num_files", _i, _vp)
_sig("kf_egs_loader_free", None, _vp)
_sig("kf_egs_batch_info", _i, _vp, C.POINTER(KfEgsBatchInfo))
_sig("kf_egs_batch_key", C.c_char_p, _vp, _i)
_sig("kf_egs_batch_features_host", _i, _vp, _vp)
_sig("kf_egs_batch_ivectors_host", _i, _vp, _vp)
_sig("kf_egs_batch_features", _i, _vp, _vp, _i, _vp)
_sig("kf_egs_batch_upload_bytes", _sz, _vp)
_sig("kf_egs_batch_free", None, _vp)
_sig("kf_egs_batch_from_examples", _vp, C.POINTER(C.POINTER(KfEgsExample)), _i)


def last_error() -> str:
    e = lib.kf_egs_last_error()
    return e.decode() if e else ""


class EgsError(KfError):
    pass


def _arr(ptr, n, dt):
    if n <= 0:
        return np.zeros(0, dt)
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dt, copy=True)


# ----------------------------------------------------------------------- values
@dataclass
class Fst:
    """parser.Fst (types.go:118-125) as arc arrays in state order."""
    start: int
    num_states: int
    num_arcs: int          # header value for compact_acceptor, counted for vector
    properties: int
    arc_off: np.ndarray
    label: np.ndarray
    weight: np.ndarray
    next_state: np.ndarray
    final: np.ndarray      # +inf = not final

    @classmethod
    def from_c(cls, f: KfEgsFst) -> "Fst":
        S = int(f.num_states)
        off = _arr(f.arc_off, S + 1, np.int32)
        A = int(off[-1]) if S >= 0 else 0
        return cls(int(f.start), S, int(f.num_arcs), int(f.properties), off,
                   _arr(f.label, A, np.int32), _arr(f.weight, A, np.float32),
                   _arr(f.next_state, A, np.int32), _arr(f.final_weight, S, np.float32))

    def arcs(self, s):
        a, b = int(self.arc_off[s]), int(self.arc_off[s + 1])
        return [(int(self.label[i]), float(self.weight[i]), int(self.next_state[i])) for i in range(a, b)]


@dataclass
class IoBlock:
    """parser.IoBlock + MatrixInfo (types.go:18-33); the matrix stays compressed."""
    name: str
    indexes: np.ndarray    # [n, 3] (n, t, x)
    format: int
    rows: int
    cols: int
    min_value: float
    range: float
    payload: bytes

    @property
    def type(self) -> str:
        return MAT_NAMES.get(self.format, "")

    @property
    def size(self) -> int:
        return len(self.indexes)


@dataclass
class Example:
    """parser.Example (types.go:3-9) + SupervisionBlock (:51-62)."""
    key: str
    num_inputs: int
    num_outputs: int
    inputs: list
    sup_name: str
    sup_indexes: np.ndarray
    weight: float
    num_sequences: int
    frames_per_seq: int
    label_dim: int
    end2end: bool
    fst: Fst | None
    deriv_weights: np.ndarray
    valid: bool = False
    usable: bool = False
    _mats: dict = field(default_factory=dict, repr=False)

    def matrix(self, i: int) -> np.ndarray:
        """Host decompression (matrix.go:10-168), fp32 [rows, cols]."""
        return self._mats[i]


def _example_from_c(p) -> Example:
    ex = p.contents
    inputs, mats = [], {}
    for i in range(ex.num_io):
        io = ex.io[i]
        n = io.num_indexes
        idx = _arr(io.indexes, 3 * n, np.int32).reshape(n, 3)
        payload = C.string_at(io.payload, io.payload_bytes) if io.payload_bytes else b""
        inputs.append(IoBlock(io.name.decode(), idx, io.format, io.rows, io.cols, io.min_value,
                              io.range, payload))
        m = np.zeros((io.rows, io.cols), np.float32)
        if lib.kf_egs_io_to_float(C.byref(io), m.ctypes.data) != 0:
            raise EgsError(last_error())
        mats[i] = m
    n = ex.sup_num_indexes
    return Example(
        key=ex.key.decode(), num_inputs=ex.num_inputs, num_outputs=ex.num_outputs, inputs=inputs,
        sup_name=ex.sup_name.decode(), sup_indexes=_arr(ex.sup_indexes, 3 * n, np.int32).reshape(n, 3),
        weight=ex.weight, num_sequences=ex.num_sequences, frames_per_seq=ex.frames_per_seq,
        label_dim=ex.label_dim, end2end=bool(ex.end2end),
        fst=Fst.from_c(ex.fst) if ex.has_fst else None,
        deriv_weights=_arr(ex.deriv_weights, ex.num_deriv_weights, np.float32),
        valid=bool(lib.kf_egs_example_valid(p)), usable=bool(lib.kf_egs_example_usable(p)), _mats=mats)


# ----------------------------------------------------------------------- reader
def detect_format(path: str) -> None:
    """parser.DetectFormat (parser.go:77-110): raises EgsError unless binary ark."""
    if lib.kf_egs_detect_format(path.encode()) != 0:
        raise EgsError(last_error())


class Reader:
    """parser.Reader (parser.go:29-131)."""

    def __init__(self, path: str):
        self._h = lib.kf_egs_open(path.encode())
        if not self._h:
            raise EgsError(last_error())

    def read_example(self) -> Example | None:
        """Next example, None at EOF, EgsError on a parse error."""
        p = C.POINTER(KfEgsExample)()
        r = lib.kf_egs_next(self._h, C.byref(p))
        if r < 0:
            raise EgsError(last_error())
        return _example_from_c(p) if r == 1 else None

    def raw_next(self):
        """Next example as the C struct pointer (valid until the next call)."""
        p = C.POINTER(KfEgsExample)()
        r = lib.kf_egs_next(self._h, C.byref(p))
        if r < 0:
            raise EgsError(last_error())
        return p if r == 1 else None

    def close(self):
        if self._h:
            lib.kf_egs_close(self._h)
            self._h = None

    def __iter__(self):
        while True:
            ex = self.read_example()
            if ex is None:
                return
            yield ex

    def __del__(self):
        self.close()


def parse_index_vector(buf: bytes, count: int):
    """readIndexVector (parser.go:484-548) on a byte buffer.
    Returns (indexes [n,3], error-or-None, bytes used)."""
    out = np.zeros((max(count, 0), 3), np.int32)
    n = _i()
    used = _sz()
    r = lib.kf_egs_parse_index_vector(buf, len(buf), count, out.ctypes.data, C.byref(n), C.byref(used))
    err = last_error() if r != 0 else None
    if count <= 0:
        return None, err, used.value
    return out[:n.value], err, used.value


def parse_fst(buf: bytes) -> Fst | None:
    """ReadFst (fst.go:18-40); None on a bad magic, type or truncation."""
    used = _sz()
    p = lib.kf_egs_parse_fst(buf, len(buf), C.byref(used))
    if not p:
        return None
    try:
        return Fst.from_c(p.contents)
    finally:
        lib.kf_egs_fst_free(p)


def parse_sparse_matrix(buf: bytes):
    """ReadSparseMatrix (matrix.go:172-192), buf after the "SM" token.
    Returns a list of rows (dim, [(index, value), ...]) or None."""
    npairs = _i()
    nrows = lib.kf_egs_parse_sparse_matrix(buf, len(buf), None, None, None, None, C.byref(npairs), None)
    if nrows < 0:
        return None
    dims = np.zeros(nrows, np.int32)
    offs = np.zeros(nrows + 1, np.int32)
    idx = np.zeros(max(npairs.value, 1), np.int32)
    val = np.zeros(max(npairs.value, 1), np.float32)
    lib.kf_egs_parse_sparse_matrix(buf, len(buf), dims.ctypes.data, offs.ctypes.data, idx.ctypes.data,
                                   val.ctypes.data, C.byref(npairs), None)
    return [(int(dims[r]), [(int(idx[k]), float(val[k])) for k in range(offs[r], offs[r + 1])])
            for r in range(nrows)]


def fst_to_csr(fst_c: KfEgsFst) -> dict:
    """sparse.FstToCSR (sparse.go:54-102) of a C FST view."""
    S, = (int(fst_c.num_states),)
    A = int(fst_c.arc_off[S]) if S > 0 else 0
    out = dict(row_ptr=np.zeros(max(S + 1, 1), np.int32), col=np.zeros(max(A, 1), np.int32),
               label=np.zeros(max(A, 1), np.int32), logw=np.zeros(max(A, 1), np.float32),
               final_state=np.zeros(max(S, 1), np.int32), final_logw=np.zeros(max(S, 1), np.float32))
    nf = _i()
    r = lib.kf_egs_fst_to_csr(C.byref(fst_c), *[out[k].ctypes.data for k in
                                                ("row_ptr", "col", "label", "logw", "final_state", "final_logw")],
                              C.byref(nf))
    if r != 0:
        raise EgsError(last_error())
    out["col"], out["label"], out["logw"] = out["col"][:A], out["label"][:A], out["logw"][:A]
    out["final_state"], out["final_logw"] = out["final_state"][:nf.value], out["final_logw"][:nf.value]
    out["row_ptr"] = out["row_ptr"][:S + 1]
    out["num_states"], out["num_arcs"], out["start_state"] = S, A, int(fst_c.start)
    return out


# ----------------------------------------------------------------------- batches
class TrainingBatch:
    """loader.TrainingBatch (dataloader.go:15-38) over a C++-owned KfEgsBatch."""

    def __init__(self, handle):
        self._h = handle
        info = KfEgsBatchInfo()
        if lib.kf_egs_batch_info(handle, C.byref(info)) != 0:
            raise EgsError(last_error())
        B = info.batch_size
        S, A, F = info.num_states, info.num_arcs, info.num_finals
        self.batch_size, self.total_frames, self.feat_dim = B, info.total_frames, info.feat_dim
        self.ivector_dim, self.label_dim = info.ivector_dim, info.label_dim
        self.num_sequences, self.weight = info.num_sequences, info.weight
        self.frame_offsets = _arr(info.frame_offsets, B, np.int32)
        self.num_frames = _arr(info.num_frames, B, np.int32)
        self.frames_per_seq = _arr(info.frames_per_seq, B, np.int32)
        self.state_offsets = _arr(info.state_offsets, B, np.int32)
        self.csr = dict(num_states=S, num_arcs=A, row_ptr=_arr(info.row_ptr, S + 1, np.int32),
                        col=_arr(info.col, A, np.int32), label=_arr(info.label, A, np.int32),
                        logw=_arr(info.logw, A, np.float32), final_state=_arr(info.final_state, F, np.int32),
                        final_logw=_arr(info.final_logw, F, np.float32))
        self.per_seq = dict(state_off=_arr(info.state_off, B + 1, np.int32),
                            arc_off=_arr(info.arc_off, B + 1, np.int32),
                            final_off=_arr(info.final_off, B + 1, np.int32),
                            row_ptr=_arr(info.per_row_ptr, S + B, np.int32),
                            dst=_arr(info.per_col, A, np.int32),
                            final_state=_arr(info.per_final_state, F, np.int32))
        self.keys = [lib.kf_egs_batch_key(handle, i).decode() for i in range(B)]

    def num_fsts(self) -> list:
        """Per-sequence numerator FSTs as the dicts kfp16.chain.pack_num_fsts takes."""
        p, c = self.per_seq, self.csr
        out = []
        for i in range(self.batch_size):
            s0, s1 = p["state_off"][i], p["state_off"][i + 1]
            a0, a1 = p["arc_off"][i], p["arc_off"][i + 1]
            f0, f1 = p["final_off"][i], p["final_off"][i + 1]
            out.append(dict(S=int(s1 - s0), A=int(a1 - a0), row_ptr=p["row_ptr"][s0 + i:s1 + i + 1].copy(),
                            dst=p["dst"][a0:a1].copy(), pdf1=c["label"][a0:a1].copy(),
                            logw=c["logw"][a0:a1].copy(), final_state=p["final_state"][f0:f1].copy(),
                            final_w=c["final_logw"][f0:f1].copy()))
        return out

    def features_host(self) -> np.ndarray:
        out = np.zeros((self.total_frames, self.feat_dim), np.float32)
        if lib.kf_egs_batch_features_host(self._h, out.ctypes.data) != 0:
            raise EgsError(last_error())
        return out

    def ivectors_host(self) -> np.ndarray:
        out = np.zeros((self.batch_size, self.ivector_dim), np.float32)
        if self.ivector_dim and lib.kf_egs_batch_ivectors_host(self._h, out.ctypes.data) != 0:
            raise EgsError(last_error())
        return out

    def features_to_device(self, dev_out: int, ldo: int, dev_ivec: int | None = None) -> None:
        """Compressed upload + GPU expansion into fp16 [total_frames, ldo] (and ivectors)."""
        if lib.kf_egs_batch_features(self._h, dev_out, ldo, dev_ivec) != 0:
            raise EgsError(last_error())

    @property
    def upload_bytes(self) -> int:
        return int(lib.kf_egs_batch_upload_bytes(self._h))

    def close(self):
        if self._h:
            lib.kf_egs_batch_free(self._h)
            self._h = None

    def __del__(self):
        self.close()


def batch_from_reader_examples(ptrs) -> TrainingBatch:
    """Assemble a TrainingBatch from raw example pointers (Reader.raw_next results must be
    copied first: each pointer is valid only until that reader's next call)."""
    arr = (C.POINTER(KfEgsExample) * len(ptrs))(*ptrs)
    h = lib.kf_egs_batch_from_examples(arr, len(ptrs))
    if not h:
        raise EgsError(last_error())
    return TrainingBatch(h)


class DataLoader:
    """loader.DataLoader (dataloader.go:41-197). pattern: glob, or a list of paths."""

    def __init__(self, pattern, batch_size: int, shuffle: bool = False, seed: int = 0,
                 drop_last: bool = False):
        if not isinstance(pattern, str):
            pattern = "\n".join(pattern) + "\n"
        self._h = lib.kf_egs_loader_create(pattern.encode(), batch_size, int(shuffle), seed, int(drop_last))
        if not self._h:
            raise EgsError(last_error())

    def next_batch(self) -> TrainingBatch | None:
        h = _vp()
        r = lib.kf_egs_loader_next(self._h, C.byref(h))
        if r < 0:
            raise EgsError(last_error())
        return TrainingBatch(h.value) if r == 1 else None

    def reset(self):
        lib.kf_egs_loader_reset(self._h)

    def stats(self):
        b, e, s = _i(), _i(), C.c_double()
        lib.kf_egs_loader_stats(self._h, C.byref(b), C.byref(e), C.byref(s))
        return dict(batches=b.value, examples=e.value, seconds=s.value)

    @property
    def num_files(self) -> int:
        return lib.kf_egs_loader_num_files(self._h)

    def close(self):
        if self._h:
            lib.kf_egs_loader_free(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __iter__(self):
        while True:
            b = self.next_batch()
            if b is None:
                return
            yield b
