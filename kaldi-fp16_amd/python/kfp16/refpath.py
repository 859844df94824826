"""The reference's own host path for the network forward, run over this build's per-op
C-ABI: the drop-in as an unchanged internal/nnet would use it.

An unchanged Go host calls one ABI entry point per step of each layer
(internal/nnet/forward.go:148-1001, internal/gpu/ops.go:55-351):

  IDCT            ops_gemm(x, idct)                                      forward.go:317-330
  batchnorm-comp. ops_copy + ops_batchnorm_forward                       forward.go:348-376
  conv-relu-bn    host im2col, upload, ops_gemm, AddBias, ops_relu,
                  ops_batchnorm_forward                                  forward.go:418-524
  TDNN-F          spliceBackward (ops_copy of row views, ops_concat_cols),
                  ops_gemm, spliceForward, ops_gemm, AddBias, ops_relu,
                  ops_batchnorm_forward, ops_add_scaled (bypass)         forward.go:589-790
  linear          ops_gemm                                               forward.go:332-346
  prefinal        ops_gemm, AddBias, ops_relu, ops_batchnorm_forward,
                  ops_gemm, ops_batchnorm_forward                        forward.go:911-968
  output          ops_gemm, AddBias                                      forward.go:971-1001

AddBias is ops.go:335-351's K = 1 GEMM against a ones column (ops_fill + ops_gemm with
beta = 1). This class issues exactly that sequence through the ctypes bindings of
libkaldi_fp16.so; nothing is fused. It is the parity and timing harness for the
drop-in claim (tests/test_gpu_refpath.py, bench.py sub_results), not the product's
training path (kf_nnet.h), and it computes nothing on the host except what the
reference computes on the host (the conv im2col, forward.go:435-456).

Deliberate differences, each the same one the product makes:
  * conv uses Kaldi's cross-product time x height offsets and keeps the height-major
    layout (the reference zips the offsets and reorders filter-major on the host,
    forward.go:442-444, :499-508); BatchNorm is then per filter on the
    [(t, h) x filters] view, which is Kaldi's per-filter statistics tiled over height;
  * ZeroTensor's host upload of zeros (tensor.go:50-62) is ops_fill(0): the spliced
    buffer is overwritten by the two ops_concat_cols either way;
  * buffers are allocated once for max_frames instead of per layer per call.
"""
from __future__ import annotations


import numpy as np

from . import DeviceBuffer, KfError, check, core, read_fp16, upload_f32, upload_fp16
from . import _f, _i, _sig, _vp

_sig(core, "ops_relu", _i, _vp, _i)
_sig(core, "ops_batchnorm_forward", _i, _vp, _i, _i, _vp, _vp, _vp, _vp, _f)
_sig(core, "ops_add_scaled", _i, _vp, _vp, _i, _f, _f)
_sig(core, "ops_copy", _i, _vp, _vp, _i)
_sig(core, "ops_fill", _i, _vp, _i, _f)
_sig(core, "ops_concat_cols", _i, _vp, _i, _i, _vp, _i, _i)


def parse_layers(text: str):
    """xconfig lines -> layer dicts (the keys this path reads; defaults of layers.go)."""
    layers, dims, prev = [], {}, None
    for line in text.splitlines():
        line = line.split("#")[0].strip()
        if not line:
            continue
        kind, *rest = line.split()
        kv = dict(tok.split("=", 1) for tok in rest)
        name = kv["name"]
        if kind == "input":
            dims[name] = int(kv["dim"])
            prev = name
            continue
        inp = kv.get("input", prev)
        if inp not in dims:
            raise KfError(f"refpath: input {inp!r} of {name} (Append inputs are not on this model)")
        din = dims[inp]
        L = dict(kind=kind, name=name, input=inp, in_dim=din, kv=kv)
        if kind == "idct-layer":
            L.update(out_dim=int(kv.get("dim", din)), lifter=float(kv.get("cepstral-lifter", 22)))
        elif kind == "batchnorm-component":
            L["out_dim"] = din
        elif kind == "conv-relu-batchnorm-layer":
            hin = int(kv["height-in"])
            L.update(hin=hin, hout=int(kv.get("height-out", hin)), sub=int(kv.get("height-subsample-out", 1)),
                     fout=int(kv["num-filters-out"]), fin=din // hin,
                     offs=[(a, b) for a in map(int, kv["time-offsets"].split(","))
                           for b in map(int, kv["height-offsets"].split(","))])
            L["out_dim"] = L["hout"] * L["fout"]
        elif kind == "tdnnf-layer":
            L.update(out_dim=int(kv["dim"]), bn_dim=int(kv["bottleneck-dim"]),
                     stride=int(kv.get("time-stride", 3)), bypass=float(kv.get("bypass-scale", 0.66)))
        elif kind == "linear-component":
            L["out_dim"] = int(kv["dim"])
        elif kind == "prefinal-layer":
            L.update(small=int(kv["small-dim"]), big=int(kv["big-dim"]), out_dim=int(kv["small-dim"]))
        elif kind == "output-layer":
            L["out_dim"] = int(kv["dim"])
        else:
            raise KfError(f"refpath: layer kind {kind} is not on the CNN-TDNN path")
        dims[name] = L["out_dim"]
        prev = name
        layers.append(L)
    return layers


def idct_matrix(dim: int, lifter: float) -> np.ndarray:
    """makeIDCTMatrix (forward.go:1190-1210): float64, then float32; y = x . M."""
    i = np.arange(dim)[:, None]
    j = np.arange(dim)[None, :]
    m = np.cos(np.pi * j * (i + 0.5) / dim) * np.where(j == 0, np.sqrt(1.0 / dim), np.sqrt(2.0 / dim))
    if lifter > 0:
        m = m * np.where(j > 0, 1.0 + (lifter / 2.0) * np.sin(np.pi * j / lifter), 1.0)
    return m.astype(np.float32)


def fp16_trunc(a) -> np.ndarray:
    """float32ToFP16Bits (tensor.go:158-173): truncation, fp16 subnormals flushed."""
    b = np.ascontiguousarray(a, np.float32).view(np.uint32)
    sign = ((b >> 16) & 0x8000).astype(np.uint16)
    exp = ((b >> 23) & 0xFF).astype(np.int32) - 127
    frac = (b & 0x7FFFFF) >> 13
    h = np.where(exp > 15, sign | 0x7C00,
                 np.where(exp < -14, sign, sign | ((exp + 15) << 10).astype(np.uint32) | frac)).astype(np.uint16)
    return h.view(np.float16)


class RefPathForward:
    """Network.Forward (forward.go:148) over the per-op ABI, for one network's weights."""

    def __init__(self, xconfig: str, params: dict, bns: dict, max_frames: int, eps: float = 1e-3,
                 start_layer: str | None = None):
        """params: fp32 weights by the product's names (kfp16.Network.params), stored fp16
        by truncation like every weight; bns: {(layer, which): (mean, var, gamma, beta)}.
        start_layer: run from that layer on, its input supplied by the caller (timing the
        TDNN-F stack without the host im2col of the conv front end)."""
        self.layers = parse_layers(xconfig)
        if start_layer is not None:
            k = [L["name"] for L in self.layers].index(start_layer)
            self.layers = self.layers[k:]
        self.T = int(max_frames)
        self.ncalls = 0
        self.eps = float(eps)
        self.h = core.ops_cublas_create()
        self.w, self.bn, self.act = {}, {}, {}
        T = self.T
        maxw = 0
        for L in self.layers:
            n, kind = L["name"], L["kind"]
            if kind == "idct-layer":
                self.w[n + ".M"] = upload_fp16(fp16_trunc(idct_matrix(L["out_dim"], L["lifter"])))
            for suffix in (".W", ".Bias", ".LinearW", ".AffineW", ".AffineBias", ".BigW", ".BigBias", ".SmallW"):
                if n + suffix in params:
                    self.w[n + suffix] = upload_fp16(fp16_trunc(params[n + suffix]))
            for which in (0, 1):
                if (n, which) in bns:
                    self.bn[(n, which)] = [upload_f32(np.asarray(a, np.float32)) for a in bns[(n, which)]]
            rows = T * L.get("hout", 1)
            self.act[n] = DeviceBuffer(T * L["out_dim"] * 2)
            maxw = max(maxw, L["in_dim"], L["out_dim"], L.get("big", 0), L.get("bn_dim", 0))
            if kind == "conv-relu-batchnorm-layer":
                L["patch"] = DeviceBuffer(rows * len(L["offs"]) * L["fin"] * 2)
        self.ones = DeviceBuffer(T * 40 * 2)  # AddBias ones column, up to T * hout rows
        self.shifted = DeviceBuffer(T * maxw * 2)
        self.spliced = DeviceBuffer(T * 2 * maxw * 2)
        self.tmp = DeviceBuffer(T * maxw * 2)
        self.tmp2 = DeviceBuffer(T * maxw * 2)

    def _c(self, rc, what):
        """one reference ABI call (counted; raises on failure like ops.go's opsErr)"""
        self.ncalls += 1
        check(rc, what)

    def close(self):
        if getattr(self, "h", None):
            core.ops_cublas_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- internal/gpu/ops.go wrappers ------------------------------------------------
    def _gemm(self, M, N, K, A, B, Cp, beta=0.0, lda=None):
        self._c(core.ops_gemm(self.h, M, N, K, 1.0, A, lda or K, B, N, beta, Cp, N), "ops_gemm")

    def _add_bias(self, x, rows, cols, bias):  # ops.go:335-351
        self._c(core.ops_fill(self.ones.ptr, rows, 1.0), "ops_fill")
        self._gemm(rows, cols, 1, self.ones.ptr, bias, x, beta=1.0, lda=1)

    def _bn(self, x, rows, cols, name, which):
        if (name, which) not in self.bn:
            return
        m, v, g, b = self.bn[(name, which)]
        self._c(core.ops_batchnorm_forward(x, rows, cols, m.ptr, v.ptr, g.ptr, b.ptr, self.eps), "ops_batchnorm_forward")

    def _view(self, buf, row, cols):
        return (buf.ptr if isinstance(buf, DeviceBuffer) else buf) + row * cols * 2

    def _splice(self, x, T, cols, stride, backward: bool):
        """spliceBackward ([x(t-s) | x(t)], t < s -> row 0) / spliceForward ([x(t) | x(t+s)],
        t + s >= T -> row T-1), forward.go:700-790: row-view copies, then two ConcatCols."""
        sh = self.shifted.ptr
        if T > stride:
            if backward:
                self._c(core.ops_copy(self._view(sh, stride, cols), x, (T - stride) * cols), "ops_copy")
            else:
                self._c(core.ops_copy(sh, self._view(x, stride, cols), (T - stride) * cols), "ops_copy")
        edge = range(min(stride, T)) if backward else range(max(T - stride, 0), T)
        src = x if backward else self._view(x, T - 1, cols)
        for t in edge:
            self._c(core.ops_copy(self._view(sh, t, cols), src, cols), "ops_copy")
        sp = self.spliced.ptr
        self._c(core.ops_fill(sp, T * 2 * cols, 0.0), "ops_fill")
        first, second = (sh, x) if backward else (x, sh)
        self._c(core.ops_concat_cols(sp, T, 2 * cols, first, cols, 0), "ops_concat_cols")
        self._c(core.ops_concat_cols(sp, T, 2 * cols, second, cols, cols), "ops_concat_cols")
        return sp

    # ---- layers ------------------------------------------------------------------------
    def forward(self, features_ptr, T: int, inputs: dict | None = None):
        """features_ptr: fp16 [T x 40] on the device; inputs: {layer name: device ptr}
        for layers whose input comes from outside (start_layer)."""
        if T > self.T:
            raise KfError(f"refpath: T={T} > max_frames={self.T}")
        self.ncalls = 0
        ptrs = dict(inputs or {})
        ptrs.setdefault("input", features_ptr)
        for L in self.layers:
            n, kind, din, dout = L["name"], L["kind"], L["in_dim"], L["out_dim"]
            x, y = ptrs[L["input"]], self.act[n].ptr
            if kind == "idct-layer":
                self._gemm(T, dout, din, x, self.w[n + ".M"].ptr, y)
            elif kind == "batchnorm-component":
                self._c(core.ops_copy(y, x, T * dout), "ops_copy")
                self._bn(y, T, dout, n, 0)
            elif kind == "conv-relu-batchnorm-layer":
                self._conv(L, x, y, T)
            elif kind == "tdnnf-layer":
                s, bnd = L["stride"], L["bn_dim"]
                lin_in = self._splice(x, T, din, s, True) if s > 0 else x
                bott = self.tmp.ptr
                self._gemm(T, bnd, (2 if s > 0 else 1) * din, lin_in, self.w[n + ".LinearW"].ptr, bott)
                aff_in = self._splice(bott, T, bnd, s, False) if s > 0 else bott
                self._gemm(T, dout, (2 if s > 0 else 1) * bnd, aff_in, self.w[n + ".AffineW"].ptr, y)
                self._add_bias(y, T, dout, self.w[n + ".AffineBias"].ptr)
                self._c(core.ops_relu(y, T * dout), "ops_relu")
                self._bn(y, T, dout, n, 0)
                if L["bypass"] > 0 and din == dout:
                    self._c(core.ops_add_scaled(y, x, T * dout, L["bypass"], 1.0), "ops_add_scaled")
            elif kind == "linear-component":
                self._gemm(T, dout, din, x, self.w[n + ".W"].ptr, y)
            elif kind == "prefinal-layer":
                big = self.tmp2.ptr
                self._gemm(T, L["big"], din, x, self.w[n + ".BigW"].ptr, big)
                self._add_bias(big, T, L["big"], self.w[n + ".BigBias"].ptr)
                self._c(core.ops_relu(big, T * L["big"]), "ops_relu")
                self._bn(big, T, L["big"], n, 0)
                self._gemm(T, dout, L["big"], big, self.w[n + ".SmallW"].ptr, y)
                self._bn(y, T, dout, n, 1)
            elif kind == "output-layer":
                self._gemm(T, dout, din, x, self.w[n + ".W"].ptr, y)
                self._add_bias(y, T, dout, self.w[n + ".Bias"].ptr)
            ptrs[n] = y
        self.T_run = T
        return ptrs

    def _conv(self, L, x, y, T):
        """forwardConvReluBN (forward.go:418-524): the im2col on the host as the reference
        does it, upload (TensorFromFP32: truncation), GEMM, AddBias, ReLU, BatchNorm."""
        hin, hout, sub, fin, fout = L["hin"], L["hout"], L["sub"], L["fin"], L["fout"]
        xin = read_fp16(x, (T, hin, fin)).astype(np.float32)
        pad = np.zeros((T + 2 * 8, hin + 2 * 8, fin), np.float32)
        pad[8:8 + T, 8:8 + hin] = xin
        hs = np.arange(hout) * sub
        cols = []
        for dt, dh in L["offs"]:
            cols.append(pad[8 + dt:8 + dt + T][:, 8 + dh + hs])       # [T, hout, fin], zero outside
        patches = np.stack(cols, axis=2).reshape(T * hout, len(L["offs"]) * fin)
        p16 = fp16_trunc(patches)
        pbuf = L["patch"]
        self._c(core.bridge_transfer_fp16(pbuf.ptr, p16.ctypes.data, p16.size), "upload patches")
        rows, K = T * hout, len(L["offs"]) * fin
        self._gemm(rows, fout, K, pbuf.ptr, self.w[L["name"] + ".W"].ptr, y)
        self._add_bias(y, rows, fout, self.w[L["name"] + ".Bias"].ptr)
        self._c(core.ops_relu(y, rows * fout), "ops_relu")
        self._bn(y, rows, fout, L["name"], 0)

    def read(self, name: str) -> np.ndarray:
        L = next(L for L in self.layers if L["name"] == name)
        return read_fp16(self.act[name].ptr, (self.T_run, L["out_dim"]))
