"""oracle.py — ctypes driver of the CPU oracle (kf_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker / CPU baseline. The product path
never loads it.

It parses the xconfig on its own (a restatement of internal/nnet/xconfig.go's
key=value grammar and layers.go's dimension rules, independent of the C++ host
layer under test) and builds the oracle's layer table from named parameters.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "_build")


def build(native: bool = False) -> str:
    env = dict(os.environ)
    if native:
        env["ORACLE_NATIVE"] = "1"
    subprocess.run(["make", "-s", "-C", HERE], check=True, env=env)
    return os.path.join(BUILD, "libkforacle_native.so" if native else "libkforacle.so")


_lib = None


def lib(native: bool = False):
    global _lib
    if _lib is None:
        path = os.path.join(BUILD, "libkforacle_native.so" if native else "libkforacle.so")
        if not os.path.exists(path):
            path = build(native)
        _lib = C.CDLL(path)
        _lib.orc_f32_to_f16_rne.restype = C.c_uint16
        _lib.orc_f32_to_f16_rne.argtypes = [C.c_float]
        _lib.orc_f32_to_f16_trunc.restype = C.c_uint16
        _lib.orc_f32_to_f16_trunc.argtypes = [C.c_float]
        _lib.orc_f16_to_f32.restype = C.c_float
        _lib.orc_f16_to_f32.argtypes = [C.c_uint16]
        _lib.orc_set_threads.argtypes = [C.c_int]
        _lib.orc_matmul.argtypes = [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        _lib.orc_net_forward.argtypes = [C.c_void_p, C.c_void_p]
        _lib.orc_net_backward.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        _lib.orc_net_backward_top.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        _lib.orc_net_free.argtypes = [C.c_void_p]
        _lib.orc_sgd.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_float, C.c_float, C.c_longlong]
        _lib.orc_mx_qdq_rows.argtypes = [C.c_void_p, C.c_void_p, C.c_longlong, C.c_int]
        _lib.gt_matmul.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int]
        _lib.gt_affine_forward.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_int,
                                           C.c_void_p, C.c_void_p, C.c_int]
        _lib.gt_net_create.restype = C.c_void_p
        _lib.gt_net_create.argtypes = [C.c_void_p, C.c_int]
        _lib.gt_net_free.argtypes = [C.c_void_p]
        _lib.gt_net_forward.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int]
        _lib.gt_net_backward.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        _lib.gt_net_sgd.argtypes = [C.c_void_p, C.c_double, C.c_double]
        _lib.gt_net_tensor.restype = C.POINTER(C.c_double)
        _lib.gt_net_tensor.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_longlong)]
    return _lib


def gotorch_affine_forward(x: np.ndarray, W: np.ndarray, b: np.ndarray, workers: int, lib_=None):
    """gotorch.AffineLayer.Forward (go/gotorch/layers.go:57-70) restated in C
    (gotorch_cpu.c): float64, rows split over `workers` threads as matmulParallel."""
    L = lib_ or lib()
    x = np.ascontiguousarray(x, np.float64)
    W = np.ascontiguousarray(W, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    M, K = x.shape
    N = W.shape[1]
    y = np.empty((M, N), np.float64)
    cache = np.empty_like(x)
    L.gt_affine_forward(x.ctypes.data, M, K, W.ctypes.data, b.ctypes.data, N, y.ctypes.data,
                        cache.ctypes.data, int(workers))
    return y


ORC = dict(IDCT=1, BATCHNORM=2, CONV=3, TDNNF=4, LINEAR=5, PREFINAL=6, OUTPUT=7, ATTENTION=8, COMBINE=9)
ROUND_NONE, ROUND_FUSED, ROUND_REF = 0, 1, 2

_fp = C.POINTER(C.c_float)


class OrcBN(C.Structure):
    _fields_ = [("mean", _fp), ("var", _fp), ("gamma", _fp), ("beta", _fp),
                ("eps", C.c_float), ("target_rms", C.c_float)]


class OrcLayer(C.Structure):
    _fields_ = [("type", C.c_int), ("input", C.c_int), ("in_dim", C.c_int), ("out_dim", C.c_int),
                ("hin", C.c_int), ("hout", C.c_int), ("sub", C.c_int), ("fin", C.c_int),
                ("fout", C.c_int), ("noff", C.c_int), ("toff", C.c_int * 9), ("hoff", C.c_int * 9),
                ("bn_dim", C.c_int), ("stride", C.c_int), ("bypass", C.c_float),
                ("small_dim", C.c_int), ("big_dim", C.c_int),
                ("W", _fp), ("b", _fp), ("W2", _fp), ("b2", _fp), ("bn", OrcBN), ("bn2", OrcBN),
                ("log_softmax", C.c_int), ("heads", C.c_int), ("kd", C.c_int), ("vd", C.c_int),
                ("ctx", C.c_int), ("nleft", C.c_int), ("astride", C.c_int), ("key_scale", C.c_float),
                ("input2", C.c_int), ("per_seq", C.c_int), ("height", C.c_int), ("nf1", C.c_int),
                ("nf2", C.c_int)]


class OrcNet(C.Structure):
    _fields_ = [("nlayers", C.c_int), ("layers", C.POINTER(OrcLayer)), ("T", C.c_int),
                ("feat_dim", C.c_int), ("round_mode", C.c_int),
                ("act", C.POINTER(_fp)), ("mask", C.POINTER(C.POINTER(C.c_uint8))),
                ("aux", C.POINTER(_fp)), ("gW", C.POINTER(_fp)), ("gb", C.POINTER(_fp)),
                ("gW2", C.POINTER(_fp)), ("gb2", C.POINTER(_fp)), ("gact", C.POINTER(_fp)),
                ("force_mask", C.POINTER(C.POINTER(C.c_uint8))), ("mx8", C.c_int),
                ("act8", C.POINTER(_fp)), ("ivec", _fp), ("B", C.c_int), ("ivec_dim", C.c_int),
                ("seq_off", C.POINTER(C.c_int)), ("feat8", _fp), ("implicit_dz", C.c_int)]


def parse_xconfig(text: str):
    """Minimal restatement of xconfig.go + layers.go for the layer kinds in configs/."""
    layers, dims, prev = [], {}, None
    for raw in text.splitlines():
        line = raw.strip()
        if not line or line.startswith("#"):
            continue
        import re as _re
        line = _re.sub(r"\(([^)]*)\)", lambda m: "(" + m.group(1).replace(" ", "") + ")", line)
        toks = line.split()
        kind, kv = toks[0], dict(t.split("=", 1) for t in toks[1:] if "=" in t)
        name = kv.get("name")
        inp = kv.get("input", prev)
        if kind == "input":
            dims[name] = int(kv["dim"])
            prev = name
            continue
        inp2, parts = None, None
        if inp.startswith("Append(") and inp.endswith(")"):       # xconfig.go:304-313
            parts = inp[7:-1].split(",")
            inp, inp2 = parts[0], parts[1]
            din = sum(dims[q] for q in parts)
        else:
            if inp.startswith("ReplaceIndex(") and inp.endswith(")"):   # xconfig.go:315-320
                inp = inp[13:-1].split(",")[0]
            din = dims[inp]
        if parts is not None and kind != "combine-feature-maps-layer":
            # general Append (forward.go:264-310): a hidden height-1 combine node per
            # further part, the same graph the product builds (host/network.cpp)
            cur = parts[0]
            for k in range(1, len(parts)):
                hn = name + ".append" + (str(k) if len(parts) > 2 else "")
                layers.append(dict(kind="combine-feature-maps-layer", name=hn, input=cur, input2=parts[k],
                                   in_dim=dims[cur] + dims[parts[k]], out_dim=dims[cur] + dims[parts[k]],
                                   height=1, nf1=dims[cur], nf2=dims[parts[k]], kv={}, hidden=True))
                dims[hn] = dims[cur] + dims[parts[k]]
                cur = hn
            inp, inp2 = cur, None
        L = dict(kind=kind, name=name, input=inp, input2=inp2, in_dim=din, kv=kv)
        if kind == "idct-layer":
            L["out_dim"] = int(kv.get("dim", din))
        elif kind == "batchnorm-component":
            L["out_dim"] = din
        elif kind == "conv-relu-batchnorm-layer":
            hin = int(kv["height-in"])
            L.update(hin=hin, hout=int(kv.get("height-out", hin)), sub=int(kv.get("height-subsample-out", 1)),
                     fout=int(kv["num-filters-out"]), fin=din // hin,
                     toffs=[int(x) for x in kv["time-offsets"].split(",")],
                     hoffs=[int(x) for x in kv["height-offsets"].split(",")])
            L["out_dim"] = L["hout"] * L["fout"]
        elif kind == "tdnnf-layer":
            L.update(out_dim=int(kv["dim"]), bn_dim=int(kv["bottleneck-dim"]),
                     stride=int(kv.get("time-stride", 3)), bypass=float(kv.get("bypass-scale", 0.66)))
        elif kind == "linear-component":
            L["out_dim"] = int(kv["dim"])
        elif kind == "prefinal-layer":
            L.update(small_dim=int(kv["small-dim"]), big_dim=int(kv["big-dim"]), out_dim=int(kv["small-dim"]))
        elif kind == "output-layer":
            L["out_dim"] = int(kv["dim"])
        elif kind == "combine-feature-maps-layer":       # layers.go:240-251
            L.update(out_dim=din, height=int(kv["height"]), nf1=int(kv.get("num-filters1", 1)),
                     nf2=int(kv.get("num-filters2", 1)))
        elif kind == "attention-relu-batchnorm-layer":   # layers.go:298-321
            nl_, nr_ = int(kv.get("num-left-inputs", 0)), int(kv.get("num-right-inputs", 0))
            L.update(heads=int(kv.get("num-heads", 1)), kd=int(kv.get("key-dim", 0)), vd=int(kv.get("value-dim", 0)),
                     nleft=nl_, ctx=1 + nl_ + nr_, astride=int(kv.get("time-stride", 1)))
            L["key_scale"] = float(kv.get("key-scale", 0)) or 1.0 / np.sqrt(L["kd"])
            L["out_dim"] = L["heads"] * (L["vd"] + L["ctx"])
        else:
            raise ValueError(f"oracle: unsupported layer kind {kind}")
        dims[name] = L["out_dim"]
        prev = name
        layers.append(L)
    return layers


def idct_matrix(dim: int, lifter: float) -> np.ndarray:
    """makeIDCTMatrix, forward.go:1190-1210 (float64 then float32)."""
    m = np.zeros((dim, dim), np.float64)
    for i in range(dim):
        for j in range(dim):
            v = np.cos(np.pi * j * (i + 0.5) / dim) * (np.sqrt(1.0 / dim) if j == 0 else np.sqrt(2.0 / dim))
            if lifter > 0 and j > 0:
                v *= 1.0 + (lifter / 2.0) * np.sin(np.pi * j / lifter)
            m[i, j] = v
    return m.astype(np.float32)


def trunc_fp16_vals(a):
    from_bits = np.vectorize(lambda x: lib().orc_f32_to_f16_trunc(float(x)), otypes=[np.uint16])
    return from_bits(np.asarray(a, np.float32)).view(np.float16).astype(np.float32)


class OracleNet:
    """The CPU restatement of Network.Forward / Backward on given parameters.

    params: name -> fp32 array, already fp16-representable (truncated) values;
    bns: (layer, which) -> (mean, var, gamma, beta)."""

    def __init__(self, xconfig: str, params: dict, bns: dict, round_mode=ROUND_FUSED, threads=None,
                 mx8=False, implicit_dz=False):
        self.L = parse_xconfig(xconfig)
        self.keep = []
        index = {"ivector": -2}
        arr = (OrcLayer * len(self.L))()
        per_seq = set()
        for i, L in enumerate(self.L):
            o = arr[i]
            o.input = index.get(L["input"], -1)
            o.input2 = index.get(L["input2"], -1) if L.get("input2") else -100
            if L.get("input2") is None and (o.input == -2 or o.input in per_seq):
                o.per_seq = 1
                per_seq.add(i)
            if L["kind"] == "combine-feature-maps-layer":
                o.type = ORC["COMBINE"]
                o.height, o.nf1, o.nf2 = L["height"], L["nf1"], L["nf2"]
            o.in_dim, o.out_dim = L["in_dim"], L["out_dim"]
            kind = L["kind"]
            if kind == "idct-layer":
                o.type = ORC["IDCT"]
                M = trunc_fp16_vals(idct_matrix(L["out_dim"], float(L["kv"].get("cepstral-lifter", 22))))
                o.W = self._p(M)
            elif kind == "batchnorm-component":
                o.type = ORC["BATCHNORM"]
                o.bn = self._bn(bns.get((L["name"], 0)), L["out_dim"], float(L["kv"].get("target-rms", 1.0)))
            elif kind == "conv-relu-batchnorm-layer":
                o.type = ORC["CONV"]
                offs = [(a, b) for a in L["toffs"] for b in L["hoffs"]]
                o.hin, o.hout, o.sub, o.fin, o.fout, o.noff = L["hin"], L["hout"], L["sub"], L["fin"], L["fout"], len(offs)
                for k, (a, b) in enumerate(offs):
                    o.toff[k], o.hoff[k] = a, b
                o.W, o.b = self._p(params[L["name"] + ".W"]), self._p(params[L["name"] + ".Bias"])
                o.bn = self._bn(bns.get((L["name"], 0)), L["fout"])
            elif kind == "tdnnf-layer":
                o.type = ORC["TDNNF"]
                o.bn_dim, o.stride, o.bypass = L["bn_dim"], L["stride"], L["bypass"]
                n = L["name"]
                o.W, o.W2, o.b2 = self._p(params[n + ".LinearW"]), self._p(params[n + ".AffineW"]), self._p(params[n + ".AffineBias"])
                o.bn = self._bn(bns.get((n, 0)), L["out_dim"])
            elif kind == "linear-component":
                o.type = ORC["LINEAR"]
                o.W = self._p(params[L["name"] + ".W"])
            elif kind == "prefinal-layer":
                o.type = ORC["PREFINAL"]
                n = L["name"]
                o.small_dim, o.big_dim = L["small_dim"], L["big_dim"]
                o.W, o.b, o.W2 = self._p(params[n + ".BigW"]), self._p(params[n + ".BigBias"]), self._p(params[n + ".SmallW"])
                o.bn = self._bn(bns.get((n, 0)), L["big_dim"])
                if (n, 1) in bns:
                    o.bn2 = self._bn(bns[(n, 1)], L["small_dim"])
            elif kind == "attention-relu-batchnorm-layer":
                o.type = ORC["ATTENTION"]
                o.heads, o.kd, o.vd, o.ctx, o.nleft, o.astride = L["heads"], L["kd"], L["vd"], L["ctx"], L["nleft"], L["astride"]
                o.key_scale = np.float32(L["key_scale"])
                o.W, o.b = self._p(params[L["name"] + ".W"]), self._p(params[L["name"] + ".Bias"])
                o.bn = self._bn(bns.get((L["name"], 0)), L["out_dim"])
            elif kind == "output-layer":
                o.type = ORC["OUTPUT"]
                o.W, o.b = self._p(params[L["name"] + ".W"]), self._p(params[L["name"] + ".Bias"])
                # layers.go:345: include-log-softmax defaults to true
                o.log_softmax = int(L["kv"].get("include-log-softmax", "true").lower() in ("true", "1", "t"))
            index[L["name"]] = i
        self.arr = arr
        self.index = index
        self.round_mode = round_mode
        self.mx8 = int(mx8)    # emulate the GPU's MXFP8 step (kf_nnet.h nnet_set_fp8: 1, or 2 = fp16 backward)
        # F mode: the GPU's implicit TDNN-F dz (kf_nnet.h nnet_set_implicit_dz, default off)
        self.implicit_dz = int(implicit_dz)
        if threads:
            lib().orc_set_threads(int(threads))
        self.net = None

    def _p(self, a):
        a = np.ascontiguousarray(a, dtype=np.float32)
        self.keep.append(a)
        return a.ctypes.data_as(_fp)

    def _bn(self, spec, dim, target_rms=1.0):
        if spec is None:
            spec = (np.zeros(dim, np.float32), np.ones(dim, np.float32), np.ones(dim, np.float32), np.zeros(dim, np.float32))
        m, v, g, b = spec
        return OrcBN(self._p(m), self._p(v), self._p(g), self._p(b), 1e-3, target_rms)

    def forward(self, features: np.ndarray, force_masks: dict = None, ivectors=None, seq_off=None,
                features8: np.ndarray = None):
        """force_masks: layer name -> uint8 ReLU decisions to replay (see kf_oracle.h).
        ivectors [B x dim] and seq_off int[B+1]: the ivector input (ReplaceIndex rows).
        features8: the features' dequantised MXFP8 copy, the GEMM input of a layer reading
        the input directly when mx8 is on (one-layer tests on the GPU's own fp8 input)."""
        x = np.ascontiguousarray(features, dtype=np.float32)
        fm = None
        if force_masks:
            fm = (C.POINTER(C.c_uint8) * len(self.L))()
            for name, m in force_masks.items():
                m = np.ascontiguousarray(m, dtype=np.uint8)
                self.keep.append(m)
                fm[self.index[name]] = m.ctypes.data_as(C.POINTER(C.c_uint8))
            self.keep.append(fm)
        self.x = x
        if self.net is not None:
            lib().orc_net_free(C.byref(self.net))
        self.net = OrcNet()
        self.net.nlayers = len(self.L)
        self.net.layers = self.arr
        self.net.T = x.shape[0]
        self.net.feat_dim = x.shape[1]
        self.net.round_mode = self.round_mode
        self.net.mx8 = int(self.mx8)   # 1: MX forward + MX strided affine dgrad; 2: MX forward only
        self.net.implicit_dz = int(self.implicit_dz)
        if ivectors is not None:
            iv = np.ascontiguousarray(ivectors, dtype=np.float32)
            so = np.ascontiguousarray(seq_off, dtype=np.int32)
            self.keep += [iv, so]
            self.net.ivec = iv.ctypes.data_as(_fp)
            self.net.B, self.net.ivec_dim = iv.shape
            self.net.seq_off = so.ctypes.data_as(C.POINTER(C.c_int))
        if fm is not None:
            self.net.force_mask = fm
        if features8 is not None:
            f8 = np.ascontiguousarray(features8, dtype=np.float32)
            assert f8.shape == x.shape
            self.keep.append(f8)
            self.net.feat8 = f8.ctypes.data_as(_fp)
        rc = lib().orc_net_forward(C.byref(self.net), x.ctypes.data)
        assert rc == 0

    def act(self, name):
        i = self.index[name]
        T, d = (self.net.B if self.arr[i].per_seq else self.net.T), self.L[i]["out_dim"]
        return np.ctypeslib.as_array(self.net.act[i], shape=(T * d,)).reshape(T, d).copy()

    def mask(self, name):
        i = self.index[name]
        L = self.L[i]
        width = L["big_dim"] if L["kind"] == "prefinal-layer" else L["out_dim"]
        p = self.net.mask[i]
        return None if not p else np.ctypeslib.as_array(p, shape=(self.net.T * width,)).copy()

    def chain_output(self) -> int:
        """Model.ChainOutput (model.go:271-281): the output layer named "output", else the first."""
        outs = [i for i, L in enumerate(self.L) if L["kind"] == "output-layer"]
        for i in outs:
            if self.L[i]["name"] == "output":
                return i
        return outs[0] if outs else len(self.L) - 1

    def backward(self, out_grad: np.ndarray):
        g = np.ascontiguousarray(out_grad, dtype=np.float32)
        rc = lib().orc_net_backward_top(C.byref(self.net), self.x.ctypes.data, g.ctypes.data, self.chain_output())
        assert rc == 0

    def grads(self) -> dict:
        """Gradients keyed by the product's parameter names."""
        out = {}
        T = self.net.T

        def get(ptrs, i, n):
            p = ptrs[i]  # no gradient reached the layer (off the chain-output path): zeros
            return np.zeros(n, np.float32) if not p else np.ctypeslib.as_array(p, shape=(n,)).copy()

        for i, L in enumerate(self.L):
            k, n = L["kind"], L["name"]
            if k == "conv-relu-batchnorm-layer":
                K = len(L["toffs"]) * len(L["hoffs"]) * L["fin"]
                out[n + ".W"] = get(self.net.gW, i, K * L["fout"]).reshape(K, L["fout"])
                out[n + ".Bias"] = get(self.net.gb, i, L["fout"]).reshape(1, -1)
            elif k == "tdnnf-layer":
                s, din, bn, dout = L["stride"], L["in_dim"], L["bn_dim"], L["out_dim"]
                kl, ka = (2 * din if s > 0 else din), (2 * bn if s > 0 else bn)
                out[n + ".LinearW"] = get(self.net.gW, i, kl * bn).reshape(kl, bn)
                out[n + ".AffineW"] = get(self.net.gW2, i, ka * dout).reshape(ka, dout)
                out[n + ".AffineBias"] = get(self.net.gb2, i, dout).reshape(1, -1)
            elif k == "linear-component":
                out[n + ".W"] = get(self.net.gW, i, L["in_dim"] * L["out_dim"]).reshape(L["in_dim"], L["out_dim"])
            elif k == "prefinal-layer":
                big, small, din = L["big_dim"], L["small_dim"], L["in_dim"]
                out[n + ".BigW"] = get(self.net.gW, i, din * big).reshape(din, big)
                out[n + ".BigBias"] = get(self.net.gb, i, big).reshape(1, -1)
                out[n + ".SmallW"] = get(self.net.gW2, i, big * small).reshape(big, small)
            elif k == "attention-relu-batchnorm-layer":
                A = L["heads"] * (2 * L["kd"] + L["vd"] + L["ctx"])
                out[n + ".W"] = get(self.net.gW, i, L["in_dim"] * A).reshape(L["in_dim"], A)
                out[n + ".Bias"] = get(self.net.gb, i, A).reshape(1, -1)
            elif k == "output-layer":
                out[n + ".W"] = get(self.net.gW, i, L["in_dim"] * L["out_dim"]).reshape(L["in_dim"], L["out_dim"])
                out[n + ".Bias"] = get(self.net.gb, i, L["out_dim"]).reshape(1, -1)
        return out

    def close(self):
        if self.net is not None:
            lib().orc_net_free(C.byref(self.net))
            self.net = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class GotorchNet:
    """The network in the reference's Go CPU style (oracle/gotorch_net.c):
    float64, AffineLayer / TDNNLayer / Conv1DLayer loop forms, matmulParallel forward
    GEMMs over `workers` threads, SGD with momentum. Built from an OracleNet's layer
    descriptors and parameters (fp32 values widened to float64)."""

    def __init__(self, onet: "OracleNet", workers: int = 1):
        self.o = onet
        self.workers = int(workers)
        self.h = lib().gt_net_create(C.cast(onet.arr, C.c_void_p), len(onet.L))
        if not self.h:
            raise ValueError("gotorch template: unsupported layer (attention / combine / ivector branch)")

    def forward(self, features: np.ndarray):
        self.x = np.ascontiguousarray(features, dtype=np.float64)
        assert lib().gt_net_forward(self.h, self.x.ctypes.data, self.x.shape[0], self.workers) == 0

    def _t(self, name, which):
        n = C.c_longlong(0)
        p = lib().gt_net_tensor(self.h, self.o.index[name], which, C.byref(n))
        return None if not p else np.ctypeslib.as_array(p, shape=(n.value,)).copy()

    def act(self, name):
        return self._t(name, 0).reshape(self.x.shape[0], -1)

    def backward(self, out_grad: np.ndarray):
        g = np.ascontiguousarray(out_grad, dtype=np.float64)
        assert lib().gt_net_backward(self.h, self.x.ctypes.data, g.ctypes.data, self.o.chain_output()) == 0

    def sgd(self, lr, momentum=0.9):
        lib().gt_net_sgd(self.h, lr, momentum)

    def grads(self) -> dict:
        """flat float64 gradients under the product's parameter names (OracleNet.grads())"""
        out = {}
        for L in self.o.L:
            n, k = L["name"], L["kind"]
            names = {"conv-relu-batchnorm-layer": [(".W", 1), (".Bias", 2)],
                     "tdnnf-layer": [(".LinearW", 1), (".AffineW", 3), (".AffineBias", 4)],
                     "linear-component": [(".W", 1)],
                     "prefinal-layer": [(".BigW", 1), (".BigBias", 2), (".SmallW", 3)],
                     "output-layer": [(".W", 1), (".Bias", 2)]}.get(k, [])
            for suf, which in names:
                out[n + suf] = self._t(n, which)
        return out

    def close(self):
        if self.h:
            lib().gt_net_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------- chain objective
_ip = C.POINTER(C.c_int)


class OrcDen(C.Structure):
    _fields_ = [("S", C.c_int), ("P", C.c_int), ("A", C.c_int), ("src", _ip), ("dst", _ip),
                ("pdf0", _ip), ("tp", _fp), ("init", _fp)]


class OrcNum(C.Structure):
    _fields_ = [("S", C.c_int), ("A", C.c_int), ("nfinal", C.c_int), ("start", C.c_int),
                ("row_ptr", _ip), ("dst", _ip), ("pdf1", _ip), ("logw", _fp),
                ("final_state", _ip), ("final_w", _fp)]


class OrcChainOpts(C.Structure):
    _fields_ = [("l2_regularize", C.c_float), ("out_of_range_regularize", C.c_float),
                ("leaky_hmm_coefficient", C.c_float), ("xent_regularize", C.c_float),
                ("supervision_weight", C.c_float)]


class OrcChainResult(C.Structure):
    _fields_ = [("objf", C.c_double), ("l2_term", C.c_double), ("total_weight", C.c_double),
                ("num_logprob", C.c_double), ("den_logprob", C.c_double), ("frames", C.c_int),
                ("out_of_range", C.c_int), ("ok", C.c_int)]


def _chain_sigs(L):
    if getattr(L, "_chain_sigs", False):
        return L
    L.orc_den_initial_probs.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_int, C.c_void_p]
    L.orc_den_forward_backward.restype = C.c_float
    L.orc_den_forward_backward.argtypes = [C.POINTER(OrcDen), C.c_void_p, C.c_int, C.c_float,
                                           C.c_void_p]
    L.orc_num_forward_backward.restype = C.c_float
    L.orc_num_forward_backward.argtypes = [C.POINTER(OrcNum), C.c_void_p, C.c_int, C.c_int,
                                           C.c_void_p]
    L.orc_chain_objf.argtypes = [C.POINTER(OrcChainOpts), C.POINTER(OrcDen), C.POINTER(OrcNum),
                                 C.c_void_p, C.c_int, C.c_void_p, C.POINTER(OrcChainResult)]
    L._chain_sigs = True
    return L


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def _ptr(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def den_initial_probs(g: dict) -> np.ndarray:
    """denominator.go:131-171 on a synth.make_den_graph dict."""
    L = _chain_sigs(lib())
    src, dst, tp = _c(g["src"], np.int32), _c(g["dst"], np.int32), _c(g["tp"], np.float32)
    out = np.empty(int(g["S"]), np.float32)
    L.orc_den_initial_probs(int(g["S"]), int(g["A"]), src.ctypes.data, dst.ctypes.data,
                            tp.ctypes.data, int(g["start"]), out.ctypes.data)
    return out


def _den_struct(g, init):
    keep = [_c(g["src"], np.int32), _c(g["dst"], np.int32), _c(g["pdf0"], np.int32),
            _c(g["tp"], np.float32), _c(init, np.float32)]
    d = OrcDen(int(g["S"]), int(g["P"]), int(g["A"]), _ptr(keep[0], C.c_int), _ptr(keep[1], C.c_int),
               _ptr(keep[2], C.c_int), _ptr(keep[3], C.c_float), _ptr(keep[4], C.c_float))
    return d, keep


def _num_struct(f):
    keep = [_c(f["row_ptr"], np.int32), _c(f["dst"], np.int32), _c(f["pdf1"], np.int32),
            _c(f["logw"], np.float32), _c(f["final_state"], np.int32), _c(f["final_w"], np.float32)]
    n = OrcNum(int(f["S"]), int(f["A"]), len(keep[4]), int(f.get("start", 0)),
               _ptr(keep[0], C.c_int), _ptr(keep[1], C.c_int), _ptr(keep[2], C.c_int),
               _ptr(keep[3], C.c_float), _ptr(keep[4], C.c_int), _ptr(keep[5], C.c_float))
    return n, keep


def den_forward_backward(g: dict, init, nnet: np.ndarray, leaky=1e-5, posteriors=True):
    """chain_den.cu:496-706 (den_forward when posteriors=False). Returns (logprob, post)."""
    L = _chain_sigs(lib())
    d, keep = _den_struct(g, init)
    x = _c(nnet, np.float32)
    T = x.shape[0]
    post = np.empty_like(x) if posteriors else None
    lp = L.orc_den_forward_backward(C.byref(d), x.ctypes.data, T, leaky,
                                    post.ctypes.data if posteriors else None)
    return float(lp), post


def num_forward_backward(f: dict, nnet: np.ndarray, posteriors=True):
    """chain_det.cu:55-237 on nnet values used as given. Returns (logprob, post)."""
    L = _chain_sigs(lib())
    n, keep = _num_struct(f)
    x = _c(nnet, np.float32)
    T, P = x.shape
    post = np.empty_like(x) if posteriors else None
    lp = L.orc_num_forward_backward(C.byref(n), x.ctypes.data, T, P,
                                    post.ctypes.data if posteriors else None)
    return float(lp), post


def chain_objf(g: dict, init, f: dict, nnet: np.ndarray, l2=0.0, oor=0.01, leaky=1e-5, weight=1.0):
    """ComputeChainObjfAndDeriv for one sequence (backward.go:224-371).
    Returns (deriv [T x P], result dict)."""
    L = _chain_sigs(lib())
    d, k1 = _den_struct(g, init)
    n, k2 = _num_struct(f)
    x = _c(nnet, np.float32)
    T = x.shape[0]
    deriv = np.empty_like(x)
    r = OrcChainResult()
    o = OrcChainOpts(l2, oor, leaky, 0.0, weight)
    L.orc_chain_objf(C.byref(o), C.byref(d), C.byref(n), x.ctypes.data, T, deriv.ctypes.data, C.byref(r))
    res = {k: getattr(r, k) for k, _ in OrcChainResult._fields_}
    return deriv, res


def mx_qdq_rows(x: np.ndarray) -> np.ndarray:
    """OCP MXFP8 quantise-dequantise of each row (blocks of 32), the oracle's rule"""
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.empty_like(x)
    lib().orc_mx_qdq_rows(x.ctypes.data, y.ctypes.data, x.shape[0], x.shape[1])
    return y
