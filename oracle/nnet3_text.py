"""TEST INFRASTRUCTURE ONLY — pure-Python restatement of the reference's nnet3 text
parser, ParseNnet3Text (internal/nnet/weight_loader.go:608-727, helpers :1118-1216),
used as the checker for kf_nnet3_parse_text (host/nnet3_import.cpp). Only tests/ may
import it. Pinned by the reference's own fixtures (tests/golden/nnet3_*.txt, extracted
from weight_loader_test.go) and the expectations of that test file.
"""
from __future__ import annotations

import math
import re

import numpy as np

_FLOAT = re.compile(r"^[+-]?((\d+(\.\d*)?|\.\d+)([eE][+-]?\d+)?|inf|infinity|nan)$", re.I)
TAGS = ("<LinearParams>", "<Params>", "<BiasParams>", "<StatsMean>", "<StatsVar>")


def parse_f32(tok):
    """strconv.ParseFloat(tok, 32): (value, ok, range_error)."""
    if not _FLOAT.match(tok):
        return 0.0, False, False
    with np.errstate(over="ignore"):
        v = np.float32(float(tok))  # decimal -> double -> float32: exact for <= 9 significant digits
    rng = bool(np.isinf(v)) and tok.lower().lstrip("+-") not in ("inf", "infinity")
    return float(v), True, rng


def parse_float_line(line):
    out = []
    for f in line.split():
        v, ok, rng = parse_f32(f)
        if ok and not rng:
            out.append(v)
    return out


def _tag_field(line, tag):
    i = line.find(tag)
    if i < 0:
        return None
    fs = line[i + len(tag):].split()
    if not fs or fs[0].startswith("<"):
        return None
    return fs[0]


def tag_f32(line, tag):
    t = _tag_field(line, tag)
    if t is None:
        return 0.0
    v, ok, _ = parse_f32(t)
    return v if ok else 0.0


def tag_f64(line, tag):
    t = _tag_field(line, tag)
    if t is None or not _FLOAT.match(t):
        return 0.0
    return float(t)


def tag_int(line, tag):
    t = _tag_field(line, tag)
    if t is None or not re.match(r"^[+-]?\d+$", t):
        return 0
    v = int(t)
    return v if -2**31 <= v < 2**31 else 0


def new_comp(line):
    c = dict(name="", type="", linear=[], rows=0, cols=0, bias=[], mean=[], var=[], count=0.0,
             eps=0.0, rms=0.0, lr=0.0, maxc=0.0, l2=0.0, nfi=0, nfo=0, hin=0, hout=0)
    i = line.find("<ComponentName>")
    parts = line[i + len("<ComponentName>"):].split()
    if len(parts) < 2:
        return c
    c["name"], c["type"] = parts[0], parts[1].strip("<>")
    c.update(lr=tag_f32(line, "<LearningRate>"), maxc=tag_f32(line, "<MaxChange>"),
             l2=tag_f32(line, "<L2Regularize>"), eps=tag_f32(line, "<Epsilon>"),
             rms=tag_f32(line, "<TargetRms>"), count=tag_f64(line, "<Count>"),
             nfi=tag_int(line, "<NumFiltersIn>"), nfo=tag_int(line, "<NumFiltersOut>"),
             hin=tag_int(line, "<HeightIn>"), hout=tag_int(line, "<HeightOut>"))
    return c


def _finish(c, tag, data, rows):
    if not data:
        return
    cols = len(data) // rows if rows > 0 else 0
    if tag in ("<LinearParams>", "<Params>"):
        c["linear"], c["rows"], c["cols"] = list(data), rows, cols
    elif tag == "<BiasParams>":
        c["bias"] = list(data)
    elif tag == "<StatsMean>":
        c["mean"] = list(data)
    elif tag == "<StatsVar>":
        c["var"] = list(data)


def parse(text: str) -> dict:
    """name -> component dict (the last definition of a name wins)."""
    comps, cur = {}, None
    buf, rows, in_m, tag = [], 0, False, ""
    for line in text.split("\n"):
        if line.endswith("\r"):
            line = line[:-1]
        if "<ComponentName>" in line:
            if cur is not None and in_m:
                _finish(cur, tag, buf, rows)
            if cur is not None:
                comps[cur["name"]] = cur
            cur = new_comp(line)
            buf, rows, in_m, tag = [], 0, False, ""
        if cur is None:
            continue
        if "<Count>" in line:
            cur["count"] = tag_f64(line, "<Count>")
        if "<Epsilon>" in line and cur["eps"] == 0:
            cur["eps"] = tag_f32(line, "<Epsilon>")
        if "<TargetRms>" in line and cur["rms"] == 0:
            cur["rms"] = tag_f32(line, "<TargetRms>")
        for t in TAGS:
            if t not in line:
                continue
            if in_m:
                _finish(cur, tag, buf, rows)
            tag, buf, rows, in_m = t, [], 0, True
            b = line.find("[")
            if b >= 0:
                after = line[b + 1:]
                if "]" in after:
                    vals = parse_float_line(after[:after.index("]")])
                    if vals:
                        buf, rows = vals, 1
                    _finish(cur, tag, buf, rows)
                    in_m = False
            break
        if in_m and "<" not in line:
            s = line.strip()
            if not s:
                continue
            close = "]" in s
            if close:
                s = s.replace("]", "", 1)
            vals = parse_float_line(s)
            if vals:
                buf = buf + vals
                rows += 1
            if close:
                _finish(cur, tag, buf, rows)
                in_m = False
    if cur is not None:
        if in_m:
            _finish(cur, tag, buf, rows)
        comps[cur["name"]] = cur
    return comps


def replace_bn(mean, var, eps, rms):
    """replaceBN (weight_loader.go:1035-1085): the double-normalising gamma / beta."""
    rms = rms if rms > 0 else 1.0
    eps = np.float32(eps if eps > 0 else 0.001)
    v = np.maximum(np.asarray(var, np.float32), np.float32(0))
    inv = (1.0 / np.sqrt((v + eps).astype(np.float64))).astype(np.float32)
    gamma = (np.float32(rms) * inv).astype(np.float32)
    beta = (-np.asarray(mean, np.float32) * gamma).astype(np.float32)
    return gamma, beta


def write_component(name, ctype, linear=None, bias=None, mean=None, var=None, header="", bn_dim=None,
                    eps=1e-3, rms=1.0, count=1000):
    """nnet3-copy style text of one component (test input generator): matrices are
    [out x in] written with Kaldi's "[\\n rows ... ]" layout, vectors inline."""
    fmt = lambda a: " ".join(repr(float(np.float32(x))) for x in a)
    if ctype == "BatchNormComponent":
        return (f"<ComponentName> {name} <BatchNormComponent> <Dim> {bn_dim} <BlockDim> {bn_dim} "
                f"<Epsilon> {eps} <TargetRms> {rms} <TestMode> F <Count> {count} <StatsMean>  [ {fmt(mean)} ]\n"
                f"<StatsVar>  [ {fmt(var)} ]\n")
    out = [f"<ComponentName> {name} <{ctype}> {header}<LinearParams>  [\n"]
    lin = np.asarray(linear, np.float32)
    for r in range(lin.shape[0]):
        out.append("  " + fmt(lin[r]) + (" ]\n" if r == lin.shape[0] - 1 else "\n"))
    if bias is not None:
        out.append(f"<BiasParams>  [ {fmt(bias)} ]\n")
    return "".join(out)
