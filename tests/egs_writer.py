"""Test infrastructure: writes Kaldi chain egs (binary ark) byte streams.

Byte layout follows what Kaldi's writers emit (NnetChainExample::Write, NnetIo::Write,
CompressedMatrix::Write, chain::Supervision::Write with an StdCompactAcceptorFst,
Vector::Write for <DW2>) as the reference's reader consumes it
(internal/parser/parser.go:163-302, fst.go, matrix.go, docs/kaldi-egs-format.md). Two
conventions are the reference reader's rather than Kaldi's and are written the
reader's way, because the reader is what is being restated:
  * long-form index entries (byte 127) carry three " \\x04<int32>" values
    (parser_edge_test.go:103-121; Kaldi writes "\\x04<int32>" without the space);
  * FM is "FM " + size byte + raw int32 rows + raw int32 cols (parser.go:369-383).
No real egs file exists in the reference, so every test ark is generated here.
"""
from __future__ import annotations

import gzip
import struct

import numpy as np

FST_MAGIC = 0x7EB2FDD6


def i32(v):
    return struct.pack("<i", int(v))


def u32(v):
    return struct.pack("<I", int(v))


def f32(v):
    return struct.pack("<f", float(v))


def basic_int(v):
    """WriteBasicType<int32> after a token: the token's trailing space + size + value."""
    return b" \x04" + i32(v)


def basic_float(v):
    return b" \x04" + f32(v)


def index_vector(idx):
    """<I1V> + count + delta bytes (parser.go:484-548). idx: [(n, t, x), ...]."""
    out = [b"<I1V>", basic_int(len(idx))]
    prev = None
    for (n, t, x) in idx:
        if prev is None:
            ok = n == 0 and x == 0 and abs(t) < 125
            d = t
        else:
            ok = n == prev[0] and x == prev[2] and abs(t - prev[1]) < 125
            d = t - prev[1]
        if ok:
            out.append(struct.pack("<b", d))
        else:
            out.append(b"\x7f" + basic_int(n) + basic_int(t) + basic_int(x))
        prev = (n, t, x)
    return b"".join(out)


def random_cm(rng, rows, cols):
    """A CM (kOneByteWithColHeaders) matrix: global header + random sorted percentiles
    per column + random column-major bytes. Returns (min, range, payload)."""
    mn = float(rng.uniform(-20, 0))
    rg = float(rng.uniform(1, 40))
    hdr = np.sort(rng.integers(0, 65536, size=(cols, 4)), axis=1).astype("<u2")
    data = rng.integers(0, 256, size=(cols, rows), dtype=np.uint8)  # column-major
    return np.float32(mn), np.float32(rg), hdr.tobytes() + data.tobytes()


def matrix_bytes(kind, rows, cols, mn=0.0, rg=1.0, payload=b""):
    if kind == "FM":
        return b"FM " + b"\x04" + i32(rows) + i32(cols) + payload
    tok = {"CM": b"CM ", "CM2": b"CM2 ", "CM3": b"CM3 "}[kind]
    return tok + f32(mn) + f32(rg) + i32(rows) + i32(cols) + payload


def random_matrix(rng, kind, rows, cols):
    """(bytes, meta) of a random stored matrix of the given kind."""
    if kind == "CM":
        mn, rg, payload = random_cm(rng, rows, cols)
    elif kind == "CM2":
        mn, rg = np.float32(rng.uniform(-5, 0)), np.float32(rng.uniform(1, 10))
        payload = rng.integers(0, 65536, size=rows * cols).astype("<u2").tobytes()
    elif kind == "CM3":
        mn, rg = np.float32(rng.uniform(-5, 0)), np.float32(rng.uniform(1, 10))
        payload = rng.integers(0, 256, size=rows * cols, dtype=np.uint8).tobytes()
    else:
        mn, rg = np.float32(0), np.float32(0)
        payload = rng.standard_normal(rows * cols).astype("<f4").tobytes()
    return matrix_bytes(kind, rows, cols, mn, rg, payload), dict(
        kind=kind, rows=rows, cols=cols, min=mn, range=rg, payload=payload)


def fst_header(fst_type, num_states, num_arcs, start=0, props=0):
    s = lambda x: u32(len(x)) + x.encode()
    return (i32(FST_MAGIC) + s(fst_type) + s("standard") + i32(2 if fst_type == "vector" else 1) + i32(0)
            + struct.pack("<Q", props) + struct.pack("<q", start) + struct.pack("<q", num_states)
            + struct.pack("<q", num_arcs))


def compact_acceptor(states, start=0):
    """states: [(arcs [(label, weight, next)], final or None)] -> compact_acceptor bytes
    (fst.go:64-121): per-state compacts, the final weight as a (0, w, -1) element."""
    offs, comp, narcs = [0], [], 0
    for arcs, final in states:
        for (l, w, n) in arcs:
            comp.append(i32(l) + f32(w) + i32(n))
            narcs += 1
        if final is not None:
            comp.append(i32(0) + f32(final) + i32(-1))
        offs.append(len(comp))
    return (fst_header("compact_acceptor", len(states), narcs, start) + b"".join(u32(o) for o in offs)
            + b"".join(comp))


def vector_fst(states, start=0):
    """VectorFst<StdArc> bytes (fst.go:127-172); header arc count 0 as OpenFst writes."""
    body = []
    for arcs, final in states:
        body.append(f32(np.inf if final is None else final) + struct.pack("<q", len(arcs)))
        for (l, w, n) in arcs:
            body.append(i32(l) + i32(l) + f32(w) + i32(n))
    return fst_header("vector", len(states), 0, start) + b"".join(body)


def random_num_fst(rng, num_states, num_pdfs=3080):
    """A chain numerator-like FST: a self-loop and a forward arc per state, weights
    -log(0.5), labels in [1, num_pdfs], last state final with weight 0."""
    states = []
    for s in range(num_states):
        arcs = [(int(rng.integers(1, num_pdfs + 1)), 0.6931, s)]
        if s + 1 < num_states:
            arcs.append((int(rng.integers(1, num_pdfs + 1)), 0.6931, s + 1))
        states.append((arcs, 0.0 if s == num_states - 1 else None))
    return states


def example_bytes(key, feats, ivec=None, *, weight=1.0, num_sequences=1, frames_per_seq=50,
                  label_dim=3080, fst_states=None, fst_kind="compact", e2e=False, deriv_weights=None,
                  dw_kind="DW2", num_inputs=None, t0=-30, sup_t0=0, input_name="input"):
    """One NnetChainExample in binary ark form. feats / ivec: (bytes, meta) pairs."""
    ins = [(input_name, feats, [(0, t0 + i, 0) for i in range(feats[1]["rows"])])]
    if ivec is not None:
        ins.append(("ivector", ivec, [(0, 0, 0)]))
    out = [key.encode(), b" \x00B", b"<Nnet3ChainEg> ", b"<NumInputs>",
           basic_int(len(ins) if num_inputs is None else num_inputs)]
    for name, (mb, _), idx in ins:
        out += [b"<NnetIo> ", name.encode(), b" ", index_vector(idx), mb, b"</NnetIo> "]
    out += [b"<NumOutputs>", basic_int(1), b"<NnetChainSup> output ",
            index_vector([(0, sup_t0 + 3 * i, 0) for i in range(frames_per_seq)]),
            b"<Supervision> <Weight>", basic_float(weight), b"<NumSequences>", basic_int(num_sequences),
            b"<FramesPerSeq>", basic_int(frames_per_seq), b"<LabelDim>", basic_int(label_dim),
            b"<End2End> ", b"T" if e2e else b"F"]
    if not e2e:
        out.append(compact_acceptor(fst_states) if fst_kind == "compact" else vector_fst(fst_states))
    out.append(b"</Supervision> ")
    if deriv_weights is not None:
        dw = np.asarray(deriv_weights, np.float32)
        if dw_kind == "DW2":
            out += [b"<DW2> FV ", b"\x04", i32(len(dw)), dw.astype("<f4").tobytes()]
        else:  # <DW>: one byte per weight, /255 on read (fst.go:235-249)
            q = np.clip(np.round(dw * 255), 0, 255).astype(np.uint8)
            out += [b"<DW> FV ", i32(len(q)), q.tobytes()]
    out += [b"</NnetChainSup> ", b"</Nnet3ChainEg> "]
    return b"".join(out)


def write_ark(path, examples: list[bytes]):
    data = b"".join(examples)
    if str(path).endswith(".gz"):
        with gzip.open(path, "wb") as f:
            f.write(data)
    else:
        with open(path, "wb") as f:
            f.write(data)


def make_egs(rng, n, *, rows=(150, 203, 224), feat_kind="CM", ivec_kind="CM2", fst_states=(40, 80),
             key_prefix="utt", fps=None, with_ivec=True, num_pdfs=3080, **kw):
    """n random examples: (list of ark bytes, list of per-example metadata)."""
    exs, meta = [], []
    for e in range(n):
        R = int(rows[e % len(rows)])
        feats = random_matrix(rng, feat_kind, R, 40)
        ivec = random_matrix(rng, ivec_kind, 1, 100) if with_ivec else None
        S = int(rng.integers(fst_states[0], fst_states[1] + 1))
        states = random_num_fst(rng, S, num_pdfs)
        key = f"{key_prefix}-{e:04d}"
        f = fps if fps is not None else max(1, (R - 60) // 3)
        exs.append(example_bytes(key, feats, ivec, fst_states=states, frames_per_seq=f, **kw))
        meta.append(dict(key=key, feats=feats[1], ivec=None if ivec is None else ivec[1], states=states, fps=f))
    return exs, meta
