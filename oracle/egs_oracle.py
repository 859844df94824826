"""TEST INFRASTRUCTURE ONLY — numpy restatement of the reference's matrix decompression
(internal/parser/matrix.go:10-168) used as the checker for the egs reader's host
decompression and for the GPU expansion kernel (csrc/egs.hip). Only tests/ may import
this module.

Every float32 operation is a separate numpy float32 op, in the reference's order (Go on
amd64 rounds each float32 op, no contraction):
  uint16ToFloat  matrix.go:11-14   min + (range * f32(1/65535)) * f32(v)
  charToFloat    matrix.go:17-26   three linear pieces, the last divides in float64
  CM2            matrix.go:100-108 min + f32(v) * (range / 65535)
  CM3            matrix.go:131-138 min + f32(v) * (range / 255)
  FM             matrix.go:158-164 raw float32
Parity status: the formulas are pinned by the reference's source only (the reference
ships no compressed-matrix test vectors and no egs file).
"""
from __future__ import annotations

import numpy as np

F = np.float32


def u16_to_float(mn, rg, v):
    v = np.asarray(v, np.uint16).astype(F)
    return F(mn) + (F(rg) * F(1.52590218966964e-05)) * v


def char_to_float(p0, p25, p75, p100, v):
    v = np.asarray(v, np.uint8)
    vf = v.astype(F)
    a = p0 + ((p25 - p0) * vf) * F(1.0 / 64.0)
    b = p25 + ((p75 - p25) * (vf - F(64))) * F(1.0 / 128.0)
    prod = ((p100 - p75) * (vf - F(192))).astype(F)
    c = (p75.astype(np.float64) + prod.astype(np.float64) / 63.0).astype(F)
    return np.where(v <= 64, a, np.where(v <= 192, b, c)).astype(F)


def decompress(kind: str, rows: int, cols: int, mn, rg, payload: bytes) -> np.ndarray:
    """fp32 [rows, cols] row-major, as matrix.go produces it."""
    if kind == "CM":
        hdr = np.frombuffer(payload, "<u2", count=4 * cols).reshape(cols, 4)
        p = [u16_to_float(mn, rg, hdr[:, k])[None, :] for k in range(4)]  # [1, cols]
        data = np.frombuffer(payload, np.uint8, count=rows * cols, offset=8 * cols).reshape(cols, rows).T
        return char_to_float(p[0], p[1], p[2], p[3], data)
    if kind == "CM2":
        v = np.frombuffer(payload, "<u2", count=rows * cols).astype(F)
        return (F(mn) + v * (F(rg) / F(65535.0))).reshape(rows, cols)
    if kind == "CM3":
        v = np.frombuffer(payload, np.uint8, count=rows * cols).astype(F)
        return (F(mn) + v * (F(rg) / F(255.0))).reshape(rows, cols)
    if kind == "FM":
        return np.frombuffer(payload, "<f4", count=rows * cols).reshape(rows, cols).astype(F)
    raise ValueError(kind)


def merge_features(metas) -> np.ndarray:
    """batch.NewBatch feature merge (batch.go:93-105)."""
    return np.concatenate([decompress(m["kind"], m["rows"], m["cols"], m["min"], m["range"], m["payload"])
                           for m in metas], axis=0)
