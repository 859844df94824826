"""Oracle fp16 conversions pinned by the reference's known-answer tests
(internal/fp16/fp16_test.go:12-265) and by numpy's independent IEEE RNE."""
import numpy as np
import pytest

import oracle

L = oracle.lib()


@pytest.mark.parametrize("val,bits", [
    (0.0, 0x0000), (-0.0, 0x8000), (1.0, 0x3C00), (-1.0, 0xBC00), (0.5, 0x3800), (2.0, 0x4000),
    (float("inf"), 0x7C00), (float("-inf"), 0xFC00), (65504.0, 0x7BFF), (65536.0, 0x7C00),
    (1e-20, 0x0000),
])
def test_rne_known_answers(val, bits):  # fp16_test.go:12-160
    assert L.orc_f32_to_f16_rne(val) == bits


def test_rne_nan_and_subnormals():  # fp16_test.go:86-100, :140-152
    h = L.orc_f32_to_f16_rne(float("nan"))
    assert (h >> 10) & 0x1F == 31 and h & 0x3FF != 0
    assert L.orc_f32_to_f16_rne(2.0 ** -24) != 0
    assert L.orc_f16_to_f32(L.orc_f32_to_f16_rne(2.0 ** -14)) == 2.0 ** -14


def test_rne_speech_feature_roundtrip():  # fp16_test.go:183-215
    for v in [104.7446, -16.8217, -14.2499, 17.5508, 0.0144, 58.4164, -18.8078, -8.4248,
              0.1, 0.2, -0.05, 1.5, -0.8, 0.001, 3.14, -2.71]:
        back = L.orc_f16_to_f32(L.orc_f32_to_f16_rne(v))
        assert abs(v - back) / abs(v) < 0.002


def test_batch_conversion_known_answers():  # fp16_test.go:220-246
    src = [1.0, -1.0, 0.5, 2.0, 0.0]
    assert [L.orc_f32_to_f16_rne(v) for v in src] == [0x3C00, 0xBC00, 0x3800, 0x4000, 0x0000]
    assert [L.orc_f16_to_f32(b) for b in (0x3C00, 0xBC00, 0x3800, 0x4000, 0x0000)] == src


def test_rne_matches_numpy_ieee():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.standard_normal(20000) * s for s in (1e-6, 1e-3, 1.0, 100.0, 3e4)])
    x = x.astype(np.float32)
    ours = np.array([L.orc_f32_to_f16_rne(float(v)) for v in x], np.uint16)
    ref = x.astype(np.float16).view(np.uint16)
    assert np.array_equal(ours, ref)


def test_f16_to_f32_exhaustive():
    bits = np.arange(0, 1 << 16, dtype=np.uint32)
    ours = np.array([L.orc_f16_to_f32(int(b)) for b in bits], np.float32)
    ref = bits.astype(np.uint16).view(np.float16).astype(np.float32)
    nan = np.isnan(ref)
    assert np.array_equal(np.isnan(ours), nan)
    assert np.array_equal(ours[~nan], ref[~nan])


def test_truncation_rule():  # internal/gpu/tensor.go:158-173
    assert L.orc_f32_to_f16_trunc(1.0) == 0x3C00
    assert L.orc_f32_to_f16_trunc(1.0 + 2 ** -10 * 0.99) == 0x3C00   # truncates, not rounds
    assert L.orc_f32_to_f16_trunc(70000.0) == 0x7C00
    assert L.orc_f32_to_f16_trunc(2.0 ** -15) == 0x0000               # subnormals flushed
    assert L.orc_f32_to_f16_trunc(-3.0) == 0xC200
