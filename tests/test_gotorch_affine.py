"""BASELINE configs[0]: the CPU plumbing case, gotorch.AffineLayer(40, 512).Forward on a
[1500 x 40] float64 input (go/gotorch/layers.go:57-70 over MatMul / matmulParallel,
ops.go:15-81), as restated in oracle/gotorch_cpu.c and timed by bench.py's
configs[0]_affine_40x512 leg.

The reference computes every output element as `sum := 0.0; for k { sum += a*b }`, then
adds the bias; the row split over goroutines changes which thread computes an element,
not its value. So: against a float64 numpy product accumulated in the same k order the
portable build (no FMA contraction) is bit-exact, at every worker count; the -march=native
build bench.py times may contract to FMA and is held to 1e-13 relative; the inputCache
clone equals the input.
"""
import numpy as np
import pytest

import oracle


def _ordered_affine(x, W, b):
    """numpy float64, per element: sum over k in ascending order from 0.0, then + b[j]"""
    acc = np.zeros((x.shape[0], W.shape[1]), np.float64)
    for k in range(x.shape[1]):
        acc += x[:, k:k + 1] * W[k:k + 1, :]
    return acc + b[None, :]


def _case(M, K, N, seed):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((M, K))
    W = rng.standard_normal((K, N)) * np.sqrt(2.0 / (K + N))   # NewAffineLayer's Xavier scale
    b = rng.standard_normal(N) * 0.1
    return x, W, b


@pytest.mark.parametrize("workers", [1, 2, 3, 7, 8, 16, 64])
def test_affine_40x512_bit_exact(workers):
    x, W, b = _case(1500, 40, 512, 0)
    y = oracle.gotorch_affine_forward(x, W, b, workers)
    want = _ordered_affine(x, W, b)
    assert y.dtype == np.float64 and y.shape == (1500, 512)
    assert np.array_equal(y, want)
    # and the product itself, independent of summation order
    np.testing.assert_allclose(y, x @ W + b, rtol=0, atol=1e-12)


@pytest.mark.parametrize("M,K,N", [(5, 4, 8), (1, 40, 512), (3, 1, 7), (2000, 40, 3), (1501, 40, 512)])
def test_affine_shapes(M, K, N):
    """matmulNaive (M*N*K <= 10000) and matmulParallel with more workers than rows, ragged
    last worker ranges, K = 1"""
    x, W, b = _case(M, K, N, M + K + N)
    for workers in (1, 4, 9):
        assert np.array_equal(oracle.gotorch_affine_forward(x, W, b, workers), _ordered_affine(x, W, b))


def test_affine_input_cache_and_native_build():
    x, W, b = _case(1500, 40, 512, 1)
    L = oracle.lib()
    import ctypes as C
    M, K, N = 1500, 40, 512
    y = np.empty((M, N))
    cache = np.full_like(x, np.nan)
    P = C.c_void_p
    L.gt_affine_forward(P(x.ctypes.data), M, K, P(W.ctypes.data), P(b.ctypes.data), N, P(y.ctypes.data),
                        P(cache.ctypes.data), C.c_int(8))
    assert np.array_equal(cache, x)          # l.inputCache = input.Clone()
    assert np.array_equal(y, _ordered_affine(x, W, b))
    # the build bench.py's CPU leg times (ORACLE_NATIVE=1: -march=native, FMA allowed)
    try:
        path = oracle.build(native=True)
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"native oracle build unavailable: {e}")
    Ln = C.CDLL(path)
    yn = np.empty((M, N))
    Ln.gt_affine_forward(P(x.ctypes.data), M, K, P(W.ctypes.data), P(b.ctypes.data), N, P(yn.ctypes.data),
                         P(cache.ctypes.data), C.c_int(8))
    np.testing.assert_allclose(yn, y, rtol=1e-13, atol=1e-14)
