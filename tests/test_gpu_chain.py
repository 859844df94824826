"""HIP chain objective vs the CPU oracle (oracle/kf_oracle_chain.c), through the C-ABI.

Tolerances: objective |Δ objf/frame| <= 1e-3 (chainverify/main.go:169);
numerator log-prob |Δ| <= 1e-2 vs the deterministic FP32 oracle. Posteriors and
output-gradient elements: |Δ| <= 1e-4 + one fp16 ulp of the value (float32
summation order differs between the GPU tree and the oracle's sequential sums).
"""
import ctypes as C

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def den():
    from kfp16 import synth
    g = synth.make_den_graph()
    return g, oracle.den_initial_probs(g)


def _x(T, P, seed, scale=2.0):
    return (np.random.default_rng(seed).standard_normal((T, P)) * scale).astype(np.float16)


def test_den_abi_matches_oracle(gpu, den):
    from kfp16 import chain
    g, init = den
    T = 490
    x = _x(T, g["P"], 11).astype(np.float32)
    x[5, :7] = [45.0, -45.0, 30.5, -30.5, 29.0, 0.0, -29.0]  # clamp edges
    fst = chain.DenFstGPU()
    rc = gpu.core.den_fst_upload(C.byref(fst), g["src"].ctypes.data, g["dst"].ctypes.data,
                                 g["pdf0"].ctypes.data, g["tp"].ctypes.data, g["A"], g["S"], g["P"])
    assert rc == 0, gpu.core.den_last_error()
    post = np.empty_like(x)
    lp = gpu.core.den_forward_backward(C.byref(fst), x.ctypes.data, init.ctypes.data, T, 1e-5,
                                       post.ctypes.data)
    lpf = gpu.core.den_forward(C.byref(fst), x.ctypes.data, init.ctypes.data, T, 1e-5)
    gpu.core.den_fst_free(C.byref(fst))
    rlp, rpost = oracle.den_forward_backward(g, init, x)
    assert lp == lpf
    assert abs(lp - rlp) / T <= 1e-5, (lp, rlp)
    np.testing.assert_allclose(post, rpost, atol=1e-5)
    np.testing.assert_allclose(post.sum(1), 1.0, atol=1e-4)


def test_den_abi_rejects_unknown_fst(gpu):
    from kfp16 import chain
    fst = chain.DenFstGPU()
    x = np.zeros((2, 4), np.float32)
    assert gpu.core.den_forward(C.byref(fst), x.ctypes.data, x.ctypes.data, 2, 1e-5) == np.float32(-1e30)
    assert gpu.core.den_last_error()


def _device_fst(gpu, f, keep):
    from kfp16 import chain
    def up(a, dt):
        a = np.ascontiguousarray(a, dt)
        b = gpu.DeviceBuffer(a.nbytes)
        gpu.check(gpu.core.bridge_transfer_int32(b.ptr, a.view(np.int32).ctypes.data, a.size))
        keep.append(b)
        return b.ptr
    return chain.ChainFstGPU(up(f["row_ptr"], np.int32), up(f["dst"], np.int32),
                             up(f["pdf1"], np.int32), up(f["logw"], np.float32),
                             up(f["final_state"], np.int32), up(f["final_w"], np.float32),
                             f["S"], f["A"], len(f["final_state"]), f.get("start", 0))


def test_num_abi_matches_oracle(gpu):
    from kfp16 import synth
    f = synth.make_num_fst(3)
    T, P = 490, 3080
    x32 = (np.random.default_rng(5).standard_normal((T, P)) * 2).astype(np.float32)
    keep = []
    fst = _device_fst(gpu, f, keep)
    dx = gpu.upload_f32(x32)
    post = gpu.DeviceBuffer(T * P * 4)
    lp = gpu.core.chain_num_forward_backward(fst.row_ptr, fst.col_idx, fst.weights, fst.labels,
                                             fst.final_states, fst.final_weights, f["S"], f["A"], 1,
                                             dx.ptr, post.ptr, T, P, None)
    got = gpu.read_f32(post.ptr, (T, P))
    rlp, rpost = oracle.num_forward_backward(f, x32.astype(np.float16).astype(np.float32))
    assert abs(lp - rlp) <= 1e-2, (lp, rlp)
    np.testing.assert_allclose(got, rpost, atol=1e-4)


def test_chain_compute_loss_abi(gpu):
    """C1 path: log-domain FB on both FSTs, grad16 = clamp(den - num, +-30)."""
    from kfp16 import chain, synth
    T, P = 60, 3080
    f = synth.make_num_fst(1, num_states=30)
    d = synth.make_num_fst(2, num_states=45)      # a second FST standing in for "den as FST"
    d["final_state"] = np.arange(d["S"], dtype=np.int32)
    d["final_w"] = np.zeros(d["S"], np.float32)
    keep = []
    nf, df = _device_fst(gpu, f, keep), _device_fst(gpu, d, keep)
    x = _x(T, P, 8)
    dx = gpu.upload_fp16(x)
    g = gpu.DeviceBuffer(T * P * 2)
    res = chain.ChainLossResult()
    rc = gpu.core.chain_compute_loss(dx.ptr, C.byref(nf), C.byref(df), T, P, g.ptr, C.byref(res))
    assert rc == 0, gpu.core.chain_last_error()
    xf = x.astype(np.float32)
    nl, npost = oracle.num_forward_backward(f, xf)
    dl, dpost = oracle.num_forward_backward(d, xf)
    assert abs(res.num_logprob - nl) <= 1e-2 and abs(res.den_logprob - dl) <= 1e-2
    assert abs(res.loss + (nl - dl)) <= 2e-2
    got = gpu.read_fp16(g.ptr, (T, P)).astype(np.float32)
    ref = np.clip(dpost - npost, -30, 30)
    assert np.all(np.abs(got - ref) <= 1e-4 + np.abs(ref) * 2 ** -10)


def test_objective_pieces_abi(gpu):
    rng = np.random.default_rng(4)
    T, P = 7, 33
    x = (rng.standard_normal((T, P)) * 20).astype(np.float32)
    g0 = rng.standard_normal((T, P)).astype(np.float32)
    num, den = rng.random((T, P)).astype(np.float32), rng.random((T, P)).astype(np.float32)
    dx, dg, dn, dd = (gpu.upload_f32(a) for a in (x, g0, num, den))
    n = gpu.core.chain_penalize_out_of_range(dx.ptr, dg.ptr, 30.0, 0.02, T, P)
    ref = g0.copy()
    even = (np.arange(T) % 2 == 0)[:, None]
    lo, hi = even & (x < -30), even & (x > 30)
    ref[lo] += (-30 - x[lo]) * 0.02
    ref[hi] += (30 - x[hi]) * 0.02
    assert n == int(lo.sum() + hi.sum())
    np.testing.assert_allclose(gpu.read_f32(dg.ptr, (T, P)), ref, rtol=1e-6, atol=1e-6)
    term = gpu.core.chain_l2_regularize(dx.ptr, dg.ptr, 0.5, T * P)
    ref = ref - 0.5 * x
    assert abs(term + 0.25 * float(np.sum(x.astype(np.float64) ** 2))) <= 1e-3 * abs(term)
    assert gpu.core.chain_add_posterior_gradient(dn.ptr, dd.ptr, dg.ptr, 2.0, T * P) == 0
    ref = ref + 2.0 * (num - den)
    np.testing.assert_allclose(gpu.read_f32(dg.ptr, (T, P)), ref, rtol=1e-5, atol=1e-5)
    h = gpu.DeviceBuffer(T * P * 2)
    assert gpu.core.chain_combine_gradient(dn.ptr, dd.ptr, 1.5, T, P, h.ptr) == 0
    np.testing.assert_array_equal(gpu.read_fp16(h.ptr, (T, P)), (1.5 * (num - den)).astype(np.float16))
    assert gpu.core.chain_grad_fp32_to_fp16(dg.ptr, h.ptr, T * P) == 0
    gpu.sync()
    np.testing.assert_array_equal(gpu.read_fp16(h.ptr, (T, P)),
                                  gpu.read_f32(dg.ptr, (T, P)).astype(np.float16))


def _batch_setup(gpu, den, negs, frames_per_eg=1500, seed=21):
    from kfp16 import chain, synth
    g, init = den
    P = g["P"]
    row0, frames, stride = synth.chain_layout(negs, frames_per_eg)
    fsts = [synth.make_num_fst(i) for i in range(negs)]
    x = _x(negs * frames_per_eg, P, seed)
    return g, init, P, row0, frames, stride, fsts, x


def test_batched_objective_matches_oracle(gpu, den):
    from kfp16 import chain
    negs = 3
    g, init, P, row0, frames, stride, fsts, x = _batch_setup(gpu, den, negs)
    frames = frames.copy()
    frames[1] = 301              # ragged: a shorter sequence
    x[row0[2] + 6 * stride, 100] = 40.0   # even frame: penalised
    x[row0[2] + 7 * stride, 101] = -40.0  # odd frame: not penalised
    dx = gpu.upload_fp16(x)
    og = gpu.upload_fp16(np.full(x.shape, 7.0, np.float16))  # sentinel
    dg = chain.DenGraph(g)
    np.testing.assert_allclose(dg.initial_probs(), init, rtol=0, atol=0)
    ch = chain.Chain(dg, max_seqs=8, max_frames=490)
    nb = chain.NumBatch(fsts)
    ch.compute(nb, dx.ptr, P, x.shape[0], row0, frames, stride, og.ptr, P)
    res = ch.result()
    got = gpu.read_fp16(og.ptr, x.shape).astype(np.float32)
    stats = ch.seq_stats(negs)
    xf = x.astype(np.float32)
    sup = np.zeros(x.shape[0], bool)
    tot_objf = 0.0
    for i in range(negs):
        rows = row0[i] + np.arange(frames[i]) * stride
        sup[rows] = True
        deriv, r = oracle.chain_objf(g, init, fsts[i], xf[rows])
        assert abs(stats[i, 0] - r["num_logprob"]) <= 1e-2
        assert abs(stats[i, 1] - r["den_logprob"]) / frames[i] <= 1e-4
        assert abs(stats[i, 2] - r["objf"]) / frames[i] <= 1e-3
        assert int(stats[i, 6]) == r["out_of_range"] and stats[i, 7] == 1.0
        tot_objf += r["objf"]
        ref = -deriv
        err = np.abs(got[rows] - ref) - (1e-4 + np.abs(ref) * 2 ** -10)
        assert np.all(err <= 0), (i, float(err.max()))
    assert int(stats[2, 6]) == 1
    assert np.all(got[~sup] == 7.0)          # rows without supervision are not touched
    assert res.num_seqs == negs and res.num_ok == negs and res.frames == int(frames.sum())
    assert abs(res.objf - tot_objf) / res.frames <= 1e-3


def test_batched_objective_nan_rule(gpu, den):
    from kfp16 import chain
    negs = 2
    g, init, P, row0, frames, stride, fsts, x = _batch_setup(gpu, den, negs, seed=5)
    # +inf on the numerator path of eg 1 at frame 0 (its first arc's pdf)
    x[row0[1], fsts[1]["pdf1"][0] - 1] = np.inf
    dx = gpu.upload_fp16(x)
    og = gpu.upload_fp16(np.full(x.shape, 7.0, np.float16))
    ch = chain.Chain(chain.DenGraph(g, init), max_seqs=2, max_frames=490)
    nb = chain.NumBatch(fsts)
    ch.compute(nb, dx.ptr, P, x.shape[0], row0, frames, stride, og.ptr, P)
    res = ch.result()
    got = gpu.read_fp16(og.ptr, x.shape).astype(np.float32)
    rows1 = row0[1] + np.arange(frames[1]) * stride
    assert not np.any(got[rows1])
    assert res.num_ok == 1
    stats = ch.seq_stats(negs)
    assert stats[1, 7] == 0.0 and stats[1, 2] == -10.0 * frames[1]
    rows0 = row0[0] + np.arange(frames[0]) * stride
    assert np.any(got[rows0] != 0)


def test_batched_objective_repeatable(gpu, den):
    """Fixed arc order + fixed-point den accumulation: bit-identical reruns."""
    from kfp16 import chain
    negs = 2
    g, init, P, row0, frames, stride, fsts, x = _batch_setup(gpu, den, negs, seed=9)
    dx = gpu.upload_fp16(x)
    og = gpu.DeviceBuffer(x.size * 2)
    ch = chain.Chain(chain.DenGraph(g, init), max_seqs=2, max_frames=490)
    nb = chain.NumBatch(fsts)
    outs = []
    for _ in range(2):
        ch.compute(nb, dx.ptr, P, x.shape[0], row0, frames, stride, og.ptr, P)
        ch.result()
        outs.append(gpu.read_fp16(og.ptr, x.shape))
    np.testing.assert_array_equal(outs[0], outs[1])


def test_den_sequence_pairs_match_single(gpu, den):
    """Sequence pairs (two sequences per workgroup set, interleaved LDS state) give the
    single-sequence recursion's results bit for bit: ragged frame counts (a pair whose
    members end at different frames, forward and backward) and an odd count (a unit
    with an absent partner)."""
    from kfp16 import chain
    negs = 5
    g, init, P, row0, frames, stride, fsts, x = _batch_setup(gpu, den, negs, seed=41)
    frames = frames.copy()
    frames[1] = 301
    frames[2] = 420
    dx = gpu.upload_fp16(x)
    og = gpu.DeviceBuffer(x.size * 2)
    ch = chain.Chain(chain.DenGraph(g, init), max_seqs=negs, max_frames=490)
    nb = chain.NumBatch(fsts)
    outs = []
    for pairs in (False, True):
        ch.debug_den_pairs(pairs)
        gpu.core.bridge_gpu_memset(og.ptr, 0, x.size * 2)
        ch.compute(nb, dx.ptr, P, x.shape[0], row0, frames, stride, og.ptr, P)
        res = ch.result()
        outs.append((res.objf, res.num_ok, ch.seq_stats(negs).copy(), gpu.read_fp16(og.ptr, x.shape)))
    ch.debug_den_pairs(True)
    assert outs[0][1] == outs[1][1] == negs
    np.testing.assert_array_equal(outs[1][2], outs[0][2])
    np.testing.assert_array_equal(outs[1][3], outs[0][3])
    assert outs[1][0] == outs[0][0]


def test_den_pairs_beyond_co_resident_grid(gpu, den):
    """More sequences than the CUs hold at G >= 2 (300 egs of 20 frames): one workgroup
    per unit (G = 1, no cross-workgroup exchange), sequence pairs and single sequences
    bit-identical, every objective finite."""
    from kfp16 import chain, synth
    g, init = den
    P, negs = g["P"], 300
    row0, frames, stride = synth.chain_layout(negs, 90)
    fsts = [synth.make_num_fst(i, num_states=10) for i in range(negs)]
    x = _x(negs * 90, P, 51)
    dx = gpu.upload_fp16(x)
    og = gpu.DeviceBuffer(x.size * 2)
    ch = chain.Chain(chain.DenGraph(g, init), max_seqs=negs, max_frames=int(frames.max()))
    nb = chain.NumBatch(fsts)
    outs = []
    for pairs in (False, True):
        ch.debug_den_pairs(pairs)
        gpu.core.bridge_gpu_memset(og.ptr, 0, x.size * 2)
        ch.compute(nb, dx.ptr, P, x.shape[0], row0, frames, stride, og.ptr, P)
        res = ch.result()
        outs.append((res.objf, res.num_ok, ch.seq_stats(negs).copy(), gpu.read_fp16(og.ptr, x.shape)))
    ch.debug_den_pairs(True)
    assert outs[0][1] == outs[1][1] == negs
    assert np.isfinite(outs[1][0])
    np.testing.assert_array_equal(outs[1][2], outs[0][2])
    np.testing.assert_array_equal(outs[1][3], outs[0][3])


def test_numerator_beyond_lds_path_matches_oracle(gpu, den):
    """A numerator FST with more than 1024 states (beyond k_num_fb's LDS layout) sends the
    batch to the global-memory numerator (k_logfb): objective and gradient of both
    sequences against the oracle, and the small sequence's gradient rows bit-identical to
    the LDS path's (the two numerator kernels share the arithmetic and its order)."""
    from kfp16 import chain, synth
    g, init = den
    P = g["P"]
    row0, frames, stride = synth.chain_layout(2, 3400)   # 1123 frames: the 1100-state path fits
    fsts = [synth.make_num_fst(0), synth.make_num_fst(1, num_states=1100)]
    x = _x(2 * 3400, P, 61)
    dx = gpu.upload_fp16(x)
    og = gpu.DeviceBuffer(x.size * 2)
    ch = chain.Chain(chain.DenGraph(g, init), max_seqs=2, max_frames=int(frames.max()))
    ch.debug_den_pairs(False)   # the one-sequence run below then has the same den units
    gpu.core.bridge_gpu_memset(og.ptr, 0, x.size * 2)
    ch.compute(chain.NumBatch(fsts), dx.ptr, P, x.shape[0], row0, frames, stride, og.ptr, P)
    res = ch.result()
    got = gpu.read_fp16(og.ptr, x.shape)
    stats = ch.seq_stats(2)
    assert res.num_ok == 2
    xf = x.astype(np.float32)
    for i in range(2):
        rows = row0[i] + np.arange(frames[i]) * stride
        deriv, r = oracle.chain_objf(g, init, fsts[i], xf[rows])
        assert abs(stats[i, 0] - r["num_logprob"]) <= 1e-2
        assert abs(stats[i, 2] - r["objf"]) / frames[i] <= 1e-3
        ref = -deriv
        err = np.abs(got[rows].astype(np.float32) - ref) - (1e-4 + np.abs(ref) * 2 ** -10)
        assert np.all(err <= 0), (i, float(err.max()))
    # sequence 0 alone fits the LDS numerator
    gpu.core.bridge_gpu_memset(og.ptr, 0, x.size * 2)
    ch.compute(chain.NumBatch(fsts[:1]), dx.ptr, P, x.shape[0], row0[:1], frames[:1], stride, og.ptr, P)
    ch.result()
    ch.debug_den_pairs(True)
    rows0 = row0[0] + np.arange(frames[0]) * stride
    np.testing.assert_array_equal(gpu.read_fp16(og.ptr, x.shape)[rows0], got[rows0])


@pytest.mark.parametrize("negs", [16, pytest.param(64, marks=pytest.mark.slow)])
def test_den_exchange_xcd_local_matches_agent_scope(gpu, den, negs):
    """The den exchange between the blocks of a sequence that share an XCD (L2-local
    stores / L1-missing loads) hands over exactly the words the agent-scope exchange
    (through to memory) does: objective, per-sequence stats and gradient bit-identical
    at 16 and at the bench's 64 egs, where den_map's XCD placement holds."""
    from kfp16 import chain
    g, init, P, row0, frames, stride, fsts, x = _batch_setup(gpu, den, negs, seed=31)
    dx = gpu.upload_fp16(x)
    og = gpu.DeviceBuffer(x.size * 2)
    ch = chain.Chain(chain.DenGraph(g, init), max_seqs=negs, max_frames=490)
    nb = chain.NumBatch(fsts)
    outs = []
    for force in (True, False, True):
        ch.debug_exchange_sys(force)
        ch.compute(nb, dx.ptr, P, x.shape[0], row0, frames, stride, og.ptr, P)
        res = ch.result()
        outs.append((res.objf, res.num_ok, ch.seq_stats(negs).copy(), gpu.read_fp16(og.ptr, x.shape)))
        c = ch.debug_census()
        assert c["forced"] == force and c["units"] == (negs + 1) // 2
        if not force:
            # the default run really took the L2-local exchange: every unit's workgroups
            # shared one XCD in both recursions (else this compares agent scope with itself)
            assert c["local_fwd"] == c["local_bwd"] == c["units"], c
    ch.debug_exchange_sys(False)
    for o in outs[1:]:
        assert o[0] == outs[0][0] and o[1] == outs[0][1] == negs
        np.testing.assert_array_equal(o[2], outs[0][2])
        np.testing.assert_array_equal(o[3], outs[0][3])


@pytest.mark.slow
def test_bench_size_objective_matches_oracle(gpu, den):
    """The bench's own objective configuration — 64 egs x 1500 frames, sequence pairs,
    G = 4 workgroups per unit, default (XCD-local) placement, the numerator co-resident on
    the side stream — against oracle.chain_objf (backward.go:224-371, chain_den.cu:496-706)
    on a sample of sequences: both members of pair 0, one mid-grid pair, the last unit and
    one ragged pair (members of unequal length). Bars of SURVEY §8d: |d objf/frame| <=
    1e-3, numerator |d| <= 1e-2, gradient rows <= 1e-4 + one fp16 ulp."""
    from kfp16 import chain
    negs = 64
    g, init, P, row0, frames, stride, fsts, x = _batch_setup(gpu, den, negs, seed=77)
    frames = frames.copy()
    frames[45] = 333                     # unit 22 = sequences 44, 45: a ragged pair
    dx = gpu.upload_fp16(x)
    og = gpu.upload_fp16(np.full(x.shape, 7.0, np.float16))
    ch = chain.Chain(chain.DenGraph(g, init), max_seqs=negs, max_frames=490)
    ch.compute(chain.NumBatch(fsts), dx.ptr, P, x.shape[0], row0, frames, stride, og.ptr, P)
    res = ch.result()
    c = ch.debug_census()
    assert res.num_ok == negs and c["units"] == negs // 2
    assert c["local_fwd"] == c["local_bwd"] == c["units"] and not c["forced"], c
    stats = ch.seq_stats(negs)
    xf = x.astype(np.float32)
    for i in (0, 1, 30, 31, 44, 45, 62, 63):
        rows = row0[i] + np.arange(frames[i]) * stride
        got = gpu.read_fp16(og.ptr + int(rows[0]) * P * 2, (int(rows[-1] - rows[0]) + 1, P))[::stride]
        deriv, r = oracle.chain_objf(g, init, fsts[i], xf[rows])
        assert abs(stats[i, 0] - r["num_logprob"]) <= 1e-2, (i, stats[i, 0], r["num_logprob"])
        assert abs(stats[i, 2] - r["objf"]) / frames[i] <= 1e-3, (i, stats[i, 2], r["objf"])
        ref = -deriv
        err = np.abs(got.astype(np.float32) - ref) - (1e-4 + np.abs(ref) * 2 ** -10)
        assert np.all(err <= 0), (i, float(err.max()))
    # the ragged member's rows past its end keep the sentinel
    tail = row0[45] + frames[45] * stride
    assert np.all(gpu.read_fp16(og.ptr + int(tail) * P * 2, (3, P)) == 7.0)


def test_den_exchange_timeout_is_sticky(gpu, den):
    """A den exchange that gives up (forced: zero polls allowed) makes the next
    kf_chain_result fail even when a later compute succeeds; the result call that
    reports it clears the count (chain_den.cu:496-706 must never yield a silently
    wrong gradient)."""
    from kfp16 import KfError, chain
    negs = 4
    g, init, P, row0, frames, stride, fsts, x = _batch_setup(gpu, den, negs, seed=21)
    dx = gpu.upload_fp16(x)
    og = gpu.DeviceBuffer(x.size * 2)
    ch = chain.Chain(chain.DenGraph(g, init), max_seqs=negs, max_frames=490)
    nb = chain.NumBatch(fsts)
    ch.compute(nb, dx.ptr, P, x.shape[0], row0, frames, stride, og.ptr, P)
    good = ch.result()
    ch.debug_spin_limit(0)           # every unsatisfied wait times out at once
    ch.compute(nb, dx.ptr, P, x.shape[0], row0, frames, stride, og.ptr, P)
    ch.debug_spin_limit(None)
    ch.compute(nb, dx.ptr, P, x.shape[0], row0, frames, stride, og.ptr, P)  # a good launch after it
    with pytest.raises(KfError, match="timed out"):
        ch.result()
    again = ch.result()               # reported once, then cleared
    assert again.num_ok == good.num_ok == negs
    assert again.objf == good.objf


def test_backward_test_fixture_through_abi(gpu):
    """internal/nnet/backward_test.go:28-140's FST and output (tests/golden/backward_test_fd.npz)
    through the GPU ABI the Go chain path calls (chain_num_forward_backward and its _det
    form; labels pdf0 + 1, chain.h). The ABI rounds the fp32 output to fp16 first
    (chain.cu / chain_det.cu:412-477), so the log-prob is compared with the restated
    computeChainLossCPU's on the fp16-rounded output (|d| <= 1e-5 per frame) and with the
    fixture's float32 value within the fp16 rounding of T outputs; posteriors are the
    fixture's one-hot num_post."""
    import os
    from kfp16 import ops_abi  # noqa: F401  (binds chain_num_forward_backward_det)
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "backward_test_fd.npz"))
    x = z["nnet"]
    T, P = x.shape
    S = T + 1
    f = dict(S=S, A=T, row_ptr=z["row_ptr"][:S + 1], dst=z["col_idx"], pdf1=z["pdf0"] + 1,
             logw=z["weights"], final_state=np.arange(S, dtype=np.int32),
             final_w=np.zeros(S, np.float32), start=0)
    keep = []
    fst = _device_fst(gpu, f, keep)
    dx = gpu.upload_f32(x)
    path = x[np.arange(T), z["pdf0"]]
    lp16 = float(path.astype(np.float16).astype(np.float64).sum())
    for fn in (gpu.core.chain_num_forward_backward, gpu.core.chain_num_forward_backward_det):
        post = gpu.DeviceBuffer(T * P * 4)
        lp = fn(fst.row_ptr, fst.col_idx, fst.weights, fst.labels, fst.final_states,
                fst.final_weights, S, T, S, dx.ptr, post.ptr, T, P, None)
        assert abs(lp - lp16) <= 1e-5 * T
        assert abs(lp - float(z["num_logprob"])) <= T * 2.0 ** -12
        gpu.sync()
        np.testing.assert_allclose(gpu.read_f32(post.ptr, (T, P)), z["num_post"], atol=1e-6)
