"""Native data-parallel exchange (include/kf_dp.h, csrc/dp.cpp) on one MI355X.

A one-rank RCCL communicator runs the same code path as N ranks: nnet_backward
issues one ncclAllReduce(avg) per planned bucket on the high-priority comm stream,
gated by events on the compute stream, and joins before returning. At one rank the
average is the identity, so a bucket exchanged too early would still leave the right
gradient behind. The kf_dp_debug hooks make timing visible on one GPU:

- SNAPSHOT: each bucket is copied on the comm stream at the moment its exchange
  starts. Every snapshot must equal the finished gradient bit for bit (the gradient
  buffer is filled with NaN first, so a bucket sent before its producers finished
  shows it). Negative control: nnet_dp_debug_early issues every bucket before the
  backward, and the snapshots must then differ.
- PEER_MEAN: each exchanged bucket is averaged with a second shard's gradient, as a
  two-rank all-reduce would. Two egs shards run the HIP backward one after the other;
  the bound backward of shard A followed at once by nnet_sgd must give the gradient
  (gA + gB) / 2 and the weights of one SGD step on that mean gradient, bit for bit.
  That checks the gates, the bucket plan's coverage of the product's gradient layout
  and kf_dp_join (SGD is enqueued without a host sync). Negative control as above.

Reference: single device only (cpp/cuda/bridge.cu:38-47); SURVEY §8e. The N > 1
arithmetic over real ranks is covered on CPU by tests/test_dist_dp.py.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BUCKET = 16 << 10  # small buckets: many exchanges inside the backward


def _setup(gpu, xconfig, T, seed=3):
    from kfp16 import synth
    net = gpu.Network(synth.load_xconfig(xconfig), max_frames=T)
    synth.init_network(net)
    feats = gpu.upload_fp16(synth.make_features(T, 40, seed=seed))
    net.forward(feats.ptr, T)
    out = net.read_activation("output")
    og = gpu.upload_fp16((np.random.default_rng(seed).standard_normal(out.shape) * 0.05).astype(np.float16))
    return net, feats, og


def _fill(gpu, ptr, n, byte):
    gpu.core.bridge_gpu_memset(ptr, byte, n * 4)


def test_bucketed_allreduce_one_rank_is_identity(gpu):
    from kfp16 import dp
    net, feats, og = _setup(gpu, "tiny.xconfig", 150)
    net.backward(og.ptr)
    ref = gpu.read_f32(net.grad_ptr, (net.num_params,)).copy()

    comm = dp.Communicator(0, 1, dp.unique_id(), 0)
    plan = net.dp_plan(BUCKET)
    assert dp.covers_exactly(plan, net.num_params) and len(plan) > 2
    net.bind_dp(comm, BUCKET)
    n0, v0 = comm.stats()
    net.backward(og.ptr)
    gpu.sync()
    n1, v1 = comm.stats()
    got = gpu.read_f32(net.grad_ptr, (net.num_params,))
    assert n1 - n0 == len(plan) and v1 - v0 == net.num_params
    np.testing.assert_array_equal(got, ref)
    net.bind_dp(None, 0)
    comm.close()
    net.close()


@pytest.mark.parametrize("xconfig,T", [("tiny.xconfig", 150), ("cnn_tdnn_17f.xconfig", 1500)])
def test_exchange_starts_after_its_gradients(gpu, xconfig, T):
    """Every bucket's exchange sees its final gradient; the early-issue control does not."""
    from kfp16 import dp
    net, feats, og = _setup(gpu, xconfig, T)
    P = net.num_params
    snap = gpu.DeviceBuffer(P * 4)
    comm = dp.Communicator(0, 1, dp.unique_id(), 0)
    plan = net.dp_plan(BUCKET)
    assert dp.covers_exactly(plan, P) and len(plan) > 4
    net.bind_dp(comm, BUCKET)
    comm.debug(comm.DEBUG_SNAPSHOT, net.grad_ptr, snap.ptr, P)

    def run(early):
        net.dp_debug_early(early)
        _fill(gpu, net.grad_ptr, P, 0xFF)   # NaN everywhere: unwritten values show
        _fill(gpu, snap.ptr, P, 0x7F)
        net.backward(og.ptr)
        gpu.sync()
        g = gpu.read_f32(net.grad_ptr, (P,)).view(np.uint32)
        s = gpu.read_f32(snap.ptr, (P,)).view(np.uint32)
        bad = [j for j, (_, b, e) in enumerate(plan) if not np.array_equal(g[b:e], s[b:e])]
        return g, bad

    g, bad = run(False)
    assert not bad, f"buckets exchanged before their gradients were final: {bad[:10]} of {len(plan)}"
    # the gradient itself was produced (no NaN left outside the 64-element pads)
    for name, (r, c, off) in net.params.items():
        assert np.isfinite(g[off:off + r * c].view(np.float32)).all(), name
    _, bad_early = run(True)
    assert bad_early, "negative control: issuing every bucket before the backward went unnoticed"
    net.dp_debug_early(False)
    comm.debug(0)
    net.bind_dp(None, 0)
    comm.close()
    net.close()


@pytest.mark.parametrize("xconfig,T", [("tiny.xconfig", 300), ("cnn_tdnn_17f.xconfig", 1500)])
def test_two_shard_mean_then_sgd(gpu, xconfig, T):
    """HIP gradients of two egs shards averaged bucket by bucket through the product's
    plan, gates and join, then SGD: equals one SGD step on the mean gradient."""
    from kfp16 import dp, synth
    net, fa, oga = _setup(gpu, xconfig, T, seed=3)
    P = net.num_params
    fb = gpu.upload_fp16(synth.make_features(T, 40, seed=8))
    ogb = gpu.upload_fp16((np.random.default_rng(8).standard_normal((T, oga.shape[1])) * 0.05)
                          .astype(np.float16))
    w0 = net.get_params()

    def grad_of(feats, og):
        net.forward(feats.ptr, T)
        _fill(gpu, net.grad_ptr, P, 0)
        net.backward(og.ptr)
        return gpu.read_f32(net.grad_ptr, (P,)).copy()

    gb = grad_of(fb, ogb)
    ga = grad_of(fa, oga)
    assert not np.array_equal(ga, gb)
    mean = ((ga + gb) * np.float32(0.5)).astype(np.float32)
    lr, mom = 1e-3, 0.9

    # reference: one SGD step on the mean gradient (no exchange)
    net.set_params(w0)
    gpu.check(gpu.core.bridge_transfer_float32(net.grad_ptr, mean.ctypes.data, P), "upload mean")
    net.sgd(lr, mom)
    w_ref = gpu.read_f32(net.master_ptr, (P,)).copy()

    peer = gpu.upload_f32(gb)
    comm = dp.Communicator(0, 1, dp.unique_id(), 0)
    net.bind_dp(comm, BUCKET)
    comm.debug(comm.DEBUG_PEER_MEAN, net.grad_ptr, peer.ptr, P)

    def bound_step(early):
        net.set_params(w0)
        net.dp_debug_early(early)
        net.forward(fa.ptr, T)
        _fill(gpu, net.grad_ptr, P, 0)
        net.backward(oga.ptr)
        net.sgd(lr, mom)            # enqueued behind kf_dp_join, no host sync between
        gpu.sync()
        return gpu.read_f32(net.grad_ptr, (P,)), gpu.read_f32(net.master_ptr, (P,))

    g, w = bound_step(False)
    np.testing.assert_array_equal(g, mean)
    np.testing.assert_array_equal(w, w_ref)
    g_early, _ = bound_step(True)
    assert not np.array_equal(g_early, mean), "negative control: early exchange went unnoticed"
    net.dp_debug_early(False)
    comm.debug(0)
    net.bind_dp(None, 0)
    comm.close()
    net.close()


def test_allreduce_mean_and_sum(gpu):
    from kfp16 import dp
    comm = dp.Communicator(0, 1, dp.unique_id(), 0)
    x = np.random.default_rng(1).standard_normal(1000).astype(np.float32)
    bx = gpu.upload_f32(x)
    comm.allreduce_mean(bx.ptr, x.size)
    d = np.arange(6, dtype=np.float64)
    bd = gpu.upload_f32(d.view(np.float32))
    comm.allreduce_sum_f64(bd.ptr, d.size)
    gpu.sync()
    np.testing.assert_array_equal(gpu.read_f32(bx.ptr, x.shape), x)
    np.testing.assert_array_equal(gpu.read_f32(bd.ptr, (2 * d.size,)).view(np.float64), d)
    comm.close()


def test_debug_hook_arguments(gpu):
    from kfp16 import dp
    comm = dp.Communicator(0, 1, dp.unique_id(), 0)
    with pytest.raises(RuntimeError):
        comm.debug(3, 16, 16)          # exclusive modes
    with pytest.raises(RuntimeError):
        comm.debug(comm.DEBUG_SNAPSHOT)  # needs both buffers
    with pytest.raises(RuntimeError):
        comm.debug(comm.DEBUG_SNAPSHOT, 16, 16)  # and their length
    # a bucket outside the registered gradient fails instead of writing past aux
    g, aux = gpu.DeviceBuffer(64 * 4), gpu.DeviceBuffer(64 * 4)
    other = gpu.DeviceBuffer(64 * 4)
    comm.debug(comm.DEBUG_SNAPSHOT, g.ptr, aux.ptr, 64)
    comm.allreduce_mean(g.ptr + 32 * 4, 32)          # inside: fine
    with pytest.raises(RuntimeError):
        comm.allreduce_mean(g.ptr + 48 * 4, 32)      # runs past the end
    with pytest.raises(RuntimeError):
        comm.allreduce_mean(other.ptr, 16)           # another buffer
    gpu.sync()
    comm.debug(0)
    comm.close()
