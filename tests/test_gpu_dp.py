"""Native data-parallel exchange (include/kf_dp.h, csrc/dp.cpp) on one MI355X.

A one-rank RCCL communicator runs the same code path as N ranks: nnet_backward
issues one ncclAllReduce(avg) per planned bucket on the high-priority comm stream,
gated by events on the compute stream, and joins before returning. With one rank
the average is the identity, so the gradient must be bit-identical to an unbound
backward, and the number of launches must equal the plan's buckets. The N > 1
arithmetic (bucket partition, averaging) is covered on CPU by tests/test_dist_dp.py.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _net(gpu, T):
    from kfp16 import synth
    net = gpu.Network(synth.load_xconfig("tiny.xconfig"), max_frames=T)
    synth.init_network(net)
    return net


def test_bucketed_allreduce_one_rank_is_identity(gpu):
    from kfp16 import dp, synth
    T = 150
    feats = gpu.upload_fp16(synth.make_features(T, 40))
    net = _net(gpu, T)
    net.forward(feats.ptr, T)
    out = net.read_activation("output")
    og = gpu.upload_fp16((np.random.default_rng(3).standard_normal(out.shape) * 0.05).astype(np.float16))
    net.backward(og.ptr)
    ref = gpu.read_f32(net.grad_ptr, (net.num_params,)).copy()

    comm = dp.Communicator(0, 1, dp.unique_id(), 0)
    bucket = 16 << 10                       # small buckets: many launches inside the backward
    plan = net.dp_plan(bucket)
    assert dp.covers_exactly(plan, net.num_params) and len(plan) > 2
    net.bind_dp(comm, bucket)
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
