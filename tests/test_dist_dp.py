"""World-size-2 data-parallel step on CPU (gloo): two ranks, each with its own
egs shard, compute oracle gradients of the chain objective through a micro
CNN-TDNN, all-reduce the flat gradient with kfp16.dp, and apply the same SGD.
Both ranks must end bit-identical and equal to one process applying the
rank-averaged gradient."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from test_oracle_net import MICRO, _setup

FRAMES, STRIDE, LEFT = 31, 3, 2


def _den():
    rng = np.random.default_rng(5)
    S, A, P = 6, 20, 5
    src = np.concatenate([np.arange(S), rng.integers(0, S, A - S)]).astype(np.int32)
    dst = np.concatenate([(np.arange(S) + 1) % S, rng.integers(0, S, A - S)]).astype(np.int32)
    o = np.argsort(src, kind="stable")
    g = dict(S=S, P=P, A=A, src=src[o], dst=dst[o], pdf0=rng.integers(0, P, A).astype(np.int32),
             tp=np.exp(-rng.uniform(0.5, 3, A)).astype(np.float32), start=0)
    return g, oracle.den_initial_probs(g)


def _num(eg, T, P):
    rng = np.random.default_rng(100 + eg)
    S = 4
    row_ptr, dst = [0], []
    for s in range(S):
        dst += [s] + ([s + 1] if s + 1 < S else [])
        row_ptr.append(len(dst))
    return dict(S=S, A=len(dst), row_ptr=np.array(row_ptr, np.int32), dst=np.array(dst, np.int32),
                pdf1=rng.integers(1, P + 1, len(dst)).astype(np.int32),
                logw=np.full(len(dst), -0.5, np.float32), final_state=np.array([S - 1], np.int32),
                final_w=np.zeros(1, np.float32), start=0)


def rank_grad(rank, params, bns):
    """One rank's step on its shard: forward, chain objective on the subsampled
    rows, backward; returns the flat gradient in a fixed parameter order."""
    g, init = _den()
    x = np.random.default_rng(1000 + rank).standard_normal((FRAMES, 8)).astype(np.float32)
    net = oracle.OracleNet(MICRO, params, bns, round_mode=oracle.ROUND_NONE)
    net.forward(x)
    out = net.act("output")
    rows = LEFT + np.arange((FRAMES - LEFT) // STRIDE) * STRIDE
    deriv, _ = oracle.chain_objf(g, init, _num(rank, len(rows), out.shape[1]), out[rows])
    og = np.zeros_like(out)
    og[rows] = -deriv
    net.backward(og)
    grads = net.grads()
    net.close()
    return np.concatenate([grads[k].ravel() for k in sorted(params)]).astype(np.float32)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                    "kaldi-fp16_amd", "python"))
    from kfp16 import dp
    dist.init_process_group("gloo", rank=rank, world_size=world)
    params, bns, _, _ = _setup()
    grad = torch.from_numpy(rank_grad(rank, params, bns))
    dp.allreduce_mean_(grad, world)
    w = np.concatenate([params[k].ravel() for k in sorted(params)]).astype(np.float32)
    v = np.zeros_like(w)
    g = grad.numpy().copy()
    oracle.lib().orc_sgd(w.ctypes.data, g.ctypes.data, v.ctypes.data, 1e-3, 0.9, w.size)
    t = dp.max_over_ranks(float(rank + 1), "cpu")
    stats = dp.sum_over_ranks([1.0, float(rank)], "cpu")
    q.put((rank, w, t, stats))
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
def test_two_rank_step_equals_averaged_gradient():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict()
    for _ in range(world):
        r, w, t, stats = q.get(timeout=240)
        res[r] = (w, t, stats)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    np.testing.assert_array_equal(res[0][0], res[1][0])      # replicas stay identical
    assert res[0][1] == res[1][1] == 2.0                       # max over ranks
    assert res[0][2] == res[1][2] == [2.0, 1.0]                # summed statistics
    params, bns, _, _ = _setup()                               # one process, averaged gradient
    g = (rank_grad(0, params, bns) + rank_grad(1, params, bns)) / 2
    w = np.concatenate([params[k].ravel() for k in sorted(params)]).astype(np.float32)
    v = np.zeros_like(w)
    oracle.lib().orc_sgd(w.ctypes.data, g.ctypes.data, v.ctypes.data, 1e-3, 0.9, w.size)
    np.testing.assert_allclose(res[0][0], w, rtol=0, atol=1e-7)
