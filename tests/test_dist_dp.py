"""World-size-2 data-parallel step on CPU (gloo): two ranks, each with its own
egs shard, compute oracle gradients of the chain objective through a micro
CNN-TDNN, exchange the flat gradient bucket by bucket in the order the product's
plan issues them (nnet_dp_plan on a layout-only network: the buckets nnet_backward
all-reduces over RCCL), and apply the same SGD. Both ranks must end bit-identical
and equal to one process applying the rank-averaged gradient.
Also: the bucket plan itself, and bench.py's own launcher (--gpus 2 --selftest)."""
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
    import kfp16
    params, bns, _, _ = _setup()
    g_sorted = rank_grad(rank, params, bns)
    # into the product's flat layout, exchanged by its bucket plan (small buckets)
    net = kfp16.Network(MICRO, max_frames=FRAMES, layout_only=True)
    flat = np.zeros(net.num_params, np.float32)
    o = 0
    for k in sorted(params):
        r, c, off = net.params[k]
        flat[off:off + r * c] = g_sorted[o:o + r * c]
        o += r * c
    plan = net.dp_plan(1024)
    assert len(plan) > 1 and dp.covers_exactly(plan, net.num_params)
    grad = torch.from_numpy(flat)
    dp.exchange_by_plan(grad, plan, world)
    g = np.concatenate([grad.numpy()[net.params[k][2]:net.params[k][2] + params[k].size] for k in sorted(params)])
    net.close()
    w = np.concatenate([params[k].ravel() for k in sorted(params)]).astype(np.float32)
    v = np.zeros_like(w)
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


def test_bucket_plan_of_the_benchmark_model():
    """nnet_dp_plan on the 17-TDNN-F model: buckets partition the flat buffer, are
    issued top layer first (descending offsets), are >= the bucket size except the
    last, and the last one covers the layers the backward reaches last (the convs)."""
    import kfp16
    from kfp16 import synth
    for xc in ("cnn_tdnn_17f.xconfig", "cnn_tdnn_17f_kaldi.xconfig", "cnn_tdnn_17f_ivec.xconfig"):
        net = kfp16.Network(synth.load_xconfig(xc), max_frames=1, layout_only=True)
        bucket = 16 << 20
        plan = net.dp_plan(bucket)
        from kfp16 import dp
        assert dp.covers_exactly(plan, net.num_params), xc
        steps = [a for a, _, _ in plan]
        assert steps == sorted(steps) and len(plan) >= 4, (xc, plan)
        assert all(e - b >= bucket // 4 for _, b, e in plan[:-1])
        assert all(plan[i][1] == plan[i + 1][2] for i in range(len(plan) - 1))
        assert plan[0][2] == net.num_params and plan[-1][1] == 0
        with pytest.raises(kfp16.KfError):
            net.forward(None, 1)          # layout-only: no device work
        net.close()


def test_plan_rules():
    """kf_dp_plan: cuts, the out-of-order fallback, bad arguments."""
    from kfp16 import dp
    # groups visited top-down: [80,100) [60,80) [0,60)
    assert dp.plan([80, 60, 0], [100, 80, 60], 100, 30) == [(1, 60, 100), (3, 0, 60)]
    assert dp.plan([80, 60, 0], [100, 80, 60], 100, 10) == [(0, 80, 100), (1, 60, 80), (3, 0, 60)]
    assert dp.plan([80, 60, 0], [100, 80, 60], 100, 1000) == [(3, 0, 100)]
    # a group writing above an exchanged range: one bucket after the backward
    assert dp.plan([80, 0, 85], [100, 60, 90], 100, 10) == [(3, 0, 100)]
    # empty groups are skipped; nothing to exchange still makes one (empty) bucket
    assert dp.plan([5, 5, 0], [10, 5, 5], 10, 2) == [(0, 5, 10), (3, 0, 5)]
    assert dp.plan([], [], 0, 1) == [(0, 0, 0)]
    with pytest.raises(RuntimeError):
        dp.plan([0], [11], 10, 1)


@pytest.mark.timeout(300)
def test_bench_launcher_two_ranks_cpu():
    """bench.py --gpus 2 without WORLD_SIZE starts two ranks itself (the driver's
    N-GPU command shape), each checks WORLD_SIZE == --gpus, and the bucketed exchange
    of the benchmark model's gradient averages over ranks."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--selftest"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    r = json.loads(lines[0])
    assert r["selftest"] and r["n_gpus"] == 2 and r["buckets"] >= 4 and r["max_abs_err"] == 0.0
    # a mismatched world is refused
    env2 = dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p2 = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--selftest"],
                        capture_output=True, text=True, timeout=120, env=env2)
    assert p2.returncode == 2 and "WORLD_SIZE" in p2.stderr
