#!/usr/bin/env python3
"""bench.py — frames/sec of the CNN-TDNN fwd+bwd training step on MI355X.

Metric (BASELINE.json): frames/sec CNN-TDNN fwd+bwd, 40-dim x 1500-frame egs,
1/2/4/8 MI355X. One step = TrainStep (train_step.go:142-283): forward, chain
LF-MMI objective + derivative (numerator and leaky-HMM denominator per eg,
backward.go:224-371), backward with the gradient all-reduce overlapped (N > 1,
kf_dp over RCCL), and SGD, over one minibatch of 64 synthetic egs (96,000 frames)
per GPU, on the pinned synthetic 17-TDNN-F model (configs/cnn_tdnn_17f.xconfig)
with the synthetic den graph and numerator FSTs of SURVEY §8d. Every timed step
also uploads its minibatch (fp32 features, numerator FSTs) on a copy stream, as
TrainStep's TransferBatch does (--no-h2d: inputs resident in HBM before timing).

Launch:
  python bench.py [--gpus N --steps K --warmup W]
    N = 1: one process on GPU 0.
    N > 1 without WORLD_SIZE in the environment: this process starts N worker
      processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*) before touching any
      GPU and exits with their status.
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
    one rank per GPU; WORLD_SIZE must equal --gpus.
  --selftest: the same launch and argument path on CPU (gloo), exchanging a flat
    gradient buffer by the network's bucket plan (no GPU needed).
Rank 0 prints ONE JSON line. At N = 1 it also carries sub-results measured in the
same run for BASELINE configs[0] (CPU affine + the GPU GEMM of the same shape),
configs[1] (forward only) and configs[4] (3072 model, MXFP8 GEMMs).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

# torch first: kfp16's libraries then bind to the same HIP runtime and RCCL (kfp16.hip_runtimes)
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kaldi-fp16_amd", "python"))

import numpy as np  # noqa: E402

METRIC = "frames/sec CNN-TDNN fwd+bwd, 40-dim×1500-frame egs, 1/2/4/8 MI355X"
METRIC_FWD = "frames/sec CNN-TDNN forward only, 40-dim×1500-frame egs, 1 MI355X"
PEAK_FP16_TFLOPS = 2500.0   # MI355X dense FP16 MFMA (MI355X_MICROARCH.md)
PEAK_FP8_TFLOPS = 5000.0    # MI355X dense FP8 (MX-scaled K=128 MFMA)
PEAK_HBM_GBPS = 8000.0      # MI355X HBM3E (MI355X_MICROARCH.md)
PEAK_L2_BPS = 34.5e12       # MI355X aggregate L2 read bandwidth (the den's arc-table streams)
FRAMES_PER_EG = 1500
# algorithmic MFLOP per input frame: forward, and forward +
# backward (dW of every layer, dX of all but IDCT and cnn1) — the step's FLOPs for the
# whole-step MFMA-roofline fraction north_star asks for
MODEL_MFLOP_PER_FRAME = {"cnn_tdnn_17f.xconfig": (66.24, 198.68),
                         "cnn_tdnn_17f_3072.xconfig": (165.27, 495.76)}
# kf_prof classes (include/kf_ops.h) and the step classes the bench line reports
PROF_CLASSES = {"gemm_fused": (0,), "conv_halo": (4,), "gemm_wgrad": (1,), "conv_wgrad": (5,),
                "slab_reduce": (6,), "chain_num": (2,), "chain_den": (3,)}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--egs", type=int, default=64, help="egs per GPU")
    p.add_argument("--xconfig", default="cnn_tdnn_17f.xconfig")
    # the reference's plain SGD has no max-change; with the chain gradient summed over
    # 31,360 supervised frames per GPU, 1e-8 keeps the random-init model from diverging
    p.add_argument("--lr", type=float, default=1e-8)
    p.add_argument("--momentum", type=float, default=0.9)
    p.add_argument("--bucket-mb", type=float, default=16.0,
                   help="gradient all-reduce bucket size (N > 1)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extra", action="store_true",
                   help="skip the configs[0]/[1]/[4] sub-results at N = 1")
    p.add_argument("--extra-steps", type=int, default=5)
    p.add_argument("--cpu-frames", type=int, default=1500)
    p.add_argument("--gt-frames", type=int, default=48, help="frames of the gotorch-style float64 CPU leg")
    p.add_argument("--cpu-threads", type=int, default=0, help="0: every host core")
    p.add_argument("--no-prof", action="store_true")
    p.add_argument("--no-h2d", action="store_true",
                   help="upload the step's inputs once before timing (default: TrainStep's per-minibatch "
                        "feature and numerator upload inside every step, overlapped on a copy stream)")
    p.add_argument("--input-pool", type=int, default=2, help="distinct host minibatches cycled through (h2d)")
    p.add_argument("--own-stream", action="store_true",
                   help="run the step on a non-blocking stream of its own instead of torch's default stream")
    p.add_argument("--h2d-mode", choices=("inline", "overlap"), default="inline",
                   help="inline: the step's uploads are the first work of the step on its stream; overlap: "
                        "on a copy stream during the previous step")
    p.add_argument("--implicit-dz", action="store_true",
                   help="TDNN-F consumers read g through the ReLU mask instead of a stored dz "
                        "(nnet_set_implicit_dz; default: dz stored)")
    p.add_argument("--no-wgrad-stream", action="store_true",
                   help="weight gradients on the main stream (default: their own stream, nnet_set_wgrad_stream)")
    p.add_argument("--all-rows", action="store_true",
                   help="train step on every row of every layer (the reference's Network.Forward / "
                        "Backward over all T rows) instead of the row-subsampled step (nnet_set_row_subsampling: "
                        "the layers above the conv stack on the rows the chain objective's output rows depend on)")
    p.add_argument("--fp8", action="store_true",
                   help="MXFP8 forward GEMMs (configs[4]; use with --xconfig cnn_tdnn_17f_3072.xconfig)")
    p.add_argument("--mode", choices=("train", "forward"), default="train",
                   help="train: the metric's fwd+bwd+SGD step; forward: configs[1], forward only")
    p.add_argument("--strict", action="store_true",
                   help="exit 3 when a sub-result or the CPU baseline failed (default: the failure is recorded "
                        "in sub_result_errors and the line, with the headline, is printed with exit status 0)")
    p.add_argument("--selftest", action="store_true",
                   help="CPU (gloo) check of the launcher and the bucketed gradient exchange")
    return p.parse_args(argv)


# --------------------------------------------------------------------------- launcher
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv):
    """Start n worker processes of this script, one per GPU, and return their exit
    status. Runs before anything touches a GPU; nothing is exec'd in place."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc
                for q in live:   # a dead rank leaves the others in a collective: stop them
                    q.terminate()
        time.sleep(0.05)
    return status


# --------------------------------------------------------------------------- helpers
def pmc_traffic(kernel_class):
    """HBM bytes per launch of a kernel class from the newest committed rocprofv3
    PMC summary (profiles/r*_pmc_traffic.json, scripts/pmc_traffic.sh), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as fh:
            rec = json.load(fh).get(kernel_class)
        return None if rec is None else {"bytes_per_launch": round(rec["hbm_bytes_per_launch"]),
                                         "source": os.path.relpath(files[-1], ROOT)}
    except (OSError, ValueError, KeyError):
        return None


def ivector_input(xcfg):
    """dim of the xconfig's `input name=ivector` (Kaldi's front end), else 0."""
    import re
    m = re.search(r"^\s*input\s+name=ivector\s+dim=(\d+)", xcfg, re.M)
    return int(m.group(1)) if m else 0


def box_hbm_probe():
    """HBM streaming rate of this box (torch copy of a [96,000 x 1536] fp16 tensor, the
    TDNN-F epilogue shape; median of 10, HIP events): the pool's MI355X boxes differ
    (memory-bound kernels run up to ~1.8x slower on some), so the line says which it ran on."""
    a = torch.empty((96000, 1536), dtype=torch.float16, device="cuda").fill_(1.0)
    c = torch.empty_like(a)
    c.copy_(a)
    ts = []
    for _ in range(10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        c.copy_(a)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = float(np.median(ts))
    del a, c
    torch.cuda.empty_cache()
    return {"copy_GBps": round(2 * 96000 * 1536 * 2 / (ms * 1e-3) / 1e9, 1),
            "probe": "torch copy of a [96000 x 1536] fp16 tensor (read + write), median of 10"}


def host_cores():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def step_classes(cls, steps, peak_tflops):
    """Per-class table of the timed steps (HIP events on each class's launch stream):
    launches and ms per step, and the class's algorithmic FLOPs / HBM bytes over its time as
    fractions of the dense MFMA and HBM peaks. The chain classes count other work: the
    numerator's arc updates (no fraction) and the den's algorithmic bytes, which stream the
    ~1 MB arc tables from L2 (fraction of the HBM peak shown for scale only)."""
    out = []
    for name, (n, ms, fl, by) in cls.items():
        if n == 0:
            continue
        sec = ms * 1e-3
        row = {"class": name, "launches_per_step": round(n / steps, 2), "ms_per_step": round(ms / steps, 3)}
        if name == "chain_num":
            row["arc_updates_per_s"] = round(fl / sec, 1) if sec > 0 else None
        elif name == "chain_den":
            # algorithmic bytes of the recursion and posteriors, mostly L2 arc-table streams
            row["alg_L2_GBps"] = round(fl / sec / 1e9, 1) if sec > 0 else None
            row["l2_frac"] = round(fl / sec / PEAK_L2_BPS, 4) if sec > 0 else None
        else:
            tf = fl / sec / 1e12 if sec > 0 else 0.0
            gbps = by / sec / 1e9 if sec > 0 else 0.0
            row.update({"mfma_tflops": round(tf, 1), "mfma_frac": round(tf / peak_tflops, 4),
                        "alg_GBps": round(gbps, 1), "hbm_frac": round(gbps / PEAK_HBM_GBPS, 4)})
        out.append(row)
    return out


def roofline(prof, steps, peak_tflops):
    """Dominant GEMM class: algorithmic FLOPs and algorithmic HBM bytes (kf_prof_collect2)
    over its HIP-event time on the launch stream. `bound` names the longer floor (FLOPs at
    the dense MFMA peak, bytes at the HBM peak); `regime` is "latency" when both floors are
    under half the measured time (neither roof binds), else the bound. `achieved` / `frac`
    are in the bound's unit, with both fractions beside them. With the weight-gradient
    stream the class's launches share the device with weight gradients, so
    their event times include that sharing."""
    dom = max(prof, key=lambda k: prof[k][1])
    n, ms, fl, by = prof[dom]
    t_mfma = fl / (peak_tflops * 1e12)
    t_hbm = by / (PEAK_HBM_GBPS * 1e9)
    sec = ms * 1e-3
    tf = fl / sec / 1e12 if sec > 0 else 0.0
    gbps = by / sec / 1e9 if sec > 0 else 0.0
    if t_hbm > t_mfma:
        r = {"bound": "hbm", "achieved": round(gbps, 1), "peak": PEAK_HBM_GBPS, "unit": "GB/s",
             "frac": round(gbps / PEAK_HBM_GBPS, 4)}
    else:
        r = {"bound": "mfma", "achieved": round(tf, 2), "peak": peak_tflops, "unit": "TFLOP/s",
             "frac": round(tf / peak_tflops, 4)}
    r["regime"] = "latency" if sec > 0 and max(t_hbm, t_mfma) < 0.5 * sec else r["bound"]
    r.update({"kernel": dom, "launches": n, "kernel_ms_per_step": round(ms / steps, 3),
              "mfma_tflops": round(tf, 2), "mfma_frac": round(tf / peak_tflops, 4),
              "alg_GBps": round(gbps, 1), "hbm_frac": round(gbps / PEAK_HBM_GBPS, 4),
              "alg_bytes_per_launch": round(by / max(n, 1)), "flops_per_launch": round(fl / max(n, 1)),
              "floor_ms_per_step": {"mfma": round(t_mfma * 1e3 / steps, 3), "hbm": round(t_hbm * 1e3 / steps, 3)},
              "all_gemm_tflops": round(sum(v[2] for v in prof.values()) /
                                       max(sum(v[1] for v in prof.values()) * 1e-3, 1e-12) / 1e12, 2)})
    return r


def cpu_baseline(xcfg, params, bns, frames, threads, den, num_fst, gt_frames=48):
    """The CPU baseline: the network in the reference's Go CPU
    style — oracle/gotorch_net.c, float64, AffineLayer / TDNNLayer / Conv1DLayer loop
    forms, forward GEMMs over `threads` as matmulParallel, SGD with momentum — timed
    on a bounded sample (forward, backward from a fixed output gradient, SGD; gotorch has
    no chain loss). Beside it, the C oracle's fp32 train step (forward, chain objective
    on the subsampled frames, backward) on a full 1500-frame eg. Restatements, not Go:
    no Go toolchain here."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from kfp16 import synth
    try:
        oracle.build(native=True)
        oracle.lib(native=True)
    except Exception:
        oracle.lib()
    tp = {k: synth.trunc_fp16(v) for k, v in params.items()}
    D = ivector_input(xcfg)
    name = "cnn_tdnn_17f with the ivector front end" if D else "cnn_tdnn_17f"
    res = {"unit": "frames/sec", "cores": threads, "host_cores": host_cores(), "kind": "port"}
    # gotorch-style float64 leg (the template has no ivector branch)
    if not D:
        on = oracle.OracleNet(xcfg, tp, bns, round_mode=oracle.ROUND_NONE, threads=threads)
        gt = oracle.GotorchNet(on, workers=threads)
        feats = synth.make_features(gt_frames, 40).astype(np.float64)
        og = np.random.default_rng(5).standard_normal((gt_frames, on.L[on.chain_output()]["out_dim"])) * 0.01
        t0 = time.perf_counter()
        gt.forward(feats)
        t_fwd = time.perf_counter() - t0
        gt.backward(og)
        gt.sgd(1e-8)
        dt = time.perf_counter() - t0
        gt.close()
        on.close()
        res.update({"value": round(gt_frames / dt, 3), "forward_frames_per_sec": round(gt_frames / t_fwd, 3),
                    "sample": f"restatement, not Go: {name} in go/gotorch's CPU style (oracle/gotorch_net.c: "
                              f"float64; TDNN-F halves as TDNNLayer and conv as Conv1DLayer loops, "
                              f"single-threaded as in layers.go:443-522 / cnn_tdnn.go:85-172; affine forward "
                              f"GEMMs as matmulParallel over {threads} threads, ops.go:49-81; SGD momentum "
                              f"0.9) on {gt_frames} frames: forward, backward from a fixed output gradient, "
                              f"SGD, {dt:.1f} s (forward {t_fwd:.1f} s)"})
    # the fp32 C oracle's train step with the chain objective, on one full eg
    on = oracle.OracleNet(xcfg, tp, bns, round_mode=oracle.ROUND_FUSED, threads=threads)
    feats = synth.make_features(frames, 40).astype(np.float32)
    g, init = den
    row0, nfr, stride = synth.chain_layout(1, frames)
    rows = row0[0] + np.arange(nfr[0]) * stride
    iv = (np.random.default_rng(5).standard_normal((1, D)) * 2).astype(np.float32) if D else None
    t0 = time.perf_counter()
    if D:
        on.forward(feats, ivectors=iv, seq_off=np.array([0, frames], np.int32))
    else:
        on.forward(feats)
    t_fwd = time.perf_counter() - t0
    out = on.act("output")
    deriv, _ = oracle.chain_objf(g, init, num_fst, out[rows])
    og = np.zeros_like(out)
    og[rows] = (-deriv).astype(np.float16).astype(np.float32)
    on.backward(og)
    dt = time.perf_counter() - t0
    on.close()
    fp32 = {"value": round(frames / dt, 2), "forward_frames_per_sec": round(frames / t_fwd, 2),
            "sample": f"restatement, not Go: C oracle train step (fwd, chain objective, bwd) of {name} on "
                      f"{frames} frames (1 eg), fp32, GEMM rows split over {threads} threads, {dt:.1f} s; "
                      f"forward alone {t_fwd:.1f} s"}
    if "value" in res:
        res["oracle_fp32"] = fp32
    else:
        res.update(fp32)
    return res


def config1_affine(threads, reps=50):
    """BASELINE configs[0]: gotorch.AffineLayer(40, 512).Forward on [1500 x 40] float64
    (go/gotorch/layers.go:57-70, ops.go:15-81), restated in C (oracle/gotorch_cpu.c),
    median of `reps`; next to the same affine on the GPU through the reference's
    ops_gemm ABI (fp16 MFMA, fp32 accumulation), median of `reps` event-timed calls."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    import kfp16
    rng = np.random.default_rng(0)
    M, K, N = 1500, 40, 512
    x = rng.standard_normal((M, K))
    W = rng.standard_normal((K, N)) * np.sqrt(2.0 / (K + N))
    b = np.zeros(N)
    L = oracle.lib()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        y = oracle.gotorch_affine_forward(x, W, b, threads, L)
        ts.append(time.perf_counter() - t0)
    cpu_ms = float(np.median(ts)) * 1e3
    # GPU: ops_gemm (ops.h) on fp16 copies, the kaldi-fp16 plumbing of the same layer
    xa = torch.from_numpy(x.astype(np.float16)).cuda()
    wa = torch.from_numpy(W.astype(np.float16)).cuda()
    ya = torch.empty((M, N), dtype=torch.float16, device="cuda")
    h = kfp16.core.ops_cublas_create()
    st = torch.cuda.current_stream()
    for _ in range(3):
        kfp16.check(kfp16.core.ops_gemm(h, M, N, K, 1.0, xa.data_ptr(), K, wa.data_ptr(), N, 0.0,
                                        ya.data_ptr(), N), "ops_gemm")
    g = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        kfp16.core.ops_gemm(h, M, N, K, 1.0, xa.data_ptr(), K, wa.data_ptr(), N, 0.0, ya.data_ptr(), N)
        e1.record(st)
        e1.synchronize()
        g.append(e0.elapsed_time(e1))
    kfp16.core.ops_cublas_destroy(h)
    err = float(np.abs(ya.float().cpu().numpy() - y).max() / np.abs(y).max())
    gpu_ms = float(np.median(g))
    return {"workload": "AffineLayer(40,512).Forward on [1500 x 40] (configs[0])",
            "cpu_ms_median": round(cpu_ms, 3), "cpu_frames_per_sec": round(M / (cpu_ms * 1e-3), 1),
            "cpu": {"kind": "port", "cores": threads, "host_cores": host_cores(), "reps": reps,
                    "sample": "restatement, not Go: oracle/gotorch_cpu.c, float64, matmulParallel rows "
                              "over the thread count"},
            "gpu_ops_gemm_ms_median": round(gpu_ms, 4), "gpu_frames_per_sec": round(M / (gpu_ms * 1e-3), 1),
            "gpu_vs_cpu_max_rel_err": round(err, 5)}


def dropin_forward(a, reps=3):
    """The drop-in path timed beside the fused one: the reference's own
    Network.Forward host sequence over the per-op C-ABI (kfp16.refpath: ops_gemm,
    K = 1-GEMM AddBias, ops_relu, ops_batchnorm_forward, ops_copy / ops_concat_cols
    splices, ops_add_scaled) against nnet_forward on the same layers and input. Both run
    the TDNN-F stack of cnn_tdnn_17f (tdnnf7 ... output, fed a [T x 2560] input in place
    of cnn6's activation: the reference's conv front end im2cols on the host,
    forward.go:435-456, which would time the host, not the ABI) at 64 egs."""
    import kfp16
    from kfp16 import refpath, synth
    text = synth.load_xconfig("cnn_tdnn_17f.xconfig").splitlines()
    k = next(i for i, l in enumerate(text) if "name=tdnnf7" in l)
    xcfg = "\n".join(["input name=input dim=2560"] + text[k:]) + "\n"
    T = a.egs * FRAMES_PER_EG
    net = kfp16.Network(xcfg, max_frames=T)
    params, bns = synth.init_network(net, seed=42)
    rp = refpath.RefPathForward(xcfg, params, bns, T)
    x = (torch.randn(T, 2560, device="cuda", generator=torch.Generator(device="cuda").manual_seed(3)) * 0.5).half()
    st = torch.cuda.current_stream()

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        e1.synchronize()
        return e0.elapsed_time(e1) / reps
    ms_fused = timed(lambda: net.forward(x.data_ptr(), T))
    ms_ref = timed(lambda: rp.forward(x.data_ptr(), T))
    got = rp.read("output").astype(np.float32)
    ref = net.read_activation("output").astype(np.float32)
    err = float(np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30))
    n_ops = rp.ncalls
    rp.close()
    net.close()
    return {"workload": f"tdnnf7 ... output of cnn_tdnn_17f, forward, {a.egs} egs x 1500 frames",
            "dropin_per_op_abi_ms": round(ms_ref, 3), "dropin_frames_per_sec": round(T / (ms_ref * 1e-3), 1),
            "fused_nnet_forward_ms": round(ms_fused, 3), "fused_frames_per_sec": round(T / (ms_fused * 1e-3), 1),
            "speedup_fused_over_dropin": round(ms_ref / ms_fused, 2), "abi_calls_per_forward": n_ops,
            "output_rel_fro_dropin_vs_fused": round(err, 5),
            "path": "kfp16.refpath: forward.go:589-1001's ABI sequence (spliceBackward / spliceForward by "
                    "ops_copy + ops_concat_cols, ops_gemm, AddBias as the K = 1 ops_gemm of ops.go:335, ops_relu, "
                    "ops_batchnorm_forward, ops_add_scaled); buffers allocated once"}


# --------------------------------------------------------------------------- selftest (CPU)
def selftest(a, rank, world):
    """gloo: the bench's launch / argument path plus the bucketed exchange of a flat
    gradient buffer laid out and planned by the product (nnet_create_layout,
    nnet_dp_plan), checked against the rank average."""
    import kfp16
    from kfp16 import dp, synth
    dist.init_process_group("gloo")
    assert dist.get_world_size() == a.gpus == world
    net = kfp16.Network(synth.load_xconfig(a.xconfig), max_frames=1, layout_only=True)
    plan = net.dp_plan(int(a.bucket_mb * (1 << 20)))
    assert dp.covers_exactly(plan, net.num_params)
    grads = [np.random.default_rng(100 + r).standard_normal(net.num_params).astype(np.float32)
             for r in range(world)]
    flat = torch.from_numpy(grads[rank].copy())
    dp.exchange_by_plan(flat, plan, world)
    want = np.mean(np.stack(grads), axis=0, dtype=np.float64).astype(np.float32)
    err = float(np.abs(flat.numpy() - want).max())
    ok = torch.tensor([1.0 if err < 1e-6 else 0.0])
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    t = dp.max_over_ranks(float(rank), "cpu")
    if rank == 0:
        print(json.dumps({"selftest": bool(ok.item() == 1.0), "n_gpus": world, "backend": "gloo",
                          "xconfig": a.xconfig, "num_params": net.num_params, "buckets": len(plan),
                          "plan": plan, "max_abs_err": err, "max_over_ranks": t}), flush=True)
    net.close()
    dist.destroy_process_group()
    return 0 if ok.item() == 1.0 else 1


# --------------------------------------------------------------------------- one workload
def run_workload(a, xconfig, mode, fp8, rank, world, comm, steps, warmup, prof_on, keep=False):
    """Build the network, den graph and egs of one workload, time `steps` steps.
    Returns (stats dict, context for the CPU baseline)."""
    import kfp16
    from kfp16 import chain, dp, synth

    T = a.egs * FRAMES_PER_EG
    xcfg = synth.load_xconfig(xconfig)
    net = kfp16.Network(xcfg, max_frames=T)
    params, bns = synth.init_network(net, seed=42)        # identical replicas on every rank
    if fp8:
        net.set_fp8(True)
    if a.no_wgrad_stream:
        net.set_wgrad_stream(False)
    if a.implicit_dz:
        net.set_implicit_dz(True)
    bucket_bytes = int(a.bucket_mb * (1 << 20))
    if comm is not None and mode == "train":
        net.bind_dp(comm, bucket_bytes)                    # bucketed all-reduce inside backward
    # row-subsampled train step (kf_nnet.h nnet_set_row_subsampling): the chain objective reads
    # the output on rows 0 (mod 3) (row0 = 1500 e + 30, frame subsampling 3), so the layers above
    # the conv stack run on those rows and the clamped-edge tail; the objective then reads the
    # compact output rows (row c = source row 3c)
    rsub = mode == "train" and not fp8 and not a.all_rows and not a.implicit_dz
    if rsub:
        try:
            net.set_row_subsampling(3)
        except kfp16.KfError:   # a topology it does not cover (e.g. attention above the convs)
            rsub = False

    P = net.layers[-1][3]
    # chain supervision: shared den graph, one numerator FST per eg
    # (seed 7 + global eg index); the objective writes the output gradient on the
    # subsampled rows (leftCtx 30, stride 3) — every other row stays zero
    den_g = synth.make_den_graph(num_pdfs=P)
    dgraph = chain.DenGraph(den_g)
    h2d = mode == "train" and not a.no_h2d
    npool = max(1, a.input_pool) if h2d else 1
    # this rank's shards of egs: features (fp32, as the loader holds them) and numerator FSTs
    # of `npool` distinct host minibatches (pool 0 is the r4 bench's minibatch)
    feats_pool = [synth.make_features(T, 40, seed=1234 + rank + 7919 * b) for b in range(npool)]
    packs = [chain.pack_num_fsts([synth.make_num_fst(dp.eg_index(rank, a.egs, e) + 104729 * b, num_pdfs=P)
                                  for e in range(a.egs)]) for b in range(npool)]
    row0, nfr, stride = synth.chain_layout(a.egs, FRAMES_PER_EG)
    objective = chain.Chain(dgraph, max_seqs=a.egs, max_frames=int(nfr.max()))
    out_ptr = net.activation("output")[0]
    ivd = ivector_input(xcfg)
    if ivd:  # Kaldi's ivector front end: one ivector per eg, one sequence per eg
        ivecs = (np.random.default_rng(99 + rank).standard_normal((a.egs, ivd)) * 2).astype(np.float16)
        ibuf = torch.from_numpy(ivecs.view(np.int16)).to("cuda")
        seq_off = np.arange(a.egs + 1, dtype=np.int32) * FRAMES_PER_EG
    obj_rows, obj_row0, obj_stride = T, row0, stride
    prime_launches = 0
    if rsub:
        # the compact row set of this T (one untimed forward), and the objective's layout in it
        fz = torch.zeros((T, 40), dtype=torch.float16, device="cuda")
        if prof_on:   # count the priming forward's fused-class launches (rocprof window check)
            kfp16.core.kf_prof_reset()
            kfp16.core.kf_prof_reserve(256)
            kfp16.core.kf_prof_enable(1)
        if ivd:
            net.forward_ivector(fz.data_ptr(), T, ibuf.data_ptr(), seq_off)
        else:
            net.forward(fz.data_ptr(), T)
        if prof_on:
            torch.cuda.synchronize()
            kfp16.core.kf_prof_enable(0)
            prime_launches = sum(1 for x in kfp16.prof_records() if x["cls"] in (0, 4))
            kfp16.core.kf_prof_reset()
        tc, tc0, _ = net.row_set()
        if tc and stride == 3 and np.all(row0 % 3 == 0):
            obj_rows, obj_row0, obj_stride = tc, row0 // 3, 1
        else:
            net.set_row_subsampling(0)
            rsub = False
        del fz
    gbuf = torch.zeros((obj_rows, P), dtype=torch.float16, device="cuda")
    torch.cuda.synchronize()


    comp = torch.cuda.current_stream()
    inline = h2d and a.h2d_mode == "inline"
    if h2d:
        # TrainStep's input stage (train_step.go:155 TransferBatch -> bridge.cu:206-267, and the
        # per-sequence FST uploads of chain_loss.go:44-97) inside every timed step: step i+1's
        # fp32 features (pinned host) and numerator FSTs (kf_num_batch_refill) go up on a copy
        # stream while step i computes; the step then rounds its features to fp16 (RNE,
        # fp16.go:12-70) on the GPU. Two device slots; events order reuse.
        if inline:
            copy = comp
        else:
            # a NON-BLOCKING copy stream (kf_stream_new): torch's streams are blocking ones,
            # which the legacy default stream the step runs on synchronises with implicitly
            import ctypes
            kfp16.core.kf_stream_new.restype = ctypes.c_void_p
            copy = torch.cuda.ExternalStream(kfp16.core.kf_stream_new())
        host = [torch.from_numpy(f).pin_memory() for f in feats_pool]
        f32 = [torch.empty((T, 40), dtype=torch.float32, device="cuda") for _ in range(2)]
        fbufs = [torch.empty((T, 40), dtype=torch.float16, device="cuda") for _ in range(2)]
        nums = [chain.NumBatch(packs[0]), chain.NumBatch(packs[min(1, npool - 1)])]
        ev_copied = [torch.cuda.Event() for _ in range(2)]
        ev_conv = [torch.cuda.Event() for _ in range(2)]
        ev_obj = [torch.cuda.Event() for _ in range(2)]
        ev_fwd = torch.cuda.Event()   # this step's forward done: the den recursion runs next
        for nb in nums:   # the first refill frees the create-time upload (one device sync), untimed
            nb.refill(packs[0], copy.cuda_stream)
        # setup, untimed: every host minibatch once through each device slot (the copy
        # engine's first transfers from a pinned buffer ran slow: with three warm-up steps the
        # first three timed steps took 27.2 / 26.8 / 26.0 ms against 24.5, and none with the
        # inputs resident)
        for b in range(npool):
            for sl in range(2):
                with torch.cuda.stream(copy):
                    f32[sl].copy_(host[b], non_blocking=True)
                nums[sl].refill(packs[b], copy.cuda_stream)
        torch.cuda.synchronize()
        state = {"i": 0}

        def stage(i):
            """step i's inputs into slot i % 2, on the copy stream (inline: the step's stream)"""
            sl = i % 2
            if not inline:
                copy.wait_event(ev_conv[sl])    # the slot's fp32 features were converted (step i - 2)
                copy.wait_event(ev_obj[sl])     # the slot's numerator was used (step i - 2)
                # and not before step i - 1's forward has finished: the copies then run under
                # its den recursion (latency-bound, ~5 ms). Issued whenever the host got there,
                # they sometimes landed under the den posteriors, which then took ~0.9 ms longer.
                copy.wait_event(ev_fwd)
            with torch.cuda.stream(copy):
                f32[sl].copy_(host[i % npool], non_blocking=True)
                ev_copied[sl].record(copy)
            nums[sl].refill(packs[i % npool], copy.cuda_stream)

        if not inline:
            stage(0)
    else:
        feats = feats_pool[0]
        fbuf = torch.from_numpy(feats.view(np.int16)).to("cuda")
        nbatch = chain.NumBatch(packs[0])

    def step():
        if h2d:
            i = state["i"]
            sl = i % 2
            if inline:
                stage(i)
            comp.wait_event(ev_copied[sl])
            kfp16.check(kfp16.core.bridge_fp32_to_fp16_gpu(fbufs[sl].data_ptr(), f32[sl].data_ptr(), T * 40),
                        "bridge_fp32_to_fp16_gpu")
            ev_conv[sl].record(comp)
            fptr, num = fbufs[sl].data_ptr(), nums[sl]
        else:
            fptr, num = fbuf.data_ptr(), nbatch
        if ivd:
            net.forward_ivector(fptr, T, ibuf.data_ptr(), seq_off)
        else:
            net.forward(fptr, T)
        if h2d:
            ev_fwd.record(comp)
        if mode == "forward":
            return
        objective.compute(num, out_ptr, P, obj_rows, obj_row0, nfr, obj_stride, gbuf.data_ptr(), P)
        if h2d:
            ev_obj[sl].record(comp)
            if not inline:
                stage(i + 1)                # the next step's inputs, overlapped with this backward
            state["i"] = i + 1
        net.backward(gbuf.data_ptr())       # + the overlapped gradient all-reduce (N > 1)
        net.sgd(a.lr, a.momentum)

    # host-side setup of the timed region before the warm-up (the per-launch events, the
    # per-step events), so the warm-up steps run straight into the timed ones: a long host
    # gap here left the GPU idle and the first timed steps 2-4 ms slower
    if prof_on:
        kfp16.core.kf_prof_reserve(256 * steps)   # ~190 profiled launches per step
    st = torch.cuda.current_stream()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    for _ in range(warmup):
        step()
        if os.environ.get("KF_BENCH_CHECK") and mode == "train":
            r = objective.result()
            print("warmup objf/frame", r.objf / max(r.frames, 1), "ok", r.num_ok, flush=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    if prof_on:
        kfp16.core.kf_prof_reset()
        kfp16.core.kf_prof_enable(1)
    dp0 = comm.stats() if comm is not None else (0, 0)
    # per-step HIP events on the launch stream (the library runs on torch's current stream):
    # the median step beside the wall-clock mean (median of the timed steps)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    t_issue = []
    for i in range(steps):
        evs[i].record(st)
        t_issue.append(time.perf_counter())
        step()
    t_issue.append(time.perf_counter())
    evs[steps].record(st)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kfp16.core.kf_prof_enable(0)
    kfp16.core.kf_take_pending(b"the bench's check after the timed steps (torch.cuda.synchronize)")
    step_ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(steps)]
    kfp16.core.kf_take_pending(b"the bench's check after torch.cuda.Event.elapsed_time")
    median_ms = dp.max_over_ranks(float(np.median(step_ms)), "cpu")
    elapsed = dp.max_over_ranks(elapsed, "cpu")
    dp1 = comm.stats() if comm is not None else (0, 0)

    prof, chain_prof, classes = {}, {}, {}
    if prof_on:
        for name, ids in PROF_CLASSES.items():
            classes[name] = kfp16.prof_collect2(ids[0])
        # the dominant class of the roofline: every fused launch (tiled GEMM + conv halo),
        # and every weight-gradient GEMM launch
        add = lambda a, b: tuple(x + y for x, y in zip(a, b))  # noqa: E731
        prof["gemm_fused"] = add(classes["gemm_fused"], classes["conv_halo"])
        prof["gemm_wgrad"] = add(classes["gemm_wgrad"], classes["conv_wgrad"])
        for name in ("chain_num", "chain_den"):
            chain_prof[name] = classes[name][:3]
        kfp16.core.kf_prof_reset()
    stats = [0.0] * 5

    def probe(where):
        """attribute a HIP error left pending by the torch call just made (kf_take_pending
        logs it under `where`; the library's own entry checks would otherwise see it first)"""
        if kfp16.core.kf_peek_error():
            kfp16.core.kf_take_pending(("the bench's check after " + where).encode())
    if mode == "train":
        # fails if a den exchange timed out in ANY step since the previous result
        # (warm-up and timed steps): a silently wrong gradient is never reported
        res = objective.result()
        probe("kf_chain_result")
        stats = dp.sum_over_ranks([res.objf, res.num_logprob, res.den_logprob, res.frames, res.num_ok],
                                  "cpu")
        probe("dp.sum_over_ranks")
    cpu_issue_ms = [(t_issue[i + 1] - t_issue[i]) * 1e3 for i in range(steps)]
    out = {"T": T, "elapsed": elapsed, "median_ms": median_ms, "step_ms": step_ms, "cpu_issue_ms": cpu_issue_ms, "steps": steps, "prof": prof, "chain_prof": chain_prof, "classes": classes,
           "xconfig": xconfig, "mode": mode, "h2d": h2d, "input_pool": npool, "rsub": rsub,
           "obj_rows": obj_rows, "prime_launches": prime_launches,
           "stats": stats, "ivd": ivd, "dp": (dp1[0] - dp0[0], dp1[1] - dp0[1]),
           "buckets": len(net.dp_plan(bucket_bytes)) if comm is not None else 0}
    ctx = (xcfg, params, bns, den_g, P) if keep else None
    torch.cuda.synchronize()
    probe("torch.cuda.synchronize")
    for nb in (nums if h2d else [nbatch]):
        nb.close()
    objective.close()
    net.close()
    return out, ctx


def describe(r, a, world, mode, fp8, xconfig, peak):
    # ms_per_step: median of the timed steps (max over ranks); value: whole-job frames over
    # the wall clock of all timed steps, whose mean step is reported beside the median
    mean_ms = r["elapsed"] / r["steps"] * 1e3
    value = r["T"] * world * r["steps"] / r["elapsed"]
    d = {"value": round(value, 1), "ms_per_step": round(r["median_ms"], 3), "ms_per_step_mean": round(mean_ms, 3),
         "row_subsampled": bool(r.get("rsub")),
         "ms_per_step_min_max": [round(min(r["step_ms"]), 3), round(max(r["step_ms"]), 3)],
         "step_ms": [round(x, 2) for x in r["step_ms"]],
         "cpu_issue_ms": [round(x, 2) for x in r["cpu_issue_ms"]]}
    mf = MODEL_MFLOP_PER_FRAME.get(r["xconfig"])
    if mf is not None:
        # whole step against the dense FP16 MFMA roofline: frames/s x algorithmic FLOPs per
        # frame / 2.5 PF. Also for the MXFP8 step, whose backward stays mostly fp16 (its
        # fp8 share is in roofline.classes): against the 5 PF fp8 peak it would read ~2x
        # low and not compare with the fp16 step
        fpf = mf[1] if r["mode"] == "train" else mf[0]
        if r.get("rsub") and r["prof"]:
            # the row-subsampled step executes fewer GEMM FLOPs than the all-rows model count:
            # price the step by what its GEMMs executed (kf_prof classes)
            gemm_fl = sum(r["classes"][k][2] for k in ("gemm_fused", "conv_halo", "gemm_wgrad", "conv_wgrad"))
            fpf = round(gemm_fl / (r["T"] * r["steps"]) / 1e6, 2)
            d["step_mflop_per_frame_all_rows"] = mf[1]
        d["step_mfma_frac"] = round(value * fpf * 1e6 / (PEAK_FP16_TFLOPS * 1e12), 4)
        d["step_mfma_peak"] = "fp16 dense 2.5 PF"
        d["step_mflop_per_frame"] = fpf
    if r["prof"]:
        d["roofline"] = roofline(r["prof"], r["steps"], peak)
        d["roofline"]["classes"] = step_classes(r["classes"], r["steps"], peak)
        # GEMM FLOPs the step executed on MFMA per frame (check of the constant above)
        gemm_fl = sum(r["classes"][k][2] for k in ("gemm_fused", "conv_halo", "gemm_wgrad", "conv_wgrad"))
        d["roofline"]["executed_gemm_mflop_per_frame"] = round(gemm_fl / (r["T"] * r["steps"]) / 1e6, 2)
        # fused-class launches of the untimed priming forward (row set), before the warm-up
        # steps: scripts/fused_class_check.py skips them to find the timed window in a trace
        d["roofline"]["priming_launches"] = r.get("prime_launches", 0)
    if mode == "train":
        st = r["stats"]
        d["objf_per_frame"] = round(float(st[0]) / max(float(st[3]), 1.0), 5)
        d["objective_finite_seqs"] = f"{int(st[4])}/{a.egs * world}"
    return d


def sub_results(a, rank, world, prof_on):
    """The N = 1 sub-results measured after the headline (configs[1], configs[4], the drop-in
    per-op path, the one-stream step), in this order. Each runs on its own: one that raises
    is recorded as {"error": ...} (with the library's pending-error log) and the rest still
    run, so a failing sub-result never discards the headline line. Returns (results, errors)."""
    import copy
    import traceback
    import kfp16
    ks, kw = a.extra_steps, 2
    extra, errors = {}, {}

    def guarded(name, fn):
        try:
            fn()
        except Exception as e:  # noqa: BLE001 -- recorded, reported, and the run continues
            torch.cuda.synchronize()
            errors[name] = {"error": f"{type(e).__name__}: {e}", "pending_log": kfp16.pending_log(),
                            "where": traceback.format_exc(limit=4)}
            extra[name] = {"error": errors[name]["error"]}
            print(f"bench.py: sub-result {name} failed: {e}", file=sys.stderr, flush=True)

    def fwd_1536():
        r, _ = run_workload(a, "cnn_tdnn_17f.xconfig", "forward", False, rank, world, None, ks, kw, prof_on)
        extra["configs[1]_forward_1536"] = dict(
            workload="cnn_tdnn_17f forward only, fp16", **describe(r, a, world, "forward", False, "", PEAK_FP16_TFLOPS))
    guarded("configs[1]_forward_1536", fwd_1536)

    # the 3072 train step in fp16 and in MXFP8, A/B/A/B in this process: each sub-result
    # is its second run; the speedup compares the means of both runs of each mode (both on
    # every row: the MXFP8 step has no row-subsampled form)
    af = copy.copy(a)
    af.all_rows = True

    def train_3072():
        ms_ab = {False: [], True: []}
        for rep in range(2):
            for f8 in (False, True):
                r, _ = run_workload(af, "cnn_tdnn_17f_3072.xconfig", "train", f8, rank, world, None, ks, kw, prof_on)
                d = describe(r, af, world, "train", f8, "", PEAK_FP8_TFLOPS if f8 else PEAK_FP16_TFLOPS)
                ms_ab[f8].append(d["ms_per_step"])
                if rep == 1 and not f8:
                    extra["configs[4]_train_3072_fp16"] = dict(
                        workload="cnn_tdnn_17f_3072 train step (fwd+bwd+SGD), fp16, every row (the MXFP8 step's "
                                 "reference point)",
                        **d)
                elif rep == 1:
                    extra["configs[4]_train_3072_mxfp8"] = dict(
                        workload="cnn_tdnn_17f_3072 train step (fwd+bwd+SGD), every row: MXFP8 forward GEMMs and "
                                 "strided TDNN-F affine input gradients, the rest fp16", **d)
        m8 = extra["configs[4]_train_3072_mxfp8"]
        m8["ms_per_step_ab"] = {"fp16": ms_ab[False], "mxfp8": ms_ab[True]}
        m16, m8ms = sum(ms_ab[False]) / 2, sum(ms_ab[True]) / 2
        m8["speedup_vs_fp16_step"] = round(m16 / m8ms, 4) if m8ms else None
    guarded("configs[4]_train_3072", train_3072)

    def fwd_3072_fp8():
        r, _ = run_workload(a, "cnn_tdnn_17f_3072.xconfig", "forward", True, rank, world, None, ks, kw, prof_on)
        extra["configs[4]_forward_3072_mxfp8"] = dict(
            workload="cnn_tdnn_17f_3072 forward only, MXFP8 GEMMs",
            **describe(r, a, world, "forward", True, "", PEAK_FP8_TFLOPS))
    guarded("configs[4]_forward_3072_mxfp8", fwd_3072_fp8)

    def dropin():
        extra["dropin_per_op_abi_forward"] = dropin_forward(a)
    guarded("dropin_per_op_abi_forward", dropin)

    # the same train step with the weight gradients on the chain's stream: its
    # roofline prices the fused class without the weight gradients running beside it
    def one_stream():
        a1 = copy.copy(a)
        a1.no_wgrad_stream = True
        r, _ = run_workload(a1, "cnn_tdnn_17f.xconfig", "train", False, rank, world, None, ks, kw, prof_on)
        extra["train_1536_one_stream"] = dict(
            workload="the headline train step with the weight gradients on the input-gradient chain's stream "
                     "(nnet_set_wgrad_stream 0): per-launch times of the fused class without co-running work",
            **describe(r, a1, world, "train", False, "cnn_tdnn_17f.xconfig", PEAK_FP16_TFLOPS))
    guarded("train_1536_one_stream", one_stream)

    # the headline step on every row of every layer (the reference's row coverage)
    def all_rows():
        r, _ = run_workload(af, "cnn_tdnn_17f.xconfig", "train", False, rank, world, None, ks, kw, prof_on)
        extra["train_1536_all_rows"] = dict(
            workload="the headline train step with every layer on all T rows (--all-rows: no row subsampling, "
                     "the reference's Network.Forward / Backward row coverage)",
            **describe(r, af, world, "train", False, "cnn_tdnn_17f.xconfig", PEAK_FP16_TFLOPS))
    guarded("train_1536_all_rows", all_rows)
    return extra, errors


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return spawn_ranks(a.gpus, sys.argv[1:])
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    if a.selftest:
        return selftest(a, rank, world)
    if world > 1:
        # control plane only (barriers, the max-over-ranks step time, the RCCL id and the
        # objective statistics, all host values): the data path's one GPU communicator is
        # kf_dp's RCCL one, so torch does not open a second RCCL communicator per GPU
        dist.init_process_group("gloo")
        assert dist.get_world_size() == a.gpus
    torch.cuda.set_device(local)

    import kfp16
    from kfp16 import dp
    kfp16.check(kfp16.core.bridge_gpu_init(local), "bridge_gpu_init")
    stream = torch.cuda.Stream() if a.own_stream else torch.cuda.current_stream()
    torch.cuda.set_stream(stream)
    kfp16.set_stream(stream.cuda_stream)
    kfp16.assert_single_hip_runtime()
    comm = dp.Communicator.from_process_group(local) if world > 1 else None
    rccl_ranks = kfp16.core.kf_dp_world(comm.h) if comm is not None else 1

    prof_on = not a.no_prof
    peak = PEAK_FP8_TFLOPS if a.fp8 else PEAK_FP16_TFLOPS
    box = box_hbm_probe()
    head, ctx = run_workload(a, a.xconfig, a.mode, a.fp8, rank, world, comm, a.steps, a.warmup, prof_on,
                             keep=True)
    extra, errors = {}, {}
    if world == 1 and not a.no_extra and a.xconfig == "cnn_tdnn_17f.xconfig" and a.mode == "train" and not a.fp8:
        extra, errors = sub_results(a, rank, world, prof_on)

    if rank == 0:
        # the box's CPU share (OMP_NUM_THREADS is set to it there; nproc shows the whole host)
        threads = a.cpu_threads or min(host_cores(), int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or
                                       host_cores())
        if world == 1 and not a.no_extra and not a.no_cpu_baseline:
            try:
                extra["configs[0]_affine_40x512"] = config1_affine(threads)
            except Exception as e:  # noqa: BLE001 -- recorded; the headline still prints
                errors["configs[0]_affine_40x512"] = {"error": f"{type(e).__name__}: {e}"}
                extra["configs[0]_affine_40x512"] = errors["configs[0]_affine_40x512"]
        fwd_only = a.mode == "forward"
        workload = ("cnn_tdnn_17f forward only (configs[1])" if fwd_only else
                    "cnn_tdnn_17f train step (fwd+bwd+SGD)") + f", {a.egs} egs x 1500 frames per GPU"
        if head["ivd"]:
            workload += f", Kaldi ivector front end ({head['ivd']}-dim ivector per eg)"
        d = describe(head, a, world, a.mode, a.fp8, a.xconfig, peak)
        out = {
            "metric": METRIC_FWD if fwd_only else METRIC, "value": d["value"], "unit": "frames/sec",
            "n_gpus": world, "rccl_ranks": rccl_ranks,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": d["ms_per_step"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "mxfp8 GEMMs (e4m3 + E8M0), fp16 storage" if a.fp8 else "fp16",
            "data": "synthetic",
            "config": {"workload": workload,
                       "xconfig": a.xconfig, "egs_per_gpu": a.egs, "frames_per_eg": FRAMES_PER_EG,
                       "global_batch_egs": a.egs * world, "parallelism": f"dp{world}",
                       "h2d_in_step": bool(head["h2d"]),
                       "inputs": (("per step, first on the step's stream: " if a.h2d_mode == "inline" else
                                   "per step, on a copy stream during the previous step: ") +
                                  "fp32 features from pinned host memory and the minibatch's numerator FSTs "
                                  "(kf_num_batch_refill) uploaded, then RNE to fp16 on the GPU; "
                                  f"{head['input_pool']} distinct host minibatches cycled")
                                 if head["h2d"] else "resident in HBM before timing",
                       "objective": "chain LF-MMI (den S=7052 A=113380, num 250 states/eg, fps 490)",
                       "rows": ("row-subsampled (nnet_set_row_subsampling 3): tdnnf7 .. output on the "
                                f"{head['obj_rows']} rows the objective's output rows 0 (mod 3) depend on, "
                                "cnn6 on those rows too (its time-strided conv), cnn1 .. cnn5 on all rows; "
                                "objective and gradients as on all rows"
                                if head.get("rsub") else "every layer on all T rows")},
        }
        out["ms_per_step_mean"] = d["ms_per_step_mean"]
        out["ms_per_step_min_max"] = d["ms_per_step_min_max"]
        out["step_ms"] = d["step_ms"]
        out["cpu_issue_ms"] = d["cpu_issue_ms"]
        for k in ("step_mfma_frac", "step_mfma_peak", "step_mflop_per_frame", "step_mflop_per_frame_all_rows", "objf_per_frame",
                  "objective_finite_seqs"):
            if k in d:
                out[k] = d[k]
        out["box"] = box
        out["wgrad_stream"] = not a.no_wgrad_stream
        out["implicit_dz"] = bool(a.implicit_dz)
        if not fwd_only:
            out["den_exchange_timeouts"] = 0   # kf_chain_result raised otherwise
        if world > 1:
            n, v = head["dp"]
            out["dp"] = {"collective": "kf_dp ncclAllReduce(avg) over RCCL, bucketed, overlapped with backward",
                         "bucket_mb": a.bucket_mb, "buckets_per_step": head["buckets"],
                         "allreduce_launches_per_step": round(n / a.steps, 2),
                         "values_per_step": int(v / a.steps)}
        cp = head["chain_prof"]
        if cp and not fwd_only:
            (nn, nms, _), (dn, dms, dbytes) = cp["chain_num"], cp["chain_den"]
            out["chain"] = {"num_ms_per_step": round(nms / a.steps, 3),
                            "den_ms_per_step": round(dms / a.steps, 3),
                            # the den streams its arc tables from L2 (~1 MB, resident): L2 bytes
                            "den_L2_GBps": round(dbytes / (dms * 1e-3) / 1e9, 1) if dms else None,
                            "den_L2_frac": round(dbytes / (dms * 1e-3) / PEAK_L2_BPS, 4) if dms else None,
                            "ok_seqs": int(head["stats"][4])}
        if "roofline" in d:
            rl = d["roofline"]
            # the committed PMC summary is of the default configuration
            rl["traffic"] = (pmc_traffic(rl["kernel"]) if (a.xconfig == "cnn_tdnn_17f.xconfig" and not a.fp8
                                                           and a.mode == "train") else None)
            out["roofline"] = rl
        if world == 1 and not a.no_cpu_baseline and not fwd_only:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle
            from kfp16 import synth
            xcfg, params, bns, den_g, P = ctx
            den = (den_g, oracle.den_initial_probs(den_g))
            try:
                out["cpu_baseline"] = cpu_baseline(xcfg, params, bns, a.cpu_frames, threads,
                                                   den, synth.make_num_fst(0, num_pdfs=P), a.gt_frames)
            except Exception as e:  # noqa: BLE001 -- recorded; the headline still prints
                errors["cpu_baseline"] = {"error": f"{type(e).__name__}: {e}"}
        one = extra.get("train_1536_one_stream", {}).get("roofline")
        if one is not None:
            # the dominant class priced without the weight gradients co-running
            out["roofline_one_stream"] = {k: one[k] for k in ("bound", "achieved", "peak", "unit", "frac", "kernel",
                                                              "launches", "kernel_ms_per_step", "mfma_frac",
                                                              "hbm_frac", "flops_per_launch",
                                                              "alg_bytes_per_launch")}
        if extra:
            out["sub_results"] = extra
        out["sub_result_errors"] = errors or None
        pend = kfp16.pending_log()
        if pend:   # HIP errors other calls left pending, consumed by the library's entry checks
            out["hip_pending_log"] = pend
        print(json.dumps(out), flush=True)
    if comm is not None:
        torch.cuda.synchronize()
        comm.close()
    if world > 1:
        dist.destroy_process_group()
    if errors and a.strict:
        return 3
    return 0


if __name__ == "__main__":
    sys.exit(main())
