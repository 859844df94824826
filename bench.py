#!/usr/bin/env python3
"""bench.py — frames/sec of the CNN-TDNN fwd+bwd training step on MI355X.

Metric (BASELINE.json): frames/sec CNN-TDNN fwd+bwd, 40-dim x 1500-frame egs,
1/2/4/8 MI355X. One step = TrainStep (train_step.go:142-283): forward, chain
LF-MMI objective + derivative (numerator and leaky-HMM denominator per eg,
backward.go:224-371), backward, gradient all-reduce (N > 1) and SGD, over one
minibatch of 64 synthetic egs (96,000 frames) per GPU, on the pinned synthetic
17-TDNN-F model (configs/cnn_tdnn_17f.xconfig) with the synthetic den graph and
numerator FSTs of SURVEY §8d. Inputs are resident in HBM before the timed region.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one process per GPU, RCCL all-reduce of the flat fp32
gradient). Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

# torch first: kfp16's libraries then bind to the same HIP runtime (kfp16.hip_runtimes)
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kaldi-fp16_amd", "python"))

import numpy as np  # noqa: E402

METRIC = "frames/sec CNN-TDNN fwd+bwd, 40-dim×1500-frame egs, 1/2/4/8 MI355X"
METRIC_FWD = "frames/sec CNN-TDNN forward only, 40-dim×1500-frame egs, 1 MI355X"
PEAK_FP16_TFLOPS = 2500.0   # MI355X dense FP16 MFMA (MI355X_MICROARCH.md)
PEAK_FP8_TFLOPS = 5000.0    # MI355X dense FP8 (MX-scaled K=128 MFMA)
FRAMES_PER_EG = 1500


def parse():
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
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-frames", type=int, default=1500)
    p.add_argument("--cpu-threads", type=int, default=16)
    p.add_argument("--no-prof", action="store_true")
    p.add_argument("--fp8", action="store_true",
                   help="MXFP8 forward GEMMs (configs[4]; use with --xconfig cnn_tdnn_17f_3072.xconfig)")
    p.add_argument("--mode", choices=("train", "forward"), default="train",
                   help="train: the metric's fwd+bwd+SGD step; forward: configs[1], forward only")
    return p.parse_args()


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


def cpu_baseline(xcfg, params, bns, frames, threads, den, num_fst):
    """The C oracle (a port of the reference's CNN-TDNN math and chain objective)
    timed on host cores: forward, objective on the subsampled frames, backward."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from kfp16 import synth
    try:
        oracle.build(native=True)
        oracle.lib(native=True)
    except Exception:
        oracle.lib()
    tp = {k: synth.trunc_fp16(v) for k, v in params.items()}
    on = oracle.OracleNet(xcfg, tp, bns, round_mode=oracle.ROUND_FUSED, threads=threads)
    feats = synth.make_features(frames, 40).astype(np.float32)
    g, init = den
    row0, nfr, stride = synth.chain_layout(1, frames)
    rows = row0[0] + np.arange(nfr[0]) * stride
    D = ivector_input(xcfg)
    iv = (np.random.default_rng(5).standard_normal((1, D)) * 2).astype(np.float32) if D else None
    t0 = time.perf_counter()
    if D:
        on.forward(feats, ivectors=iv, seq_off=np.array([0, frames], np.int32))
    else:
        on.forward(feats)
    out = on.act("output")
    deriv, _ = oracle.chain_objf(g, init, num_fst, out[rows])
    og = np.zeros_like(out)
    og[rows] = (-deriv).astype(np.float16).astype(np.float32)
    on.backward(og)
    dt = time.perf_counter() - t0
    on.close()
    name = "cnn_tdnn_17f with the ivector front end" if D else "cnn_tdnn_17f"
    return {"value": round(frames / dt, 2), "unit": "frames/sec", "cores": threads, "kind": "port",
            "sample": f"C oracle train step (fwd, chain objective, bwd) of {name} on {frames} "
                      f"frames (1 eg), fp32 math, {threads} threads for the GEMMs, {dt:.1f} s"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)

    import kfp16
    from kfp16 import dp, synth
    kfp16.check(kfp16.core.bridge_gpu_init(local), "bridge_gpu_init")
    stream = torch.cuda.current_stream()
    kfp16.set_stream(stream.cuda_stream)
    kfp16.assert_single_hip_runtime()

    T = a.egs * FRAMES_PER_EG
    xcfg = synth.load_xconfig(a.xconfig)
    net = kfp16.Network(xcfg, max_frames=T)
    params, bns = synth.init_network(net, seed=42)        # identical replicas on every rank
    if a.fp8:
        net.set_fp8(True)
    grad = torch.zeros(net.num_params, dtype=torch.float32, device="cuda")
    net.bind_grad_buffer(grad.data_ptr())

    feats = synth.make_features(T, 40, seed=1234 + rank)   # this rank's shard of egs
    fbuf = torch.from_numpy(feats.view(np.int16)).to("cuda")
    P = net.layers[-1][3]
    # chain supervision: shared den graph, one numerator FST per eg
    # (seed 7 + global eg index); the objective writes the output gradient on the
    # subsampled rows (leftCtx 30, stride 3) — every other row stays zero
    from kfp16 import chain
    den_g = synth.make_den_graph(num_pdfs=P)
    dgraph = chain.DenGraph(den_g)
    fsts = [synth.make_num_fst(dp.eg_index(rank, a.egs, e), num_pdfs=P) for e in range(a.egs)]
    nbatch = chain.NumBatch(fsts)
    row0, nfr, stride = synth.chain_layout(a.egs, FRAMES_PER_EG)
    objective = chain.Chain(dgraph, max_seqs=a.egs, max_frames=int(nfr.max()))
    out_ptr = net.activation("output")[0]
    gbuf = torch.zeros((T, P), dtype=torch.float16, device="cuda")
    torch.cuda.synchronize()

    # Kaldi's ivector front end: one ivector per eg, one sequence per eg
    ivd = ivector_input(xcfg)
    if ivd:
        ivecs = (np.random.default_rng(99 + rank).standard_normal((a.egs, ivd)) * 2).astype(np.float16)
        ibuf = torch.from_numpy(ivecs.view(np.int16)).to("cuda")
        seq_off = np.arange(a.egs + 1, dtype=np.int32) * FRAMES_PER_EG

    def step():
        if ivd:
            net.forward_ivector(fbuf.data_ptr(), T, ibuf.data_ptr(), seq_off)
        else:
            net.forward(fbuf.data_ptr(), T)
        if a.mode == "forward":
            return
        objective.compute(nbatch, out_ptr, P, T, row0, nfr, stride, gbuf.data_ptr(), P)
        net.backward(gbuf.data_ptr())
        dp.allreduce_mean_(grad, world)   # the one data-path collective (RCCL)
        net.sgd(a.lr, a.momentum)

    for _ in range(a.warmup):
        step()
        if os.environ.get("KF_BENCH_CHECK"):
            r = objective.result()
            print("warmup objf/frame", r.objf / max(r.frames, 1), "ok", r.num_ok, flush=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    if not a.no_prof:
        kfp16.core.kf_prof_reset()
        kfp16.core.kf_prof_enable(1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kfp16.core.kf_prof_enable(0)
    elapsed = dp.max_over_ranks(elapsed, "cuda")

    prof, chain_prof = {}, {}
    if not a.no_prof:
        for cls, name in ((0, "gemm_fused"), (1, "gemm_wgrad")):
            n, ms, fl = kfp16.prof_collect(cls)
            prof[name] = (n, ms, fl)
        for cls, name in ((2, "chain_num"), (3, "chain_den")):
            chain_prof[name] = kfp16.prof_collect(cls)
        kfp16.core.kf_prof_reset()
    stats = [0.0] * 5
    if a.mode == "train":
        res = objective.result()
        stats = dp.sum_over_ranks([res.objf, res.num_logprob, res.den_logprob, res.frames, res.num_ok],
                                  "cuda")

    if rank == 0:
        ms_step = elapsed / a.steps * 1e3
        frames = T * world * a.steps
        value = frames / elapsed
        fwd_only = a.mode == "forward"
        workload = ("cnn_tdnn_17f forward only (configs[1])" if fwd_only else
                    "cnn_tdnn_17f train step (fwd+bwd+SGD)") + f", {a.egs} egs x 1500 frames per GPU"
        if ivd:
            workload += f", Kaldi ivector front end ({ivd}-dim ivector per eg)"
        out = {
            "metric": METRIC_FWD if fwd_only else METRIC, "value": round(value, 1), "unit": "frames/sec", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "mxfp8 GEMMs (e4m3 + E8M0), fp16 storage" if a.fp8 else "fp16",
            "data": "synthetic",
            "config": {"workload": workload,
                       "xconfig": a.xconfig, "egs_per_gpu": a.egs, "frames_per_eg": FRAMES_PER_EG,
                       "global_batch_egs": a.egs * world, "parallelism": f"dp{world}",
                       "objective": "chain LF-MMI (den S=7052 A=113380, num 250 states/eg, fps 490)"},
        }
        if not fwd_only:
            out["objf_per_frame"] = round(float(stats[0]) / max(float(stats[3]), 1.0), 5)
            out["objective_finite_seqs"] = f"{int(stats[4])}/{a.egs * world}"
        if chain_prof and not fwd_only:
            (nn, nms, _), (dn, dms, dbytes) = chain_prof["chain_num"], chain_prof["chain_den"]
            out["chain"] = {"num_ms_per_step": round(nms / a.steps, 3),
                            "den_ms_per_step": round(dms / a.steps, 3),
                            "den_algorithmic_GBps": round(dbytes / (dms * 1e-3) / 1e9, 1) if dms else None,
                            "ok_seqs": int(stats[4])}
        if prof:
            dom = max(prof, key=lambda k: prof[k][1])
            n, ms, fl = prof[dom]
            ach = fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
            peak = PEAK_FP8_TFLOPS if a.fp8 else PEAK_FP16_TFLOPS
            out["roofline"] = {"bound": "mfma", "achieved": round(ach, 2), "peak": peak,
                               "unit": "TFLOP/s", "frac": round(ach / peak, 4),
                               # the committed PMC summary is of the default configuration
                               "traffic": pmc_traffic(dom) if (a.xconfig == "cnn_tdnn_17f.xconfig" and
                                                              not a.fp8 and a.mode == "train") else None,
                               "kernel": dom, "launches": n, "kernel_ms_per_step": round(ms / a.steps, 3),
                               "all_gemm_tflops": round(sum(v[2] for v in prof.values()) /
                                                        (sum(v[1] for v in prof.values()) * 1e-3) / 1e12, 2)}
        if world == 1 and not a.no_cpu_baseline and not fwd_only:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle
            den = (den_g, oracle.den_initial_probs(den_g))
            out["cpu_baseline"] = cpu_baseline(xcfg, params, bns, a.cpu_frames, a.cpu_threads,
                                               den, synth.make_num_fst(0, num_pdfs=P))
        print(json.dumps(out), flush=True)
    objective.close()
    net.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
