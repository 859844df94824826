"""kfp16.trainer — the chain training step driven by real egs minibatches.

Restates nnet.TrainStep (internal/nnet/train_step.go:142-283) over the build's pieces:
  1. TransferBatch + Forward      -> TrainingBatch.features_to_device (compressed upload,
                                     GPU expansion to fp16) + Network.forward
  2. ComputeChainLossBatch        -> one batched kf_chain_compute; the rows of each eg are
     (chain_loss.go:221-294)         frame_offset + left_context + k * subsampling for
                                     k < frames_per_seq, cut where the eg ends
  3. Backward                     -> Network.backward (seeded at the chain output)
  4. optimizer.Update per tensor  -> Network.sgd over the flat buffer (optimize.go:95-142)
plus, for data parallel, the flat-gradient all-reduce between 3 and 4 (kfp16.dp).

The numerator FSTs come from the batch's per-sequence CSRs (TrainingBatch.PerSeqCSRs),
the denominator from a DenGraph the caller builds (NativeDenominator's transitions).
Everything runs on the GPU; this module only sequences the calls.

A network with Kaldi's ivector input (`input name=ivector`, ReplaceIndex(ivector, t, 0))
gets the batch's per-eg ivectors, expanded on the GPU next to the features, with one
sequence per eg (nnet_forward_ivector). The reference drops them at this point.
"""
from __future__ import annotations

import re
from dataclasses import dataclass

import numpy as np

from . import DeviceBuffer, Network, core, sync
from . import chain as _chain


@dataclass
class TrainConfig:
    """TrainConfig (train_step.go:20-30) fields the step uses."""
    learning_rate: float = 1e-4
    momentum: float = 0.9
    subsampling_factor: int = 3
    left_context: int = 30
    opts: _chain.KfChainOpts | None = None


def chain_rows(frame_offsets, num_frames, frames_per_seq, subsampling: int, left_context: int):
    """Per-eg (first output row, supervised frames) as ComputeChainLossBatch forms them
    (chain_loss.go:240-255): the eg's view is cut at left_context + fps * subsampling
    input rows, then every subsampling-th row from left_context is taken."""
    row0, frames = [], []
    for off, T, fps in zip(frame_offsets, num_frames, frames_per_seq):
        eff = min(left_context + int(fps) * subsampling, int(T))
        n = max(0, -(-(eff - left_context) // subsampling))  # ceil
        row0.append(int(off) + left_context)
        frames.append(min(int(fps), n))
    return np.asarray(row0, np.int32), np.asarray(frames, np.int32)


class EgsTrainer:
    """One network + objective, stepping on loader.TrainingBatch minibatches."""

    def __init__(self, xconfig: str, den_graph: dict, max_egs: int, max_frames: int,
                 config: TrainConfig | None = None, grad_buffer_ptr: int | None = None):
        self.cfg = config or TrainConfig()
        self.net = Network(xconfig, max_frames=max_frames)
        self.P = self.net.layers[[n for n, *_ in self.net.layers].index("output")][3] \
            if any(n == "output" for n, *_ in self.net.layers) else self.net.layers[-1][3]
        self.max_frames = max_frames
        self.feat = DeviceBuffer(max_frames * 40 * 2)
        self.grad_out = DeviceBuffer(max_frames * self.P * 2)
        self.dgraph = _chain.DenGraph(den_graph)
        self.objective = _chain.Chain(self.dgraph, max_seqs=max_egs,
                                      max_frames=max(1, max_frames // self.cfg.subsampling_factor + 1))
        if grad_buffer_ptr is not None:
            self.net.bind_grad_buffer(grad_buffer_ptr)
        self.out_ptr = self.net.activation("output")[0]
        m = re.search(r"^\s*input\s+name=ivector\s+dim=(\d+)", xconfig, re.M)
        self.ivec_dim = int(m.group(1)) if m else 0
        self.ivec = DeviceBuffer(max_egs * self.ivec_dim * 2) if self.ivec_dim else None
        self.max_egs = max_egs

    def step(self, batch, allreduce=None):
        """One TrainStep on `batch` (kfp16.egs.TrainingBatch). allreduce: optional callable
        run between backward and SGD (data parallel). Asynchronous on the library stream;
        call result() for the objective."""
        T = batch.total_frames
        if T > self.max_frames or batch.feat_dim != 40:
            raise ValueError(f"batch of {T} frames x {batch.feat_dim} does not fit the trainer")
        if self.ivec_dim:
            if batch.ivector_dim != self.ivec_dim or batch.batch_size > self.max_egs:
                raise ValueError(f"batch of {batch.batch_size} egs with {batch.ivector_dim}-dim ivectors does "
                                 f"not fit the trainer's {self.ivec_dim}-dim ivector input")
            batch.features_to_device(self.feat.ptr, 40, self.ivec.ptr)
        else:
            batch.features_to_device(self.feat.ptr, 40)
        # rows the objective does not write must be zero for this batch
        core.bridge_gpu_memset(self.grad_out.ptr, 0, T * self.P * 2)
        if self.ivec_dim:
            seq = np.append(np.asarray(batch.frame_offsets, np.int32), np.int32(T))
            self.net.forward_ivector(self.feat.ptr, T, self.ivec.ptr, seq)
        else:
            self.net.forward(self.feat.ptr, T)
        num = _chain.NumBatch(batch.num_fsts())
        row0, frames = chain_rows(batch.frame_offsets, batch.num_frames, batch.frames_per_seq,
                                  self.cfg.subsampling_factor, self.cfg.left_context)
        self.objective.compute(num, self.out_ptr, self.P, T, row0, frames, self.cfg.subsampling_factor,
                               self.grad_out.ptr, self.P, self.cfg.opts)
        self._num = num  # kept alive until the stream has consumed it
        self.net.backward(self.grad_out.ptr)
        if allreduce is not None:
            allreduce()
        self.net.sgd(self.cfg.learning_rate, self.cfg.momentum)

    def result(self):
        sync()
        return self.objective.result()
