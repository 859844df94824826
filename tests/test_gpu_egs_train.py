"""TrainStep on real-format egs (kfp16.trainer over kfp16.egs): a binary ark ->
DataLoader -> compressed upload + GPU expansion -> forward -> batched chain objective
on the batch's own numerator CSRs -> backward -> SGD (train_step.go:142-283).

Parity: the egs path must give the same objective, bit for bit, as the established
path fed with the host-decompressed features and the same FSTs (the pieces of which
are checked against the oracle elsewhere); and gradient steps must improve the
objective on a fixed batch."""
import numpy as np
import pytest

import egs_writer as W

pytestmark = pytest.mark.gpu


def _setup(kf, tmp_path, n=6):
    from kfp16 import egs, synth, trainer
    rng = np.random.default_rng(31)
    # numerator FSTs shorter than the shortest eg (23 supervised frames): always reachable
    exs, meta = W.make_egs(rng, n, rows=(150, 183, 129), num_pdfs=200, fst_states=(8, 20))
    W.write_ark(tmp_path / "cegs.1.ark", exs)
    batch = egs.DataLoader(str(tmp_path / "cegs.*.ark"), batch_size=n).next_batch()
    den = synth.make_den_graph(num_states=300, num_arcs=3000, num_pdfs=200)
    return batch, den, trainer


def test_egs_train_step_matches_direct_path(gpu, tmp_path):
    kf = gpu
    from kfp16 import chain, synth
    batch, den, trainer = _setup(kf, tmp_path)
    xcfg = synth.load_xconfig("tiny.xconfig")
    cfg = trainer.TrainConfig(learning_rate=0.0, momentum=0.0)
    tr = trainer.EgsTrainer(xcfg, den, max_egs=8, max_frames=1200, config=cfg)
    synth.init_network(tr.net)
    tr.step(batch)
    r1 = tr.result()
    assert r1.num_ok == batch.batch_size and np.isfinite(r1.objf) and abs(r1.objf / r1.frames) < 50
    # the same step through the established path: host features, pack_num_fsts
    net = kf.Network(xcfg, max_frames=1200)
    synth.init_network(net)
    T = batch.total_frames
    fbuf = kf.upload_fp16(batch.features_host().astype(np.float16))
    net.forward(fbuf.ptr, T)
    obj = chain.Chain(chain.DenGraph(den), max_seqs=8, max_frames=401)
    row0, frames = trainer.chain_rows(batch.frame_offsets, batch.num_frames, batch.frames_per_seq, 3, 30)
    g = kf.DeviceBuffer(T * 200 * 2)
    kf.core.bridge_gpu_memset(g.ptr, 0, T * 200 * 2)
    obj.compute(chain.NumBatch(batch.num_fsts()), net.activation("output")[0], 200, T, row0, frames, 3, g.ptr, 200)
    r2 = obj.result()
    assert (r1.objf, r1.num_logprob, r1.den_logprob, r1.frames) == (r2.objf, r2.num_logprob, r2.den_logprob, r2.frames)
    np.testing.assert_array_equal(kf.read_fp16(tr.grad_out.ptr, (T, 200)), kf.read_fp16(g.ptr, (T, 200)))


def test_egs_training_improves_objective(gpu, tmp_path):
    kf = gpu
    from kfp16 import synth
    batch, den, trainer = _setup(kf, tmp_path)
    cfg = trainer.TrainConfig(learning_rate=2e-4, momentum=0.0)
    tr = trainer.EgsTrainer(synth.load_xconfig("tiny.xconfig"), den, max_egs=8, max_frames=1200, config=cfg)
    synth.init_network(tr.net)
    objs = []
    for _ in range(4):
        tr.step(batch)
        r = tr.result()
        objs.append(r.objf / r.frames)
    assert all(np.isfinite(objs)), objs
    assert objs[-1] > objs[0], objs


def test_egs_training_with_ivectors(gpu, tmp_path):
    """Kaldi's ivector front end fed from the egs' own ivectors (one per eg): the step's
    objective equals the direct path fed with the host-decompressed features and
    ivectors, and training improves it."""
    kf = gpu
    from kfp16 import chain, synth
    batch, den, trainer = _setup(kf, tmp_path)
    assert batch.ivector_dim == 100
    xcfg = synth.load_xconfig("tiny_ivec.xconfig")
    tr = trainer.EgsTrainer(xcfg, den, max_egs=8, max_frames=1200,
                            config=trainer.TrainConfig(learning_rate=0.0, momentum=0.0))
    synth.init_network(tr.net)
    tr.step(batch)
    r1 = tr.result()
    assert r1.num_ok == batch.batch_size and np.isfinite(r1.objf)
    net = kf.Network(xcfg, max_frames=1200)
    synth.init_network(net)
    T = batch.total_frames
    fbuf = kf.upload_fp16(batch.features_host().astype(np.float16))
    ibuf = kf.upload_fp16(batch.ivectors_host().astype(np.float16))
    net.forward_ivector(fbuf.ptr, T, ibuf.ptr, np.append(np.asarray(batch.frame_offsets, np.int32), T))
    obj = chain.Chain(chain.DenGraph(den), max_seqs=8, max_frames=401)
    row0, frames = trainer.chain_rows(batch.frame_offsets, batch.num_frames, batch.frames_per_seq, 3, 30)
    g = kf.DeviceBuffer(T * 200 * 2)
    kf.core.bridge_gpu_memset(g.ptr, 0, T * 200 * 2)
    obj.compute(chain.NumBatch(batch.num_fsts()), net.activation("output")[0], 200, T, row0, frames, 3, g.ptr, 200)
    r2 = obj.result()
    assert (r1.objf, r1.den_logprob) == (r2.objf, r2.den_logprob)
    tr2 = trainer.EgsTrainer(xcfg, den, max_egs=8, max_frames=1200,
                             config=trainer.TrainConfig(learning_rate=2e-4, momentum=0.0))
    synth.init_network(tr2.net)
    objs = []
    for _ in range(4):
        tr2.step(batch)
        r = tr2.result()
        objs.append(r.objf / r.frames)
    assert all(np.isfinite(objs)) and objs[-1] > objs[0], objs
