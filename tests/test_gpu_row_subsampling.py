"""Row-subsampled train step (kf_nnet.h nnet_set_row_subsampling) against the full-row
computation of the same network on the same egs.

TrainStep (train_step.go:142-283) reads the network output only through the chain
objective, on rows row0 + 3k (frame subsampling 3, every eg's first supervised row at 0 mod
3), and every other output row gets a zero gradient. The layers above the conv stack then
need only the rows 0 (mod 3) and a tail of rows T-1, T-4, ... (the splices' clamp at T-1);
nnet_set_row_subsampling(3) runs them on that set. Checked here, on the benchmark model at
2 egs (T = 3000, T-1 = 2 mod 3: with a tail) and at T = 2998 (T-1 = 0 mod 3: no tail):

- every output row of the set, rows 0 (mod 3), bit-identical to the full forward;
- the conv stack's activations and every conv weight / bias gradient bit-identical (the
  gradient into the conv stack is scattered to the same values); cnn6 evaluated on the
  compact rows only (time-strided conv operand) gives those rows bit-identically;
- the TDNN-F / prefinal / output weight gradients (and cnn6's when it runs on the compact
  rows) within 1e-5 (relative Frobenius) of the full computation: the same products, summed
  in another split-K order (fewer rows);
- the objective's inputs: the supervised output rows equal, so the objective is equal.
"""
import numpy as np
import pytest
import torch

from conftest import rel_fro

pytestmark = pytest.mark.gpu


def _run(kfp16, xcfg, T, sub, seed_grad=3, two_stream=True, conv_rows=True, ivec=0):
    import os
    from kfp16 import synth
    net = kfp16.Network(xcfg, max_frames=T)
    synth.init_network(net, seed=42)
    net.set_wgrad_stream(two_stream)
    if sub:
        os.environ["KF_RSUB_CONV"] = "1" if conv_rows else "0"
        try:
            net.set_row_subsampling(3)
        finally:
            os.environ.pop("KF_RSUB_CONV", None)
    fb = kfp16.upload_fp16(synth.make_features(T, 40))
    if ivec:   # Kaldi's ivector front end: one ivector per 1500-frame eg
        B = (T + 1499) // 1500
        iv = kfp16.upload_fp16((np.random.default_rng(5).standard_normal((B, ivec)) * 2).astype(np.float16))
        seq = np.minimum(np.arange(B + 1) * 1500, T).astype(np.int32)
        net.forward_ivector(fb.ptr, T, iv.ptr, seq)
    else:
        net.forward(fb.ptr, T)
    P = net.layers[-1][3]
    # output gradient on the supervised rows only (2 egs' chain layout: row0 = 1500 e + 30)
    g = np.zeros((T, P), np.float16)
    rng = np.random.default_rng(seed_grad)
    sup = []
    for e in range((T + 1499) // 1500):
        r0 = 1500 * e + 30
        sup += [r for r in range(r0, min(T, 1500 * e + 1500), 3)]
    sup = np.array(sup)
    g[sup] = (rng.standard_normal((len(sup), P)) * 0.05).astype(np.float16)
    tc, tc0, rows = net.row_set()
    if sub:
        assert tc > 0, "the row set was not used"
        assert np.all(rows[:tc0] == 3 * np.arange(tc0))
        gc = g[rows]
        gb = kfp16.upload_fp16(gc)
    else:
        assert tc == 0
        gb = kfp16.upload_fp16(g)
    out = net.read_activation("output").astype(np.float32)
    names = ["cnn6", "tdnnf7", "tdnnf23", "prefinal-chain"] + [n for n, *_ in net.layers if n == "output-xent"]
    acts = {n: net.read_activation(n) for n in names}
    net.backward(gb.ptr)
    torch.cuda.synchronize()
    grads = net.read_grads()
    res = dict(out=out, acts=acts, grads=grads, rows=rows, tc=tc, tc0=tc0, sup=sup)
    net.close()
    return res


@pytest.mark.parametrize("T,conv_rows,model", [(3000, True, "plain"), (2998, True, "plain"), (3000, False, "plain"),
                                               (3000, True, "ivec"), (3000, True, "kaldi")])
def test_row_subsampled_step_matches_full(gpu, T, conv_rows, model):
    """conv_rows: cnn6 (the conv below the compact layers) computes only the compact rows
    (time-strided halo operand, two launches: rows 0 (mod 3) and the tail); else it runs on
    all rows and tdnnf7 reads its output gathered. model ivec: Kaldi's ivector front end
    (cnn_tdnn_17f_ivec, nnet_forward_ivector) under the same TDNN-F stack; kaldi: the recipe
    topology (ivector front end and the xent branch on prefinal-l, also on the row set)"""
    kfp16 = gpu
    from kfp16 import synth
    xcfg = synth.load_xconfig({"ivec": "cnn_tdnn_17f_ivec.xconfig", "kaldi": "cnn_tdnn_17f_kaldi.xconfig"}
                              .get(model, "cnn_tdnn_17f.xconfig"))
    ivec = 100 if model in ("ivec", "kaldi") else 0
    full = _run(kfp16, xcfg, T, False, ivec=ivec)
    sub = _run(kfp16, xcfg, T, True, conv_rows=conv_rows, ivec=ivec)
    tc, tc0, rows = sub["tc"], sub["tc0"], sub["rows"]
    assert tc0 == (T - 1) // 3 + 1
    assert (tc > tc0) == ((T - 1) % 3 != 0)
    # outputs of the set's rows 0 (mod 3): bit-identical
    assert np.array_equal(sub["out"][:tc0].view(np.uint32), full["out"][rows[:tc0]].view(np.uint32))
    # the supervised rows, through which the objective reads the network
    c_sup = sub["sup"] // 3
    assert np.array_equal(sub["out"][c_sup], full["out"][full["sup"]])
    # the conv stack: cnn6 on the compact rows (or all rows), the same sums in the same order
    if conv_rows:
        assert sub["acts"]["cnn6"].shape[0] == tc
        assert np.array_equal(sub["acts"]["cnn6"].view(np.uint16), full["acts"]["cnn6"][rows].view(np.uint16))
    else:
        assert np.array_equal(sub["acts"]["cnn6"], full["acts"]["cnn6"])
    for name in [n for n in full["acts"] if n != "cnn6"]:
        assert np.array_equal(sub["acts"][name][:tc0].view(np.uint16), full["acts"][name][rows[:tc0]].view(np.uint16)), name
    for k, v in full["grads"].items():
        w = sub["grads"][k]
        if k.startswith(("cnn", "idct", "ivector")) and not (conv_rows and k.startswith("cnn6")):
            assert np.array_equal(w, v), k
        else:
            assert rel_fro(w, v) <= 1e-5, (k, rel_fro(w, v))


def test_row_subsampling_off_and_limits(gpu):
    """stride 0 switches it off (full rows); other strides and unsupported topologies fail
    loudly; a forward too short for the tail runs on full rows"""
    kfp16 = gpu
    from kfp16 import synth
    net = kfp16.Network(synth.load_xconfig("cnn_tdnn_17f.xconfig"), max_frames=3000)
    synth.init_network(net, seed=1)
    with pytest.raises(kfp16.KfError):
        net.set_row_subsampling(2)
    net.set_row_subsampling(3)
    fb = kfp16.upload_fp16(synth.make_features(3000, 40))
    net.forward(fb.ptr, 60)           # 20 compact rows: too short for the 20-row tail
    assert net.row_set()[0] == 0
    net.forward(fb.ptr, 3000)
    assert net.row_set()[0] > 0
    net.set_row_subsampling(0)
    net.forward(fb.ptr, 3000)
    assert net.row_set()[0] == 0
    net.close()
    tiny = kfp16.Network(synth.load_xconfig("tiny_att.xconfig"), max_frames=300)
    with pytest.raises(kfp16.KfError):
        tiny.set_row_subsampling(3)
    tiny.close()
