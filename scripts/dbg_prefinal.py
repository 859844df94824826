import sys, os
sys.path[:0] = ['kaldi-fp16_amd/python', 'oracle', 'tests']
import numpy as np, kfp16
from kfp16 import synth
kfp16.check(kfp16.core.bridge_gpu_init(0))
xcfg = synth.load_xconfig("tiny.xconfig")
T = 150
net = kfp16.Network(xcfg, T)
params, bns = synth.init_network(net)
feats = synth.make_features(T, 40)
fb = kfp16.upload_fp16(feats)
net.forward(fb.ptr, T)
og = (np.random.default_rng(7).standard_normal((T, 200)) * 0.05).astype(np.float16)
gb = kfp16.upload_fp16(og)
li = [l[0] for l in net.layers].index("prefinal-chain")
kfp16.check(kfp16.nnet.nnet_backward_n(net.h, gb.ptr, 2))
rd = lambda p, shp: kfp16.read_fp16(p, shp).astype(np.float64)
dsmall = rd(kfp16.nnet.nnet_debug_tensor(net.h, b"dz0", 0), (T, 64))
dzbig = rd(kfp16.nnet.nnet_debug_tensor(net.h, b"dbott", 0), (T, 256))
big = rd(kfp16.nnet.nnet_debug_tensor(net.h, b"aux", li), (T, 256))
maskb = kfp16.read_fp16(kfp16.nnet.nnet_debug_tensor(net.h, b"mask", li), (T * 256 // 16,)).view(np.uint8)
mask = np.unpackbits(maskb, bitorder="little")[:T * 256].reshape(T, 256)
sc = kfp16.read_f32(kfp16.nnet.nnet_debug_tensor(net.h, b"bn_scale", li), (256,))
sc2 = kfp16.read_f32(kfp16.nnet.nnet_debug_tensor(net.h, b"bn2_scale", li), (64,))
tp = {k: synth.trunc_fp16(v).astype(np.float64) for k, v in params.items()}
x = net.read_activation("prefinal-l").astype(np.float64)
# recompute from product tensors
zbig = x @ tp["prefinal-chain.BigW"] + tp["prefinal-chain.BigBias"]
print("mask agree", np.mean(mask == (zbig > 0)))
m, v, g, b = bns[("prefinal-chain", 0)]
print("scale agree", np.max(np.abs(sc - g / np.sqrt(v + 1e-3))))
m2, v2, g2, b2 = bns[("prefinal-chain", 1)]
print("scale2 agree", np.max(np.abs(sc2 - g2 / np.sqrt(v2 + 1e-3))))
ds_ref = (og.astype(np.float64) @ tp["output.W"].T) * sc2
print("dsmall err", np.linalg.norm(dsmall - ds_ref) / np.linalg.norm(ds_ref))
dzb_ref = (dsmall @ tp["prefinal-chain.SmallW"].T) * sc * mask
print("dzbig err", np.linalg.norm(dzbig - dzb_ref) / np.linalg.norm(dzb_ref))
dzb_ref2 = (dsmall @ tp["prefinal-chain.SmallW"].T) * sc * (zbig > 0)
print("dzbig err (recomputed mask)", np.linalg.norm(dzbig - dzb_ref2) / np.linalg.norm(dzb_ref2))
g = net.read_grads()
print("BigW err", np.linalg.norm(g["prefinal-chain.BigW"] - x.T @ dzbig) / np.linalg.norm(x.T @ dzbig))
print("SmallW err", np.linalg.norm(g["prefinal-chain.SmallW"] - big.T @ dsmall) / np.linalg.norm(big.T @ dsmall))
import oracle
on = oracle.OracleNet(xcfg, {k: synth.trunc_fp16(v) for k, v in params.items()}, bns, round_mode=oracle.ROUND_FUSED)
on.forward(feats.astype(np.float32))
on.backward(og.astype(np.float32))
oli = on.index["prefinal-chain"]
obig = np.ctypeslib.as_array(on.net.aux[oli], shape=(T * 256,)).reshape(T, 256).astype(np.float64)
omask = np.ctypeslib.as_array(on.net.mask[oli], shape=(T * 256,)).reshape(T, 256)
ox = on.act("prefinal-l").astype(np.float64)
print("x vs oracle", np.linalg.norm(x - ox) / np.linalg.norm(ox))
print("big vs oracle", np.linalg.norm(big - obig) / np.linalg.norm(obig))
print("mask agree vs oracle", np.mean(mask == omask))
og_ = on.grads()
print("oracle BigW vs x^T dzbig(product)", np.linalg.norm(og_["prefinal-chain.BigW"] - x.T @ dzbig) / np.linalg.norm(x.T @ dzbig))
print("oracle SmallW vs product", np.linalg.norm(og_["prefinal-chain.SmallW"] - g["prefinal-chain.SmallW"]) / np.linalg.norm(og_["prefinal-chain.SmallW"]))
print("oracle BigBias vs colsum", np.linalg.norm(og_["prefinal-chain.BigBias"].ravel() - dzbig.sum(0)) / np.linalg.norm(dzbig.sum(0)))
for k in ("prefinal-l.W", "output.W"):
    print(k, np.linalg.norm(og_[k] - g[k]) / np.linalg.norm(og_[k]))
m1, v1, g1, b1 = bns[("prefinal-chain", 0)]
sc1 = g1 / np.sqrt(v1 + 1e-3)
ds_o = ((og.astype(np.float64) @ tp["output.W"].T) * sc2).astype(np.float16).astype(np.float64)
print("ds numpy vs product dsmall", np.linalg.norm(ds_o - dsmall) / np.linalg.norm(dsmall))
dzb_o = ((ds_o @ tp["prefinal-chain.SmallW"].T) * sc1 * omask).astype(np.float16).astype(np.float64)
print("dzb numpy(oracle mask) vs product", np.linalg.norm(dzb_o - dzbig) / np.linalg.norm(dzbig))
print("oracle BigW vs ox^T dzb_o", np.linalg.norm(og_["prefinal-chain.BigW"] - ox.T @ dzb_o) / np.linalg.norm(ox.T @ dzb_o))
print("sc1 vs product sc", np.max(np.abs(sc1 - sc)))
print("tp SmallW dtype", tp["prefinal-chain.SmallW"].dtype, params["prefinal-chain.SmallW"][:1,:4])
