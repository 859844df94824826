"""Test infrastructure: writes a network's parameters as `nnet3-copy --binary=false`
text, with the component names and matrix orientation (Kaldi [out x in]) the
reference's loader expects (internal/nnet/weight_loader.go:65-437)."""
import numpy as np

import nnet3_text as T


def default_idct(dim, lifter=22.0):
    """The build's idct-layer matrix (makeIDCTMatrix, forward.go:1190-1210; network.cpp
    idct_matrix), y = x . M orientation, float32."""
    i = np.arange(dim)[:, None].astype(np.float64)
    j = np.arange(dim)[None, :].astype(np.float64)
    v = np.cos(np.pi * j * (i + 0.5) / dim)
    v = v * np.where(j == 0, np.sqrt(1.0 / dim), np.sqrt(2.0 / dim))
    if lifter > 0:
        v = v * np.where(j > 0, 1.0 + (lifter / 2.0) * np.sin(np.pi * j / lifter), 1.0)
    return v.astype(np.float32)


def network_text(layers, params, bns, idct=None, drop_bias=(), rms=1.0, eps=1e-3):
    """layers: kfp16.Network.layers; params: name -> [in x out] arrays; bns: (layer, which)
    -> (mean, var, gamma, beta) (gamma = 1, beta = 0 expected); idct: optional [D x D]
    matrix in the y = x . M orientation."""
    out = []
    tr = lambda a: np.asarray(a, np.float32).T
    bias = lambda k: None if k in drop_bias else np.asarray(params[k], np.float32).reshape(-1)
    for name, ty, din, dout in layers:
        if ty == 1:  # the reference requires an idct component (weight_loader.go:760-764)
            m = default_idct(din) if idct is None else idct
            out.append(T.write_component("idct", "FixedAffineComponent", tr(m), np.zeros(din)))
        elif ty == 2:
            out.append(T.write_component(name, "LinearComponent", tr(params[name + ".W"])).replace(
                "<LinearParams>", "<Params>"))
        elif ty == 3:
            m, v, _, _ = bns[(name, 0)]
            out.append(T.write_component(name, "BatchNormComponent", mean=m, var=v, bn_dim=len(m), eps=eps, rms=rms))
        elif ty == 6:
            out.append(T.write_component(name + ".conv", "TimeHeightConvolutionComponent", tr(params[name + ".W"]),
                                         bias(name + ".Bias")))
            out.append(f"<ComponentName> {name}.relu <RectifiedLinearComponent> <Dim> {dout} <ValueAvg>  [ ]\n")
            m, v, _, _ = bns[(name, 0)]
            out.append(T.write_component(name + ".batchnorm", "BatchNormComponent", mean=m, var=v, bn_dim=len(m),
                                         eps=eps, rms=rms))
        elif ty == 7:
            out.append(T.write_component(name + ".linear", "TdnnComponent", tr(params[name + ".LinearW"]),
                                         header="<MaxChange> 0.75 <TimeOffsets> [ 0 ]\n"))
            out.append(T.write_component(name + ".affine", "TdnnComponent", tr(params[name + ".AffineW"]),
                                         bias(name + ".AffineBias")))
            m, v, _, _ = bns[(name, 0)]
            out.append(T.write_component(name + ".batchnorm", "BatchNormComponent", mean=m, var=v, bn_dim=len(m),
                                         eps=eps, rms=rms))
        elif ty == 9:
            pre = "prefinal-xent" if "xent" in name else "prefinal-chain"
            out.append(T.write_component(pre + ".affine", "NaturalGradientAffineComponent", tr(params[name + ".BigW"]),
                                         bias(name + ".BigBias")))
            for which, tag in ((0, "batchnorm1"), (1, "batchnorm2")):
                m, v, _, _ = bns[(name, which)]
                out.append(T.write_component(f"{pre}.{tag}", "BatchNormComponent", mean=m, var=v, bn_dim=len(m),
                                             eps=eps, rms=rms))
            out.append(T.write_component(pre + ".linear", "LinearComponent", tr(params[name + ".SmallW"])))
        elif ty == 10:
            out.append(T.write_component(name + ".affine", "NaturalGradientAffineComponent", tr(params[name + ".W"]),
                                         bias(name + ".Bias")))
    return "".join(out)
