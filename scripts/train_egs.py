"""Chain training from Kaldi egs on one MI355X (the reference's cmd/traintest loop:
DataLoader -> TrainStep -> log), through kfp16.egs / kfp16.trainer.

  python scripts/train_egs.py --egs 'exp/chain/egs/cegs.*.ark' --den-fst exp/chain/den.fst \
      --xconfig configs/cnn_tdnn_17f.xconfig --batch 64 [--model final.txt]

--model: optional nnet3 text (nnet3-copy --binary=false) to start from (NewNetworkFromKaldi);
otherwise the synthetic initialisation of kfp16.synth is used."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kaldi-fp16_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--egs", required=True)
    ap.add_argument("--den-fst", required=True)
    ap.add_argument("--xconfig", default=os.path.join(ROOT, "configs", "cnn_tdnn_17f.xconfig"))
    ap.add_argument("--model")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--lr", type=float, default=1e-5)
    ap.add_argument("--momentum", type=float, default=0.9)
    ap.add_argument("--left-context", type=int, default=30)
    ap.add_argument("--max-frames", type=int, default=64 * 1500)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--shuffle-seed", type=int, default=0)
    a = ap.parse_args()

    import torch  # noqa: F401  (one HIP runtime for torch and the libraries)
    import kfp16
    from kfp16 import chain, egs, model, synth, trainer
    kfp16.check(kfp16.core.bridge_gpu_init(0), "bridge_gpu_init")
    xcfg = open(a.xconfig).read()
    tr0 = kfp16.Network(xcfg, max_frames=16)
    P = [l for l in tr0.layers if l[0] == "output"][0][3]
    tr0.close()
    cfg = trainer.TrainConfig(learning_rate=a.lr, momentum=a.momentum, left_context=a.left_context)
    tr = trainer.EgsTrainer(xcfg, chain.den_graph_from_fst(a.den_fst, P), a.batch, a.max_frames, cfg)
    if a.model:
        st = model.Nnet3Model.from_file(a.model).load_into(tr.net, model.LOAD_NEW)
        print(f"loaded {a.model}: {st.layers_loaded} layers, {st.params} params", flush=True)
    else:
        synth.init_network(tr.net)
    dl = egs.DataLoader(a.egs, a.batch, shuffle=a.shuffle_seed != 0, seed=a.shuffle_seed, drop_last=True)
    for ep in range(a.epochs):
        t0, n, frames = time.perf_counter(), 0, 0
        for batch in dl:
            tr.step(batch)
            r = tr.result()
            n += 1
            frames += batch.total_frames
            print(f"epoch {ep} batch {n}: objf/frame {r.objf / max(r.frames, 1):.4f} ok {r.num_ok}/{r.num_seqs} "
                  f"{frames / (time.perf_counter() - t0):.0f} frames/s", flush=True)
        dl.reset()
        print(f"epoch {ep}: {n} batches, loader {dl.stats()}", flush=True)


if __name__ == "__main__":
    main()
