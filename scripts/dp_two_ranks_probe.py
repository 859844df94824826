"""Probe: can two ranks of kf_dp (the product's RCCL communicator, include/kf_dp.h) share
one GPU? Starts two child processes (no exec from a GPU process); rank 0 writes the
communicator id to a file, rank 1 reads it; both all-reduce (mean) a device buffer of
rank + 1 and report what they got (1.5 everywhere when the exchange works).

  python3 scripts/dp_two_ranks_probe.py [--timeout 60]
"""
import argparse
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(rank, idfile):
    import numpy as np
    import torch  # noqa: F401  (the HIP runtime first)
    sys.path.insert(0, os.path.join(ROOT, "kaldi-fp16_amd", "python"))
    import kfp16
    from kfp16 import dp
    kfp16.check(kfp16.core.bridge_gpu_init(0))
    if rank == 0:
        uid = dp.unique_id()
        with open(idfile + ".tmp", "wb") as fh:
            fh.write(uid)
        os.replace(idfile + ".tmp", idfile)
    else:
        t0 = time.time()
        while not os.path.exists(idfile):
            if time.time() - t0 > 30:
                raise SystemExit("rank 1: no id")
            time.sleep(0.05)
        uid = open(idfile, "rb").read()
    comm = dp.Communicator(rank, 2, uid, 0)
    n = 1 << 20
    buf = kfp16.upload_f32(np.full(n, rank + 1.0, np.float32))
    comm.allreduce_mean(buf.ptr, n)
    kfp16.check(kfp16.core.bridge_gpu_sync() if hasattr(kfp16.core, "bridge_gpu_sync") else 0)
    got = kfp16.read_f32(buf.ptr, (n,))
    print(f"rank {rank}: min {got.min()} max {got.max()} (expect 1.5)", flush=True)
    comm.close()
    return 0 if np.all(got == 1.5) else 1


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--timeout", type=int, default=60)
    p.add_argument("--child", type=int, default=-1)
    p.add_argument("--idfile", default="")
    a = p.parse_args()
    if a.child >= 0:
        return child(a.child, a.idfile)
    idfile = os.path.join(tempfile.mkdtemp(), "kfdp.id")
    env = dict(os.environ)
    procs = [subprocess.Popen([sys.executable, __file__, "--child", str(r), "--idfile", idfile], env=env)
             for r in range(2)]
    rc = 0
    t0 = time.time()
    for pr in procs:
        try:
            rc |= pr.wait(timeout=max(1, a.timeout - (time.time() - t0)))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            print("timeout", flush=True)
            return 124
    print("two ranks on one GPU:", "ok" if rc == 0 else f"failed rc={rc}", flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
