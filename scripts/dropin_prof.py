"""The drop-in per-op ABI forward of bench.py (dropin_forward) alone, for a rocprofv3
kernel summary: python scripts/dropin_prof.py [reps]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kaldi-fp16_amd", "python"))
import bench  # noqa: E402
import kfp16  # noqa: E402

torch.cuda.set_device(0)
kfp16.check(kfp16.core.bridge_gpu_init(0), "init")
kfp16.set_stream(torch.cuda.current_stream().cuda_stream)
a = argparse.Namespace(egs=64)
print(json.dumps(bench.dropin_forward(a, reps=int(sys.argv[1]) if len(sys.argv) > 1 else 3)))
