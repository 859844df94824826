"""Headroom reference only (not the product path): hipBLASLt via torch.matmul
on the plain GEMM shapes of scripts/gemm_bench.py, fp16 in / fp16 out."""
import torch

T = 96000
shapes = [("sq8192", 8192, 8192, 8192), ("tdnnf_lin_fwd", T, 160, 3072),
          ("tdnnf_aff_fwd", T, 1536, 320), ("output_fwd", T, 3080, 256),
          ("conv6_fwd(plain)", T * 10, 256, 2304), ("conv2_fwd(plain)", T * 40, 64, 576),
          ("conv4_fwd(plain)", T * 20, 128, 1152),
          ("wgrad_lin", 3072, 160, T), ("wgrad_aff", 320, 1536, T)]
for label, M, N, K in shapes:
    if label.startswith("wgrad"):
        a = torch.randn(K, M, device="cuda", dtype=torch.float16).t()
        b = torch.randn(K, N, device="cuda", dtype=torch.float16)
    else:
        a = torch.randn(M, K, device="cuda", dtype=torch.float16)
        b = torch.randn(K, N, device="cuda", dtype=torch.float16)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        c = a @ b
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 10 * 1e3
    print(f"{label:24s} {us:9.1f} us {2*M*N*K/us/1e6:8.1f} TFLOP/s")
    del a, b, c
