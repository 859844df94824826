"""Streaming reference rates on the box (torch kernels, HIP events): a write-only fill,
a copy (read + write) and a read + read + write add of [96,000 x 1536] fp16 tensors, the
shape of the TDNN-F K = 320 GEMMs' epilogue tensors."""
import torch

torch.cuda.set_device(0)
T, N = 96000, 1536
a = torch.randn(T, N, device="cuda").half()
b = torch.randn(T, N, device="cuda").half()
c = torch.empty_like(a)
nbytes = a.numel() * 2


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for name, fn, mult in [("fill (write)", lambda: c.fill_(1.0), 1), ("copy (r+w)", lambda: c.copy_(a), 2),
                       ("add (2r+w)", lambda: torch.add(a, b, out=c), 3)]:
    us = timeit(fn)
    print(f"{name:14s} {us:8.1f} us  {mult * nbytes / us / 1e3:7.0f} GB/s")
