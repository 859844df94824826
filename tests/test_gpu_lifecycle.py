"""Object lifecycle and HIP error hygiene across the C-ABI.

BENCH_r05 died in bench.py's 7th network of one process: nnet_set_fp8 reported
"operation not permitted when stream is capturing", an error some earlier HIP call had
left pending and kf_quant_mxfp8_batch's hipGetLastError() then picked up. These tests
replay the bench's whole create / run / close sequence in one process at a small size,
and check that an error left pending before an entry point is consumed and logged
(kf_take_pending, include/kf_ops.h) instead of failing that entry.
"""
import pytest
import torch


@pytest.mark.gpu
def test_pending_error_is_not_misattributed(gpu):
    kf = gpu
    kf.core.kf_pending_clear()
    n = 4096
    src = torch.randn(n, device="cuda", dtype=torch.float32)
    dst = torch.empty(n, device="cuda", dtype=torch.float16)
    torch.cuda.synchronize()
    # a failing HIP call whose status is read by nobody: an impossible allocation
    assert not kf.core.bridge_gpu_malloc(1 << 62)
    kf.core.bridge_clear_error()
    pend = kf.core.kf_peek_error()
    rc = kf.core.bridge_fp32_to_fp16_gpu(dst.data_ptr(), src.data_ptr(), n)
    assert rc == 0, kf.core.bridge_last_error()
    torch.cuda.synchronize()
    assert torch.equal(dst, src.half())
    assert kf.core.kf_peek_error() == 0
    if pend:
        log = kf.pending_log()
        assert log is not None and "pending before bridge_fp32_to_fp16_gpu" in log, log
    kf.core.kf_pending_clear()
    assert kf.pending_log() is None
    # the next checked entry reports clean
    assert kf.core.bridge_fp32_to_fp16_gpu(dst.data_ptr(), src.data_ptr(), n) == 0
    assert kf.pending_log() is None


@pytest.mark.gpu
def test_bench_create_close_sequence(gpu):
    """bench.py's sequence at 2 egs: headline train 1536 (two streams), forward 1536,
    3072 train fp16 / MXFP8 twice, 3072 forward MXFP8, the drop-in per-op forward and the
    one-stream train step, all in this process, with no sub-result error and nothing left
    pending."""
    import bench
    kf = gpu
    a = bench.parse(["--egs", "2", "--extra-steps", "1", "--no-cpu-baseline"])
    kf.core.kf_pending_clear()
    head, _ = bench.run_workload(a, a.xconfig, "train", False, 0, 1, None, 2, 1, True)
    assert head["stats"][4] == a.egs
    extra, errors = bench.sub_results(a, 0, 1, True)
    assert not errors, errors
    for k in ("configs[1]_forward_1536", "configs[4]_train_3072_fp16", "configs[4]_train_3072_mxfp8",
              "configs[4]_forward_3072_mxfp8", "dropin_per_op_abi_forward", "train_1536_one_stream"):
        assert k in extra and "error" not in extra[k], k
    assert extra["dropin_per_op_abi_forward"]["output_rel_fro_dropin_vs_fused"] < 2e-2
    torch.cuda.synchronize()
    assert kf.core.kf_peek_error() == 0
    assert kf.pending_log() is None, kf.pending_log()
