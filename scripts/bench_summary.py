"""One-screen summary of a bench.py JSON line: headline, step MFMA fraction, the per-class
roofline table, chain times, sub-results. usage: python scripts/bench_summary.py LOG"""
import json
import sys

for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    print(f"value {d['value']:.0f} frames/s  {d['ms_per_step']} ms/step  step_mfma_frac {d.get('step_mfma_frac')}")
    rl = d.get("roofline")
    if rl:
        print(f"roofline {rl['kernel']} bound {rl['bound']} frac {rl['frac']} mfma {rl['mfma_frac']} hbm {rl['hbm_frac']}")
        for c in rl.get("classes", []):
            print("   ", {k: v for k, v in c.items()})
    if d.get("chain"):
        print("chain", d["chain"])
    for k, v in d.get("sub_results", {}).items():
        print(k, {kk: vv for kk, vv in v.items() if kk in ("value", "ms_per_step", "step_mfma_frac", "dropin_per_op_abi_ms",
                                                           "fused_nnet_forward_ms", "cpu_ms_median", "gpu_ops_gemm_ms_median")})
