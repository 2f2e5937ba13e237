"""Attention kernel micro-benchmark at the SmolLM-1.7B shape (B=4, S=1024, H=32, D=64, causal) and
optionally D=128 / GQA. Times every kernel id live with the library's HIP-event timer and prints
one JSON line per config (TFLOP/s against the algorithmic causal FLOPs).

  python scripts/attn_bench.py [--iters 50] [--configs c2,d128]
  PICO_LIB_PATH=... selects an alternative build of the library (ablation variants).
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CONFIGS = {
    "c2": (4, 1024, 32, 32, 64, True),
    "c2_full": (4, 1024, 32, 32, 64, False),
    "d128": (4, 1024, 16, 16, 128, True),   # Llama-2-7B per TP rank (tp2), the reference's micro-batch 4
    "d128_b2": (2, 1024, 16, 16, 128, True),   # the same at micro-batch 2 (half the work: one 256-CU round)
    "gqa4": (4, 1024, 32, 8, 64, True),
    "s4096": (1, 4096, 32, 32, 64, True),   # CP block size of config 5
    "s4096_full": (1, 4096, 32, 32, 64, False),  # config 5's off-diagonal ring blocks
    "s2048": (2, 2048, 32, 32, 64, True),
    "d128_full": (4, 1024, 16, 16, 128, False),
    "d128_s4096": (1, 4096, 16, 16, 128, True),
    "d128_gqa4": (4, 1024, 32, 8, 128, True),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--configs", default="c2,d128")
    ap.add_argument("--strided", action="store_true",
                    help="q / k / v as strided views of one [B, S, (Hq + 2 Hkv) D] buffer (the training step's layout)")
    ap.add_argument("--cold", action="store_true",
                    help="overwrite a 1-GiB buffer before every iteration (the inputs leave L2 and the Infinity Cache)")
    args = ap.parse_args()
    from picotron_amd import _lib as L
    from picotron_amd import ops
    L.load()
    for name in args.configs.split(","):
        B, S, Hq, Hkv, D, causal = CONFIGS[name]
        torch.manual_seed(0)
        if args.strided:
            qkv = torch.randn(B, S, Hq + 2 * Hkv, D, dtype=torch.bfloat16, device="cuda")
            q, k, v = qkv.split([Hq, Hkv, Hkv], dim=2)
        else:
            q = torch.randn(B, S, Hq, D, dtype=torch.bfloat16, device="cuda")
            k = torch.randn(B, S, Hkv, D, dtype=torch.bfloat16, device="cuda")
            v = torch.randn(B, S, Hkv, D, dtype=torch.bfloat16, device="cuda")
        do = torch.randn(B, S, Hq, D, dtype=torch.bfloat16, device="cuda")
        sc = 1 / math.sqrt(D)
        for _ in range(3):
            o, lse = ops.attention_block_fwd(q, k, v, sc, causal)
            ops.attention_block_bwd(do, q, k, v, o, lse, sc, causal)
        torch.cuda.synchronize()
        ids = [L.K_ATTN_FWD, L.K_ATTN_BWD_DKV, L.K_ATTN_BWD_Q,
               L.K_ATTN_BWD_KV]
        for i in ids:
            L.prof_enable(i, args.iters + 4)
        flush = torch.empty(1 << 29, dtype=torch.bfloat16, device="cuda") if args.cold else None
        for _ in range(args.iters):
            if flush is not None:
                flush.fill_(1.0)
            o, lse = ops.attention_block_fwd(q, k, v, sc, causal)
            if flush is not None:
                flush.fill_(2.0)
            ops.attention_block_bwd(do, q, k, v, o, lse, sc, causal)
        torch.cuda.synchronize()
        fl = 4.0 * B * Hq * S * S * D * (0.5 if causal else 1.0)
        res = {"config": name, "strided": args.strided, "cold": args.cold, "B": B, "S": S, "Hq": Hq, "Hkv": Hkv, "D": D, "causal": causal}
        # wall time of the whole backward call on the caller's stream (kernel timers off): the dQ and dK/dV
        # kernels plus the launch gaps between them
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            ops.attention_block_bwd(do, q, k, v, o, lse, sc, causal)
        e1.record()
        torch.cuda.synchronize()
        res["bwd_wall_us"] = round(1e3 * e0.elapsed_time(e1) / args.iters, 2)
        tot_bwd = 0.0
        for i in ids:
            ms, n = L.prof_collect(i)
            us = 1e3 * ms / max(n, 1)
            res[L.KERNEL_NAMES[i] + "_us"] = round(us, 2)
            if i != L.K_ATTN_FWD:
                tot_bwd += us
        L.load().pico_prof_enable(0, 0)
        res["fwd_tflops"] = round(fl / (res["attn_fwd_us"] * 1e-6) / 1e12, 1)
        res["bwd_total_tflops"] = round(2.5 * fl / (tot_bwd * 1e-6) / 1e12, 1)
        res["bwd_wall_tflops"] = round(2.5 * fl / (res["bwd_wall_us"] * 1e-6) / 1e12, 1)
        res["fwd_bwd_tflops"] = round(3.5 * fl / ((res["attn_fwd_us"] + tot_bwd) * 1e-6) / 1e12, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
