"""Numerics check of the attention kernels of the loaded library (PICO_LIB_PATH selects an A/B
variant) against a torch fp32 reference on the GPU: one JSON line per case with the relative L2 error
of O, dQ, dK, dV. Used to gate kernel variants before timing them (scripts/ab_attn.sh).

  python scripts/attn_check.py [--cases c2,odd,s4096]
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CASES = {  # B, S, Hq, Hkv, D, causal
    "c2": (4, 1024, 32, 32, 64, True),
    "odd": (2, 640, 8, 8, 64, True),       # 5 query / key blocks: the middle block of a pair runs alone
    "ragged": (1, 1000, 4, 4, 64, True),
    "gqa4": (4, 1024, 32, 8, 64, True),
    "s4096": (1, 4096, 32, 32, 64, True),
    "s4096_full": (1, 4096, 8, 8, 64, False),
    "s3000": (1, 3000, 8, 4, 64, True),
    "full": (2, 1024, 8, 8, 64, False),
    "fold5": (6, 640, 32, 32, 64, True),      # 5 blocks x 192 heads > one round: one folded pair per head
    "fold_ragged": (7, 1000, 32, 32, 64, True),  # ragged last block inside a folded pair
    "grp_ragged": (4, 1000, 32, 32, 64, True),   # one-round block groups (dQ and dK/dV) with a ragged last block
    "grp_10": (4, 1280, 32, 32, 64, True),       # ten blocks per head into six groups
    "d128": (4, 1024, 16, 16, 128, True),   # Llama-2-7B per tp-2 rank, the reference's micro-batch 4
    "d128_b2": (2, 1024, 16, 16, 128, True),
    "d128_ragged": (1, 1000, 8, 8, 128, True),
    "d128_full": (4, 1024, 16, 16, 128, False),
    "d128_s4096": (1, 4096, 16, 16, 128, True),
}


def ref(q, k, v, do, scale, causal):
    qf, kf, vf = [t.float().transpose(1, 2).requires_grad_() for t in (q, k, v)]
    G = qf.shape[1] // kf.shape[1]
    ke, ve = kf.repeat_interleave(G, 1), vf.repeat_interleave(G, 1)
    s = qf @ ke.transpose(-1, -2) * scale
    if causal:
        S = s.shape[-1]
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    o = torch.softmax(s, -1) @ ve
    o.backward(do.float().transpose(1, 2))
    return [t.transpose(1, 2) for t in (o.detach(), qf.grad, kf.grad, vf.grad)]


def rel(a, b):
    return float((a.float() - b).norm() / b.norm().clamp_min(1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="c2,odd,ragged,gqa4,s4096,full")
    args = ap.parse_args()
    from picotron_amd import ops
    worst = 0.0
    for name in args.cases.split(","):
        B, S, Hq, Hkv, D, causal = CASES[name]
        torch.manual_seed(1)
        q = torch.randn(B, S, Hq, D, dtype=torch.bfloat16, device="cuda")
        k = torch.randn(B, S, Hkv, D, dtype=torch.bfloat16, device="cuda")
        v = torch.randn(B, S, Hkv, D, dtype=torch.bfloat16, device="cuda")
        do = torch.randn(B, S, Hq, D, dtype=torch.bfloat16, device="cuda")
        sc = 1 / math.sqrt(D)
        o, lse = ops.attention_block_fwd(q, k, v, sc, causal)
        dq, dk, dv = ops.attention_block_bwd(do, q, k, v, o, lse, sc, causal)
        torch.cuda.synchronize()
        ro, rdq, rdk, rdv = ref(q, k, v, do, sc, causal)
        res = {"case": name, "o": rel(o, ro), "dq": rel(dq, rdq), "dk": rel(dk, rdk), "dv": rel(dv, rdv)}
        res = {kk: (round(vv, 6) if isinstance(vv, float) else vv) for kk, vv in res.items()}
        worst = max(worst, res["dq"], res["dk"], res["dv"], res["o"])
        print(json.dumps(res), flush=True)
    if worst > 1e-2:
        print(f"FAIL worst rel-L2 {worst}", flush=True)
        sys.exit(1)


if __name__ == "__main__":
    main()
