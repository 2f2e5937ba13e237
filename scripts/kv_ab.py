"""dK / dV kernel A/B through pico_select(PICO_SEL_ATTN_KVP, sel): D = 128 sel 0 = the 32-row attn_bwd_kv_kernel<128>,
1 = attn_bwd_kvp128_kernel; D = 64 sel 0 = 32-row, 1 = attn_bwd_kvp_kernel (the 64-keys-per-wave kernel that
took sel 2 was removed after measuring slower, commit 273720e). Per config: rel-L2 of dQ / dK / dV against an fp32 torch reference for
every selection, each selection's dK / dV against the first's, and the mean launch time of the dK/dV and dQ kernels
(library HIP-event timer) over --rounds interleaved rounds. One JSON line per config.

  python scripts/kv_ab.py [--configs d128,c2,...] [--sels 0,1] [--iters 30] [--rounds 3]
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CONFIGS = {  # B, S, Hq, Hkv, D, causal
    "d128": (4, 1024, 16, 16, 128, True),
    "d128_b2": (2, 1024, 16, 16, 128, True),
    "d128_full": (4, 1024, 16, 16, 128, False),
    "d128_gqa4": (4, 1024, 32, 8, 128, True),
    "d128_ragged": (1, 1000, 8, 8, 128, True),
    "d128_small": (1, 100, 2, 2, 128, True),
    "d128_s4096": (1, 4096, 16, 16, 128, True),
    "c2": (4, 1024, 32, 32, 64, True),
    "c2_full": (4, 1024, 32, 32, 64, False),
    "gqa4": (4, 1024, 32, 8, 64, True),
    "ragged": (1, 1000, 8, 8, 64, True),
    "small": (1, 100, 2, 2, 64, True),
    "cross": (2, 96, 200, 4, 4, 64, False),
    "s2048": (2, 2048, 32, 32, 64, True),
    "s4096": (1, 4096, 32, 32, 64, True),
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
    return [t.transpose(1, 2) for t in (qf.grad, kf.grad, vf.grad)]


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="d128_small,d128_ragged,d128,d128_full,d128_gqa4,d128_b2,d128_s4096")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--no-ref", action="store_true")
    ap.add_argument("--sels", default="0,1")
    args = ap.parse_args()
    from picotron_amd import _lib as L
    from picotron_amd import ops
    L.load()
    worst = 0.0
    for name in args.configs.split(","):
        cfg = CONFIGS[name]
        if len(cfg) == 7:  # cross lengths
            B, S, Sk, Hq, Hkv, D, causal = cfg
        else:
            B, S, Hq, Hkv, D, causal = cfg
            Sk = S
        torch.manual_seed(1)
        q = torch.randn(B, S, Hq, D, dtype=torch.bfloat16, device="cuda")
        k = torch.randn(B, Sk, Hkv, D, dtype=torch.bfloat16, device="cuda")
        v = torch.randn(B, Sk, Hkv, D, dtype=torch.bfloat16, device="cuda")
        do = torch.randn(B, S, Hq, D, dtype=torch.bfloat16, device="cuda")
        sc = 1 / math.sqrt(D)
        o, lse = ops.attention_block_fwd(q, k, v, sc, causal)
        res = {"config": name, "B": B, "S": S, "Hq": Hq, "Hkv": Hkv, "D": D, "causal": causal}
        outs = {}
        rg = None if args.no_ref else ref(q, k, v, do, sc, causal)
        sels = [(int(x), "s" + x) for x in args.sels.split(",")]
        for sel, tag in sels:
            L.select(L.SEL_ATTN_KVP, sel)
            g = ops.attention_block_bwd(do, q, k, v, o, lse, sc, causal)
            torch.cuda.synchronize()
            outs[tag] = g
            if rg is not None:
                for nm, a, b in zip(("dq", "dk", "dv"), g, rg):
                    res[f"{tag}_{nm}"] = round(rel(a, b), 6)
                    worst = max(worst, res[f"{tag}_{nm}"])
            res[f"{tag}_finite"] = bool(all(torch.isfinite(t).all() for t in g))
        for _, tag in sels[1:]:
            for i, nm in ((1, "dk"), (2, "dv")):
                res[f"{tag}_vs_{sels[0][1]}_{nm}"] = round(rel(outs[tag][i], outs[sels[0][1]][i]), 6)
        for rnd in range(args.rounds):
            for sel, tag in sels:
                L.select(L.SEL_ATTN_KVP, sel)
                for _ in range(3):
                    ops.attention_block_bwd(do, q, k, v, o, lse, sc, causal)
                torch.cuda.synchronize()
                for kid in (L.K_ATTN_BWD_KV, L.K_ATTN_BWD_Q):
                    L.prof_enable(kid, args.iters + 4)
                for _ in range(args.iters):
                    ops.attention_block_bwd(do, q, k, v, o, lse, sc, causal)
                torch.cuda.synchronize()
                for kid, nm in ((L.K_ATTN_BWD_KV, "kv"), (L.K_ATTN_BWD_Q, "q")):
                    ms, n = L.prof_collect(kid)
                    res.setdefault(f"{tag}_{nm}_us", []).append(round(1e3 * ms / max(n, 1), 2))
                L.load().pico_prof_enable(0, 0)
        L.select(L.SEL_ATTN_KVP, L.SEL_AUTO)
        for _, tag in sels:
            for nm in ("kv", "q"):
                res[f"{tag}_{nm}_us_min"] = min(res[f"{tag}_{nm}_us"])
        fl = 4.0 * B * Hq * S * Sk * D * (0.5 if causal else 1.0)
        for _, tag in sels:
            res[f"{tag}_kv_tflops"] = round(2.0 * fl / (res[f"{tag}_kv_us_min"] * 1e-6) / 1e12, 1)
        print(json.dumps(res), flush=True)
    if worst > 1e-2:
        print(f"FAIL worst rel-L2 {worst}", flush=True)
        sys.exit(1)


if __name__ == "__main__":
    main()
