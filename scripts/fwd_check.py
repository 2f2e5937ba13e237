"""Attention forward: the persistent 64-row-per-wave kernel (attn_fwdp.hip) against the 32-row kernel (attn_fwd.hip)
and an fp32 torch reference, in the plain form and in the training step's form (q rotated in the kernel, O^T
written). One JSON line per case: rel-L2 of O and max |dLSE| vs fp32 for both kernels, the new kernel's O / O^T /
rotated-q / LSE against the old kernel's, and the mean launch time of each (library HIP-event timer).

  python scripts/fwd_check.py [--cases c2,c2_full,...] [--iters 30]
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
    "c2_full": (4, 1024, 32, 32, 64, False),
    "gqa4": (4, 1024, 32, 8, 64, True),
    "odd": (2, 1344, 4, 4, 64, True),      # 21 tiles: a partial last 256-row block, odd block count
    "small": (1, 128, 2, 2, 64, True),      # nJ = 1: no pairs
    "s4096": (1, 4096, 32, 32, 64, True),
    "s4096_full": (1, 4096, 32, 32, 64, False),
    "cross_full": (2, 512, 4, 4, 64, False),
    "d128": (4, 1024, 16, 16, 128, True),
    "d128_full": (2, 1024, 16, 16, 128, False),
}


def ref(q, k, v, scale, causal):
    qf, kf, vf = [t.float().transpose(1, 2) for t in (q, k, v)]
    G = qf.shape[1] // kf.shape[1]
    ke, ve = kf.repeat_interleave(G, 1), vf.repeat_interleave(G, 1)
    s = qf @ ke.transpose(-1, -2) * scale
    if causal:
        S = s.shape[-1]
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    return (torch.softmax(s, -1) @ ve).transpose(1, 2), torch.logsumexp(s, -1)


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="c2,c2_full,gqa4,odd,small,s4096,s4096_full,cross_full,d128,d128_full")
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    from picotron_amd import _lib as L
    from picotron_amd import ops
    from picotron_amd.model import get_cos_sin
    L.load()
    for name in args.cases.split(","):
        B, S, Hq, Hkv, D, causal = CASES[name]
        torch.manual_seed(0)
        q = torch.randn(B, S, Hq, D, dtype=torch.bfloat16, device="cuda")
        k = torch.randn(B, S, Hkv, D, dtype=torch.bfloat16, device="cuda")
        v = torch.randn(B, S, Hkv, D, dtype=torch.bfloat16, device="cuda")
        sc = 1 / math.sqrt(D)
        o_ref, lse_ref = ref(q, k, v, sc, causal)
        cos, sin = get_cos_sin(S, D, base=10000.0)
        cos, sin = cos.cuda()[:, : D // 2], sin.cuda()[:, : D // 2]
        res = {"case": name, "B": B, "S": S, "Hq": Hq, "Hkv": Hkv, "D": D, "causal": causal}
        outs = {}
        for sel, tag in ((0, "old"), (1, "new")):
            L.select(L.SEL_ATTN_FWD, sel)
            o, lse = ops.attention_block_fwd(q, k, v, sc, causal)
            # the step's form: unrotated q in, rotated q written back, O^T
            qs = q.clone()
            o_t = torch.empty(Hq * D, B * S, dtype=torch.bfloat16, device="cuda")
            o2, lse2 = ops.attention_block_fwd(qs, k, v, sc, causal, o_t=o_t, rope_q=(cos, sin))
            torch.cuda.synchronize()
            outs[tag] = (o, lse, o2, lse2, qs, o_t)
            res[f"{tag}_o_rel"] = round(rel(o, o_ref), 6)
            res[f"{tag}_lse_maxabs"] = float((lse - lse_ref).abs().max())
            # timing: plain and step form
            for form in ("plain", "step"):
                for _ in range(3):
                    if form == "plain":
                        ops.attention_block_fwd(q, k, v, sc, causal)
                    else:
                        ops.attention_block_fwd(qs, k, v, sc, causal, o_t=o_t, rope_q=(cos, sin))
                torch.cuda.synchronize()
                L.prof_enable(L.K_ATTN_FWD, args.iters + 4)
                for _ in range(args.iters):
                    if form == "plain":
                        ops.attention_block_fwd(q, k, v, sc, causal)
                    else:
                        qs.copy_(q)
                        ops.attention_block_fwd(qs, k, v, sc, causal, o_t=o_t, rope_q=(cos, sin))
                torch.cuda.synchronize()
                ms, n = L.prof_collect(L.K_ATTN_FWD)
                L.load().pico_prof_enable(0, 0)
                res[f"{tag}_{form}_us"] = round(1e3 * ms / max(n, 1), 2)
        L.select(L.SEL_ATTN_FWD, L.SEL_AUTO)
        a, b = outs["old"], outs["new"]
        res["new_vs_old_o"] = round(rel(b[0], a[0]), 6)
        res["new_vs_old_lse_maxabs"] = float((b[1] - a[1]).abs().max())
        res["new_vs_old_step_o"] = round(rel(b[2], a[2]), 6)
        res["new_vs_old_step_lse"] = float((b[3] - a[3]).abs().max())
        res["rot_q_equal"] = bool(torch.equal(b[4], a[4]))
        res["o_t_vs_o"] = round(rel(b[5][:, : B * S].reshape(Hq, D, B, S).permute(2, 3, 0, 1), b[2]), 6)
        fl = 4.0 * B * Hq * S * S * D * (0.5 if causal else 1.0)
        res["new_tflops"] = round(fl / (res["new_plain_us"] * 1e-6) / 1e12, 1)
        res["old_tflops"] = round(fl / (res["old_plain_us"] * 1e-6) / 1e12, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
