"""Cost of the training step's extras in the attention forward: mean launch time (library HIP-event timer) of the
plain forward, + q rotated in the kernel (PICO_ATTN_ROPE_Q_FWD, rotated q written back), + O^T written, and both
(the form the step runs), at the C2 shape (and others with --configs).

  python scripts/fwd_forms.py [--configs c2,d128] [--iters 50]
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CONFIGS = {"c2": (4, 1024, 32, 64), "d128": (4, 1024, 16, 128)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    from picotron_amd import _lib as L
    from picotron_amd import ops
    from picotron_amd.model import get_cos_sin
    L.load()
    for name in args.configs.split(","):
        B, S, H, D = CONFIGS[name]
        torch.manual_seed(0)
        q, k, v = [torch.randn(B, S, H, D, dtype=torch.bfloat16, device="cuda") for _ in range(3)]
        cos, sin = get_cos_sin(S, D, base=10000.0)
        cos, sin = cos.cuda()[:, : D // 2], sin.cuda()[:, : D // 2]
        o_t = torch.empty(H * D, B * S, dtype=torch.bfloat16, device="cuda")
        qs = q.clone()
        forms = {"plain": {}, "rope": {"rope_q": (cos, sin)}, "o_t": {"o_t": o_t},
                 "step": {"rope_q": (cos, sin), "o_t": o_t}}
        res = {"config": name, "B": B, "S": S, "H": H, "D": D}
        for rnd in range(args.rounds):
            for form, kw in forms.items():
                for _ in range(3):
                    ops.attention_block_fwd(qs, k, v, 1 / math.sqrt(D), True, **kw)
                torch.cuda.synchronize()
                L.prof_enable(L.K_ATTN_FWD, args.iters + 4)
                for _ in range(args.iters):
                    ops.attention_block_fwd(qs, k, v, 1 / math.sqrt(D), True, **kw)
                torch.cuda.synchronize()
                ms, n = L.prof_collect(L.K_ATTN_FWD)
                L.load().pico_prof_enable(0, 0)
                res.setdefault(form + "_us", []).append(round(1e3 * ms / max(n, 1), 2))
        for form in forms:
            res[form + "_us_min"] = min(res[form + "_us"])
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
