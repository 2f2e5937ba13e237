"""Time the attention backward with the fused RoPE^-1 (PICO_ATTN_ROPE_BWD) against the unfused
sequence (attention backward, then pico_rope(conjugate=1) in place on dq|dk) at the SmolLM shape,
q/k/v as strided views of one qkv buffer like the model. Prints one JSON line (microseconds)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import ops  # noqa: E402
from picotron_amd.model import get_cos_sin  # noqa: E402


def main(iters=30):
    B, S, H, D = 4, 1024, 32, 64
    torch.manual_seed(0)
    qkv = torch.randn(B, S, 3 * H, D, dtype=torch.bfloat16, device="cuda")
    q, k, v = qkv[:, :, :H], qkv[:, :, H:2 * H], qkv[:, :, 2 * H:]
    do = torch.randn(B, S, H, D, dtype=torch.bfloat16, device="cuda")
    cos, sin = get_cos_sin(S, D, base=10000.0)
    cos, sin = cos.to("cuda", torch.bfloat16)[:, : D // 2], sin.to("cuda", torch.bfloat16)[:, : D // 2]
    sc = 1 / math.sqrt(D)
    o, lse = ops.attention_block_fwd(q, k, v, sc, True)
    dqkv = torch.empty_like(qkv)
    dq, dk, dv = dqkv[:, :, :H], dqkv[:, :, H:2 * H], dqkv[:, :, 2 * H:]

    def fused():
        ops._attention_bwd_into(do, q, k, v, o, lse, sc, True, dq, dk, dv, rope=(cos, sin))

    def unfused():
        ops._attention_bwd_into(do, q, k, v, o, lse, sc, True, dq, dk, dv)
        dqk = dqkv[:, :, : 2 * H]
        ops._rope_launch(dqk, dqk, cos, sin, True)

    res = {}
    for name, fn in (("unfused", unfused), ("fused", fused), ("unfused2", unfused), ("fused2", fused)):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        res[name + "_us"] = round(s.elapsed_time(e) / iters * 1e3, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
