"""Time the attention forward with RoPE on q fused in (PICO_ATTN_ROPE_Q_FWD) against the unfused sequence
(pico_rope on q|k, then the plain forward) at the SmolLM shape, q/k/v as strided views of one qkv buffer like
the model. Prints one JSON line (microseconds per call, mean over `iters` back-to-back calls).
PICO_LIB_PATH selects a library variant (scripts/build_variants.py)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import ops  # noqa: E402
from picotron_amd.model import get_cos_sin  # noqa: E402


def timed(fn, iters):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000.0 / iters


def main(iters=100):
    B, S, H, D = 4, 1024, 32, 64
    torch.manual_seed(0)
    qkv = torch.randn(B, S, 3 * H, D, dtype=torch.bfloat16, device="cuda")
    q, k, v = qkv[:, :, :H], qkv[:, :, H:2 * H], qkv[:, :, 2 * H:]
    cos, sin = get_cos_sin(S, D, base=10000.0)
    cos, sin = cos.to("cuda", torch.bfloat16)[:, : D // 2], sin.to("cuda", torch.bfloat16)[:, : D // 2]
    sc = 1 / math.sqrt(D)
    qk = qkv[:, :, : 2 * H]
    res = {
        "lib": os.path.basename(os.environ.get("PICO_LIB_PATH", "shipped")),
        "fwd_us": timed(lambda: ops.attention_block_fwd(q, k, v, sc, True), iters),
        "fwd_rope_q_us": timed(lambda: ops.attention_block_fwd(q, k, v, sc, True, rope_q=(cos, sin)), iters),
        "rope_qk_us": timed(lambda: ops._rope_launch(qk, qk, cos, sin, False), iters),
        "rope_k_us": timed(lambda: ops._rope_launch(k, k, cos, sin, False), iters),
    }
    print(json.dumps({kk: (round(vv, 2) if isinstance(vv, float) else vv) for kk, vv in res.items()}), flush=True)


if __name__ == "__main__":
    main()
