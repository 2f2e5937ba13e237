"""Time the attention forward with RoPE on q fused in (PICO_ATTN_ROPE_Q_FWD) against the unfused sequence
(pico_rope on q|k, then the plain forward) and the training step's form (rope on q fused + O^T written), at the SmolLM shape, q/k/v as strided views of one qkv buffer like
the model. Prints one JSON line (microseconds per call, mean over `iters` back-to-back calls).
PICO_LIB_PATH selects a library variant (scripts/build_variants.py)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import _lib as L  # noqa: E402
from picotron_amd import ops  # noqa: E402
from picotron_amd.model import get_cos_sin  # noqa: E402


def timed(fn, iters, kid):
    """Mean kernel duration (the library's per-launch HIP-event timer), not the host-bound call rate."""
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    L.prof_enable(kid, iters + 8)
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    ms, n = L.prof_collect(kid)
    L.load().pico_prof_enable(0, 0)
    return 1000.0 * ms / max(n, 1)


def main(iters=100):
    B, S, H, D = 4, 1024, 32, 64
    torch.manual_seed(0)
    qkv = torch.randn(B, S, 3 * H, D, dtype=torch.bfloat16, device="cuda")
    q, k, v = qkv[:, :, :H], qkv[:, :, H:2 * H], qkv[:, :, 2 * H:]
    cos, sin = get_cos_sin(S, D, base=10000.0)
    cos, sin = cos.to("cuda", torch.bfloat16)[:, : D // 2], sin.to("cuda", torch.bfloat16)[:, : D // 2]
    sc = 1 / math.sqrt(D)
    qk = qkv[:, :, : 2 * H]
    o_t = torch.empty(H * D, B * S, dtype=torch.bfloat16, device="cuda")
    res = {
        "lib": os.path.basename(os.environ.get("PICO_LIB_PATH", "shipped")),
        "fwd_us": timed(lambda: ops.attention_block_fwd(q, k, v, sc, True), iters, L.K_ATTN_FWD),
        "fwd_rope_q_us": timed(lambda: ops.attention_block_fwd(q, k, v, sc, True, rope_q=(cos, sin)), iters, L.K_ATTN_FWD),
        "fwd_step_us": timed(lambda: ops.attention_block_fwd(q, k, v, sc, True, o_t=o_t, rope_q=(cos, sin)), iters, L.K_ATTN_FWD),
        "rope_qk_us": timed(lambda: ops._rope_launch(qk, qk, cos, sin, False), iters, L.K_ROPE),
        "rope_k_us": timed(lambda: ops._rope_launch(k, k, cos, sin, False), iters, L.K_ROPE),
    }
    print(json.dumps({kk: (round(vv, 2) if isinstance(vv, float) else vv) for kk, vv in res.items()}), flush=True)


if __name__ == "__main__":
    main()
