"""Time the SmolLM-1.7B training GEMMs (hipBLASLt via torch) at micro-batch 4 x 1024 tokens:
forward y = x W^T, dgrad dx = dy W, wgrad dW = dy^T x, for the separate and the fused
(q|k|v, gate|up) weight layouts. Prints one JSON line per shape. Run twice to compare
PYTORCH_TUNABLEOP_ENABLED=0/1."""
import json
import os
import sys

import torch
import torch.nn.functional as F

T, H, I, V = 4096, 2048, 8192, 49152
SHAPES = {
    "q/k/v/o": (H, H),
    "qkv_fused": (3 * H, H),
    "gate/up": (I, H),
    "gate_up_fused": (2 * I, H),
    "down": (H, I),
    "lm_head": (V, H),
}


def bench(fn, it=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    torch.manual_seed(0)
    dev = "cuda"
    tag = os.environ.get("PYTORCH_TUNABLEOP_ENABLED", "0")
    for name, (N, K) in SHAPES.items():
        x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        dy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * T * N * K
        res = {"shape": name, "M": T, "N": N, "K": K, "tunableop": tag}
        for kind, fn in (("fwd", lambda: F.linear(x, w)), ("dgrad", lambda: dy @ w), ("wgrad", lambda: dy.t() @ x)):
            ms = bench(fn)
            res[kind + "_us"] = round(ms * 1e3, 1)
            res[kind + "_tflops"] = round(fl / ms / 1e9, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
