"""Time one AdamW step over the SmolLM-1.7B (15 layers) bf16 parameter set: torch.optim.AdamW(fused=True)
(the reference's optimizer, ref train.py:204-209) vs picotron_amd.optim.AdamW (pico_adamw_bf16).
Prints one JSON line per optimizer: ms per step and algorithmic GB/s (14 B per parameter)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(iters=10):
    from picotron_amd.model import build_llama, smollm_1_7b
    from picotron_amd.optim import AdamW
    torch.manual_seed(0)
    m = build_llama(smollm_1_7b(num_hidden_layers=15, seq_length=1024), device="cuda", dtype=torch.bfloat16)
    params = list(m.parameters())
    for p in params:
        p.grad = torch.randn_like(p) * 1e-3
    n = sum(p.numel() for p in params)
    for name, opt in (("torch_fused", torch.optim.AdamW(params, lr=3e-4, fused=True)),
                      ("pico", AdamW(params, lr=3e-4))):
        for _ in range(2):
            opt.step()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            opt.step()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / iters
        print(json.dumps({"optimizer": name, "params": n, "ms": round(ms, 3),
                          "GB_s": round(14 * n / (ms * 1e-3) / 1e9, 1)}), flush=True)
        opt.state.clear()


if __name__ == "__main__":
    main()
