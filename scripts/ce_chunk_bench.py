"""LM head + cross-entropy per micro-batch (forward + backward) at C2 (T 4096, H 2048, V 49152): the
unchunked fused form vs chunked forms (ops.lm_head_cross_entropy grad_scale / chunk), HIP events,
weight gradient accumulated onto an existing bf16 .grad. One JSON line per variant."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import ops  # noqa: E402


def main():
    T, H, V = 4096, 2048, 49152
    torch.manual_seed(0)
    x = (torch.randn(T, H, device="cuda") * 0.5).to(torch.bfloat16).requires_grad_(True)
    w = (torch.randn(V, H, device="cuda") * 0.02).to(torch.bfloat16).requires_grad_(True)
    w.grad = torch.zeros_like(w)
    tgt = torch.randint(0, V, (T,), device="cuda")
    for chunk in [0] + [int(c) for c in (sys.argv[1:] or ["512", "1024", "2048", "4096"])]:
        def run():
            if chunk == 0:
                loss = ops.lm_head_cross_entropy(x, w, tgt) / 32
            else:
                loss = ops.lm_head_cross_entropy(x, w, tgt, grad_scale=1 / 32, chunk=chunk)
            loss.backward()
            x.grad = None
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats()
        base = torch.cuda.memory_allocated()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 10
        e0.record()
        for _ in range(n):
            run()
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"chunk": chunk, "ms": round(e0.elapsed_time(e1) / n, 3),
                          "peak_extra_MB": round((torch.cuda.max_memory_allocated() - base) / 2**20, 1)}), flush=True)


if __name__ == "__main__":
    main()
