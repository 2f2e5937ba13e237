"""Weight-gradient GEMM with the micro-batch accumulation folded in (beta = 1) vs GEMM + separate add.
  bf16: G += dY^T X          (DP=1: .grad accumulates in the param dtype)
  fp32: M += dY^T X (fp32 C)  (DP>1: DataParallelBucket's fp32 main_grad)
One JSON line per shape; SmolLM-1.7B micro-batch 4 x 1024 tokens."""
import json

import torch

T, H, I = 4096, 2048, 8192
SHAPES = {"o_proj": (H, H), "qkv": (3 * H, H), "gate_up": (2 * I, H), "down": (H, I)}


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
    return s.elapsed_time(e) / it * 1e3


def main():
    torch.manual_seed(0)
    for name, (N, K) in SHAPES.items():
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        g = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
        m = torch.zeros(N, K, device="cuda", dtype=torch.float32)
        res = {"shape": name, "N": N, "K": K}
        res["plain_us"] = bench(lambda: torch.mm(dy.t(), x))
        res["plain_plus_add_bf16_us"] = bench(lambda: g.add_(torch.mm(dy.t(), x)))
        res["addmm_bf16_beta1_us"] = bench(lambda: torch.addmm(g, dy.t(), x, out=g))
        res["plain_plus_add_fp32_us"] = bench(lambda: m.add_(torch.mm(dy.t(), x)))
        try:
            res["addmm_fp32_beta1_us"] = bench(lambda: torch.addmm(m, dy.t(), x, out_dtype=torch.float32, out=m))
            ref = m.clone().zero_()
            torch.addmm(ref, dy.t(), x, out_dtype=torch.float32, out=ref)
            res["fp32_check_maxabs"] = float((ref - dy.float().t() @ x.float()).abs().max())
        except Exception as ex:  # noqa: BLE001
            res["addmm_fp32_error"] = str(ex)[:200]
        res = {k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.items()}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
