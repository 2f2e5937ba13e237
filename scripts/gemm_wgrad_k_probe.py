"""Probe: the weight-gradient GEMMs of the C2 step (dW[N, K] += dy[T, N]^T x[T, K], bf16, beta = 1, the
production call torch.addmm(g, dy.t(), x, out=g) with x given as the transposed view of x^T where the step keeps
x^T) at T = 4096 tokens (one micro-batch) vs T = 8192 (two micro-batches in one GEMM): is one K = 8192 GEMM
cheaper than two K = 4096 ones? One JSON line per projection.

  python scripts/gemm_wgrad_k_probe.py [--iters 30]
"""
import argparse
import json

import torch

SHAPES = {  # name: (N out rows, K in cols, x kept transposed)
    "qkv": (6144, 2048, True),
    "out": (2048, 2048, True),
    "gate_up": (16384, 2048, True),
    "down": (2048, 8192, True),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--tokens", default="4096,8192", help="comma list of T")
    ap.add_argument("--layouts", default="t", help="x operand layouts: t (the transposed view of a stored x^T, the "
                                                     "step's form), r (row-major x), or t,r")
    args = ap.parse_args()
    TOKENS = [int(t) for t in args.tokens.split(",")]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for (name, (N, K, _)), lay in [(it, lay) for it in SHAPES.items() for lay in args.layouts.split(",")]:
        xt = lay == "t"
        g = torch.zeros(N, K, device=dev, dtype=torch.bfloat16)
        res = {"gemm": name, "N": N, "K": K, "x_layout": "x^T stored" if xt else "x row-major"}
        for T in TOKENS:
            dy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
            x = torch.randn(K, T, device=dev, dtype=torch.bfloat16).t() if xt else \
                torch.randn(T, K, device=dev, dtype=torch.bfloat16)
            best = 1e9
            for _ in range(3):
                for _ in range(3):
                    torch.addmm(g, dy.t(), x, out=g)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    torch.addmm(g, dy.t(), x, out=g)
                e1.record()
                torch.cuda.synchronize()
                best = min(best, 1e3 * e0.elapsed_time(e1) / args.iters)
            res[f"T{T}_us"] = round(best, 2)
            res[f"T{T}_tflops"] = round(2.0 * T * N * K / best / 1e6, 1)
        if "T4096_us" in res and "T8192_us" in res:
            res["two_4096_vs_one_8192_us"] = [round(2 * res["T4096_us"], 2), res["T8192_us"]]
        if "T4096_us" in res and "T16384_us" in res:
            res["four_4096_vs_one_16384_us"] = [round(4 * res["T4096_us"], 2), res["T16384_us"]]
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
