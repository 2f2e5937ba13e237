"""Probe: the forward projection GEMMs of the C2 step (T = 4096 tokens) with the activation read as stored
(row-major [T, K], the form the step runs) vs read from its transposed copy ([K, T], which the producing
kernel already writes for the weight-gradient GEMM: y^T of the RMSNorm, h^T of the SwiGLU). If the transposed
form is no slower, the producers could skip their row-major write (16.8 MB per norm, 67 MB per SwiGLU).

  python scripts/gemm_at_probe.py [--iters 50] [--rounds 3]

One JSON line per shape: microseconds per GEMM for both forms (best of the interleaved rounds).
"""
import argparse
import json

import torch

SHAPES = {  # name: (K, N) of y[T, K] @ W[N, K]^T
    "qkv": (2048, 6144),
    "gate_up": (2048, 16384),
    "down": (8192, 2048),
    "out": (2048, 2048),
    "lm_head_chunk": (2048, 49152),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--tokens", type=int, default=4096)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    T = args.tokens
    torch.manual_seed(0)
    for name, (K, N) in SHAPES.items():
        x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
        xt = x.t().contiguous()  # [K, T]
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        ref = torch.matmul(x, w.t())
        alt = torch.matmul(xt.t(), w.t())
        same = bool(torch.equal(ref, alt))
        best = {"rows": 1e9, "t": 1e9}
        for _ in range(args.rounds):
            for form, a in (("rows", x), ("t", xt.t())):
                for _ in range(3):
                    torch.matmul(a, w.t())
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    torch.matmul(a, w.t())
                e1.record()
                torch.cuda.synchronize()
                best[form] = min(best[form], 1e3 * e0.elapsed_time(e1) / args.iters)
        fl = 2.0 * T * K * N
        print(json.dumps({"gemm": name, "T": T, "K": K, "N": N, "rows_us": round(best["rows"], 2),
                          "t_us": round(best["t"], 2), "rows_tflops": round(fl / best["rows"] / 1e6, 1),
                          "t_tflops": round(fl / best["t"] / 1e6, 1), "bitwise_equal": same}), flush=True)


if __name__ == "__main__":
    main()
