"""Sustained GEMM rate: one decoder layer's worth of the step's GEMM shapes (SmolLM-1.7B, T = 4096: q|k|v, out,
gate|up, down; forward, dgrad against a contiguous W^T, wgrad) issued back to back for --seconds, the rate
reported per window. Tells a GEMM's isolated burst rate from what the chip sustains over a training step's
duration (clock / power), the question behind the in-step GEMM rate.

  python scripts/gemm_sustained.py [--seconds 6] [--window 0.25]
  python scripts/gemm_sustained.py --each 1.0   (each GEMM of the layer alone, sustained for 1 s: its rate)
"""
import argparse
import json
import time

import torch
import torch.nn.functional as F

T, H, I = 4096, 2048, 8192


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--window", type=float, default=0.25)
    ap.add_argument("--each", type=float, default=0.0)
    args = ap.parse_args()
    torch.manual_seed(0)
    dev = "cuda"
    bf = torch.bfloat16
    ops, flops, named = [], 0.0, []
    for nm, N, K in (("qkv", 3 * H, H), ("out", H, H), ("gate_up", 2 * I, H), ("down", H, I)):
        x = torch.randn(T, K, device=dev, dtype=bf)
        w = torch.randn(N, K, device=dev, dtype=bf) * 0.02
        wt = w.t().contiguous()
        dy = torch.randn(T, N, device=dev, dtype=bf)
        g = torch.zeros(N, K, device=dev, dtype=bf)
        fs = [lambda x=x, w=w: F.linear(x, w), lambda dy=dy, wt=wt: F.linear(dy, wt),
              lambda dy=dy, x=x, g=g: torch.addmm(g, dy.t(), x, out=g)]
        ops += fs
        named += [(nm + "_" + k, f, 2.0 * T * N * K) for k, f in zip(("fwd", "dgrad", "wgrad"), fs)]
        flops += 3 * 2.0 * T * N * K
    if args.each > 0:
        for nm, f, fl in named:
            for _ in range(5):
                f()
            torch.cuda.synchronize()
            n, t0 = 0, time.perf_counter()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            while time.perf_counter() - t0 < args.each:
                f()
                n += 1
                if n % 32 == 0:
                    torch.cuda.synchronize()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / n
            print(json.dumps({"gemm": nm, "calls": n, "us": round(1e3 * ms, 1), "pflops": round(fl / ms / 1e12, 3)}),
                  flush=True)
        return

    def layer():
        for f in ops:
            f()
    for _ in range(3):
        layer()
    torch.cuda.synchronize()
    t_end = time.perf_counter() + args.seconds
    while time.perf_counter() < t_end:
        n = 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < args.window:
            layer()
            n += 1
            if n % 8 == 0:
                torch.cuda.synchronize()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        print(json.dumps({"t_s": round(args.seconds - (t_end - time.perf_counter()), 2), "layers": n,
                          "ms_per_layer": round(ms / n, 3), "pflops": round(flops * n / ms / 1e12, 3)}), flush=True)


if __name__ == "__main__":
    main()
