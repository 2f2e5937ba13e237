"""Probe hipBLASLt layout sensitivity for the SmolLM-1.7B training GEMMs (M = 4096 tokens):
dgrad dx = dy @ W (NN) vs the same product in the forward's NT form F.linear(dy, W^T contiguous),
and wgrad dW = dy^T @ x (TN) vs (x^T @ dy)^T variants. One JSON line per shape (microseconds)."""
import json

import torch
import torch.nn.functional as F

T, H, I, V = 4096, 2048, 8192, 49152
SHAPES = {"qkv": (3 * H, H), "o": (H, H), "gate_up": (2 * I, H), "down": (H, I), "lm_head": (V, H)}


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
    return round(s.elapsed_time(e) / it * 1e3, 1)


def main():
    torch.manual_seed(0)
    for name, (N, K) in SHAPES.items():
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        wt = w.t().contiguous()
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        xt = x.t().contiguous()
        dyt = dy.t().contiguous()
        r = {"shape": name, "N": N, "K": K}
        r["fwd_NT"] = bench(lambda: F.linear(x, w))
        r["dgrad_NN"] = bench(lambda: dy @ w)
        r["dgrad_NT_wt"] = bench(lambda: F.linear(dy, wt))
        r["wgrad_TN"] = bench(lambda: dy.t() @ x)
        r["wgrad_NN_dyt"] = bench(lambda: dyt @ x)
        r["wgrad_NT_xt"] = bench(lambda: F.linear(dyt, xt))
        r["transpose_w"] = bench(lambda: w.t().contiguous())
        print(json.dumps(r), flush=True)


if __name__ == "__main__" and not {"--wgrad", "--fwd", "--dyt"} & set(__import__("sys").argv):
    main()


def wgrad_main():
    """wgrad as actually issued (beta = 1 accumulation into a bf16 grad) per input layout."""
    torch.manual_seed(0)
    for name, (N, K) in SHAPES.items():
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        xt, dyt = x.t().contiguous(), dy.t().contiguous()
        g = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
        r = {"shape": name, "N": N, "K": K}
        r["acc_TN"] = bench(lambda: torch.addmm(g, dy.t(), x, out=g))
        r["acc_NN_dyt"] = bench(lambda: torch.addmm(g, dyt, x, out=g))
        r["acc_NT_dyt_xt"] = bench(lambda: torch.addmm(g, dyt, xt.t(), out=g))
        r["acc_TT_dy_xt"] = bench(lambda: torch.addmm(g, dy.t(), xt.t(), out=g))
        if name == "lm_head":
            wt = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
            r["dgradT_NN"] = bench(lambda: wt @ dyt)   # dx^T = W^T dlogits^T
            r["dgrad_TN_dyt"] = bench(lambda: dyt.t() @ wt.t())
        r["transpose_dy"] = bench(lambda: dy.t().contiguous())
        print(json.dumps(r), flush=True)


if __name__ == "__main__" and "--wgrad" in __import__("sys").argv:
    wgrad_main()


def fwd_main():
    """forward y = x W^T with x given row-major (NT) vs as a transposed view of x^T [K, T] (TT)."""
    torch.manual_seed(0)
    for name in ("qkv", "gate_up", "lm_head", "o", "down"):
        N, K = SHAPES[name]
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        xt = x.t().contiguous()
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        r = {"shape": name, "N": N, "K": K}
        r["fwd_NT"] = bench(lambda: F.linear(x, w))
        r["fwd_from_xt"] = bench(lambda: torch.matmul(xt.t(), w.t()))
        print(json.dumps(r), flush=True)


if __name__ == "__main__" and "--fwd" in __import__("sys").argv:
    fwd_main()


def dyt_main():
    """Everything a layer's backward would issue if the producer of dy wrote ONLY dy^T ([N, T]):
    dgrad dx = dy W from dy^T (two forms) against the current form F.linear(dy, W^T), and the wgrad
    accumulation dW += dy^T x in the NT form (dy^T, x^T given) against the current TT form (dy, x^T)."""
    torch.manual_seed(0)
    for name, (N, K) in SHAPES.items():
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        wt = w.t().contiguous()
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        xt, dyt = x.t().contiguous(), dy.t().contiguous()
        g = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
        r = {"shape": name, "N": N, "K": K}
        r["dgrad_cur_linear_dy_wt"] = bench(lambda: F.linear(dy, wt))
        r["dgrad_dyt_mm_w"] = bench(lambda: dyt.t() @ w)
        r["dgrad_dyt_linear_wt"] = bench(lambda: F.linear(dyt.t(), wt))
        r["wgrad_cur_TT"] = bench(lambda: torch.addmm(g, dy.t(), xt.t(), out=g))
        r["wgrad_NT_dyt_xt"] = bench(lambda: torch.addmm(g, dyt, xt.t(), out=g))
        print(json.dumps(r), flush=True)


if __name__ == "__main__" and "--dyt" in __import__("sys").argv:
    dyt_main()
