"""HBM-bound kernel micro-benchmark at the SmolLM-1.7B micro-batch shapes (T = 4 x 1024 tokens,
hidden 2048, intermediate 8192, 32 + 32 heads of 64): RMSNorm fwd/bwd (residual form), RoPE (q|k in
place on the fused qkv buffer), SwiGLU fwd/bwd (strided halves of the gate|up buffer), embedding
bwd. Times each launch with the library's HIP-event timer; prints one JSON line per kernel with
algorithmic GB/s (every input read once + every output written once).

  python scripts/kernel_bench.py [--cold] [--iters 50]

--cold reads a 1 GiB buffer between launches (untimed: the kernel timer brackets the kernel alone), so every
launch reads its inputs from HBM instead of the 256 MB MALL / L2 that a back-to-back loop leaves them in.
--cold-write fills the buffer instead: the caches are then also full of dirty lines whose write-back competes
with the kernel (round-4 first form; slower than the training step itself: too pessimistic)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--cold", action="store_true")
    ap.add_argument("--cold-write", action="store_true")
    args = ap.parse_args()
    iters = args.iters
    from picotron_amd import _lib as L
    from picotron_amd import ops
    L.load()
    T, H, I, NH, D, V = 4096, 2048, 8192, 32, 64, 49152
    bf = torch.bfloat16
    dev = "cuda"
    torch.manual_seed(0)
    x = torch.randn(T, H, dtype=bf, device=dev, requires_grad=True)
    r = torch.randn(T, H, dtype=bf, device=dev, requires_grad=True)
    w = torch.ones(H, dtype=bf, device=dev, requires_grad=True)
    qkv = torch.randn(4, 1024, 3 * NH, D, dtype=bf, device=dev)
    cos = torch.randn(1024, D // 2, dtype=bf, device=dev)
    sin = torch.randn(1024, D // 2, dtype=bf, device=dev)
    gu = torch.randn(T, 2 * I, dtype=bf, device=dev)
    h = torch.empty(T, I, dtype=bf, device=dev)
    dh = torch.randn(T, I, dtype=bf, device=dev)
    dgu = torch.empty_like(gu)
    ht = torch.empty(I, T, dtype=bf, device=dev)
    ids = torch.randint(0, V, (4, 1024), device=dev)
    dy_emb = torch.randn(4, 1024, H, dtype=bf, device=dev)
    gemb = torch.zeros(V, H, dtype=bf, device=dev)
    xt = torch.empty(H, T, dtype=bf, device=dev)
    wgu = torch.randn(2 * I, H, dtype=bf, device=dev)
    wgut = torch.empty(H, 2 * I, dtype=bf, device=dev)
    logits = torch.randn(T, V, dtype=bf, device=dev) * 4
    tgt = torch.randint(0, V, (T,), device=dev)
    lse = torch.empty(T, dtype=torch.float32, device=dev)
    loss_rows = torch.empty(T, dtype=torch.float32, device=dev)
    gscale = torch.full((1,), 1.0 / T, dtype=torch.float32, device=dev)

    def run_ce():  # fused LM-head CE pass: dlogits written over the logits (values drift; timing only)
        L.check(L.load().pico_cross_entropy_fwd_grad(L.ptr(logits), logits.stride(0), L.ptr(tgt), L.ptr(lse),
                                                     L.ptr(loss_rows), L.ptr(gscale), T, V, -100, L.stream_of(logits)),
                "pico_cross_entropy_fwd_grad")

    def run_norm():
        y, res = ops.rms_norm(x, w, 1e-5, residual=r, prenorm=True)
        torch.autograd.backward([y, res], [torch.ones_like(y), torch.ones_like(res)])

    dy2 = torch.randn(T, H, dtype=bf, device=dev)
    rstd = torch.rand(T, dtype=torch.float32, device=dev) + 0.5
    dxc = torch.empty(T, H, dtype=bf, device=dev)
    nb = int(L.load().pico_rmsnorm_bwd_partial_rows(T, H))
    ws_a = torch.zeros(nb, H, dtype=torch.float32, device=dev)
    ws_b = torch.zeros(nb, H, dtype=torch.float32, device=dev)
    mg_prev = torch.zeros(H, dtype=torch.float32, device=dev)

    def run_norm_chain():  # the in-step form: reduce the previous norm's partial rows (fp32 main_grad, mode 2)
        L.check(L.load().pico_rmsnorm_bwd_chain(
            L.ptr(dy2), L.ptr(r), L.ptr(x), L.ptr(w), L.ptr(rstd), L.ptr(dxc), None, 2, 1.0, L.ptr(ws_a), T, H, 0,
            L.ptr(ws_b), nb, H, L.ptr(mg_prev), 2, 1.0, L.stream_of(x)), "pico_rmsnorm_bwd_chain")

    def run_norm_t():
        ops._RMSNormFn.apply(x.detach(), r.detach(), w.detach(), 1e-5, True, True)

    cases = [
        ("rmsnorm", run_norm, [L.K_RMSNORM_FWD, L.K_RMSNORM_BWD, L.K_RMSNORM_DW]),
        ("rmsnorm_t", run_norm_t, [L.K_RMSNORM_FWD]),
        ("rmsnorm_chain", run_norm_chain, [L.K_RMSNORM_BWD]),
        ("rope", lambda: ops._rope_launch(qkv[:, :, :2 * NH], qkv[:, :, :2 * NH], cos, sin, False), [L.K_ROPE]),
        ("rope_k", lambda: ops._rope_launch(qkv[:, :, NH:2 * NH], qkv[:, :, NH:2 * NH], cos, sin, False), [L.K_ROPE]),
        ("swiglu", lambda: (ops._swiglu_fwd(gu, gu[:, I:], h, T, I, 2 * I, I),
                            ops._swiglu_bwd(dh, gu, gu[:, I:], dgu, dgu[:, I:], T, I, 2 * I, I)),
         [L.K_SWIGLU_FWD, L.K_SWIGLU_BWD]),
        ("swiglu_t", lambda: L.check(L.load().pico_swiglu_fwd_t(L.ptr(gu), L.ptr(gu[:, I:]), L.ptr(h), L.ptr(ht), T, I,
                                                                2 * I, I, T, L.stream_of(gu)), "pico_swiglu_fwd_t"),
         [L.K_SWIGLU_FWD]),
        ("embedding", lambda: ops._embedding_bwd_into(gemb, ids, dy_emb, 1.0), [L.K_SORT_IDS, L.K_EMBEDDING_BWD]),
        ("ce_fwd_grad", run_ce, [L.K_CE_FWD]),
        ("transpose_x", lambda: ops.transpose_2d(x.detach(), out=xt), [L.K_TRANSPOSE]),
        ("transpose_wgu", lambda: ops.transpose_2d(wgu, out=wgut), [L.K_TRANSPOSE]),
    ]
    flush = torch.ones(1 << 29, dtype=torch.bfloat16, device=dev) if (args.cold or args.cold_write) else None
    sink = torch.empty((), dtype=torch.float32, device=dev)
    work = {L.K_RMSNORM_FWD: 4 * T * H * 2 + 4 * T, L.K_RMSNORM_BWD: 4 * T * H * 2 + 4 * T,
            L.K_ROPE: 2 * T * 2 * NH * D * 2, L.K_SWIGLU_FWD: 3 * T * I * 2, L.K_SWIGLU_BWD: 5 * T * I * 2,
            L.K_EMBEDDING_BWD: T * H * 2 + 2 * T * H * 2, L.K_CE_FWD: 2 * T * V * 2}
    tbytes = {"transpose_x": 2 * T * H * 2, "transpose_wgu": 2 * 2 * I * H * 2}
    for name, fn, kids in cases:
        if L.K_TRANSPOSE in kids:
            work[L.K_TRANSPOSE] = tbytes[name]
        work[L.K_SWIGLU_FWD] = (4 if name == "swiglu_t" else 3) * T * I * 2
        work[L.K_ROPE] = 2 * T * (1 if name == "rope_k" else 2) * NH * D * 2
        # the y^T form also writes y^T (x, r read; residual, y, y^T written)
        work[L.K_RMSNORM_FWD] = (5 if name == "rmsnorm_t" else 4) * T * H * 2 + 4 * T
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        for k in kids:
            L.prof_enable(k, iters + 8)
        for _ in range(iters):
            if args.cold_write:
                flush.fill_(1.0)
            elif flush is not None:
                torch.sum(flush, dim=0, dtype=torch.float32, out=sink)
            fn()
        torch.cuda.synchronize()
        for k in kids:
            ms, n = L.prof_collect(k)
            us = 1e3 * ms / max(n, 1)
            out = {"cold": "write" if args.cold_write else bool(args.cold), "kernel": L.KERNEL_NAMES[k] + ("" if k not in (L.K_TRANSPOSE,) and name not in ("rmsnorm_t", "swiglu_t", "rmsnorm_chain", "rope_k") else ":" + name), "avg_us": round(us, 2), "launches": n}
            if k in work:
                out["GB_s"] = round(work[k] / (us * 1e-6) / 1e9, 1)
                out["frac_of_8TBs"] = round(out["GB_s"] / 8000, 3)
            print(json.dumps(out), flush=True)
        L.load().pico_prof_enable(0, 0)


if __name__ == "__main__":
    main()
