"""The HBM-bound kernels timed inside eager training micro-batches (the regime of bench.py's `kernels` table):
SmolLM-1.7B width (hidden 2048, 32 heads, I 8192, V 49152) at `--layers` layers, micro-batch 4 x seq 1024, the
model's own fused path (RMSNorm residual form with y^T, RoPE on k, SwiGLU with h^T, the chunked LM-head CE).
Each kernel id is timed with the library's launch-carried HIP events over `--mb` micro-batches after warm-up;
one JSON line: {kernel: {avg_us, launches, GB/s, frac of 8 TB/s}} with bench.py's algorithmic bytes.
A/B: PICO_LIB_PATH=picotron_amd/lib/variants/<v>.so selects a library variant.

  python scripts/hbm_instep.py [--layers 4] [--mb 4]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--mb", type=int, default=4)
    args = ap.parse_args()
    import bench
    from picotron_amd import _lib as L
    from picotron_amd.data import SyntheticDataLoader
    from picotron_amd.model import build_llama, smollm_1_7b
    from picotron_amd.train import train_step
    L.load()
    cfg = smollm_1_7b(num_hidden_layers=args.layers, seq_length=1024)
    torch.manual_seed(42)
    m = build_llama(cfg, device="cuda", dtype=torch.bfloat16)
    loader = SyntheticDataLoader(4, 1024, args.mb, cfg.vocab_size, seed=1234, kind="uniform", num_batches=args.mb,
                                 device="cuda")
    train_step(m, loader, "cuda", graphs=None)  # warm-up: W^T copies, gradient buffers, pair buffers
    torch.cuda.synchronize()
    ids = [L.K_RMSNORM_FWD, L.K_RMSNORM_BWD, L.K_ROPE, L.K_SWIGLU_FWD, L.K_SWIGLU_BWD]
    for k in ids:
        L.prof_enable(k, args.mb * (args.layers * 4 + 8) + 16)
    train_step(m, loader, "cuda", graphs=None)
    torch.cuda.synchronize()
    out = {}
    for k in ids:
        tot, n = L.prof_collect(k)
        if not n:
            continue
        avg = 1e3 * tot / n
        w = bench.kernel_work(k, cfg, 4, 1024)
        gbs = w[0] / (avg * 1e-6) / 1e9 if w else None
        out[L.KERNEL_NAMES[k]] = {"avg_us": round(avg, 2), "launches": n,
                                  "GBps": round(gbs, 1) if gbs else None,
                                  "frac": round(gbs / bench.HBM_PEAK_GBS, 4) if gbs else None}
    L.load().pico_prof_enable(0, 0)
    print(json.dumps({"layers": args.layers, "micro_batches": args.mb, "lib": os.environ.get("PICO_LIB_PATH", "default"),
                      "kernels": out}))


if __name__ == "__main__":
    main()
