"""Workgroup timeline of attn_fwd_kernel from the PICO_FWD_WGSTAMP diagnostic build (C2 causal by default):
per workgroup s_memrealtime (100 MHz) at entry, loop start, loop end, stores drained. Prints the kernel span,
mean prologue / loop / epilogue per workgroup, the loop share of the summed workgroup time, the mean number of
workgroups resident over the span and the loop time per tile by query block.
PICO_LIB_PATH=picotron_amd/lib/variants/fwdstamp.so python scripts/fwd_wgstamps.py [--full] [--shape B,S,H,D]
(--shape 4,1024,16,128: C4's per-rank D = 128 forward)"""
import ctypes
import json
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import _lib as L  # noqa: E402
from picotron_amd import ops  # noqa: E402


def main():
    causal = "--full" not in sys.argv
    B, S, H, D = 4, 1024, 32, 64
    if "--shape" in sys.argv:
        B, S, H, D = (int(x) for x in sys.argv[sys.argv.index("--shape") + 1].split(","))
    torch.manual_seed(0)
    q, k, v = [torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16) for _ in range(3)]
    o = torch.empty_like(q)
    lse = torch.empty(B, H, S, device="cuda", dtype=torch.float32)
    a = ops._attn_args(q, k, v, o, lse, 1 / math.sqrt(D), causal)
    nmb = S // 128
    nwg = nmb * B * H
    st_buf = torch.zeros(nwg * 4, dtype=torch.int64, device="cuda")
    a.workspace = L.ptr(st_buf)
    lib = L.load()
    for _ in range(20):
        L.check(lib.pico_attn_fwd(ctypes.byref(a), L.stream_of(q)), "fwd")
    torch.cuda.synchronize()
    st = st_buf.cpu().numpy().reshape(-1, 4).astype(np.float64) / 100.0  # us
    st -= st[:, 0].min()
    span = st[:, 3].max()
    pro, loop, epi = st[:, 1] - st[:, 0], st[:, 2] - st[:, 1], st[:, 3] - st[:, 2]
    life = st[:, 3] - st[:, 0]
    ts = np.linspace(0, span, 200)
    resident = [int(((st[:, 0] <= t) & (st[:, 3] > t)).sum()) for t in ts]
    nbh = B * H
    lin = np.arange(nwg)
    if causal and os.getenv("PICO_FWD_SNAKE", "1") != "0":  # mirror the kernel's snake (rounds of 256 CUs)
        rnd, pos = lin // 256, lin % 256
        odd = ((rnd & 1) == 1) & ((rnd + 1) * 256 <= nwg)
        lin = np.where(odd, rnd * 256 + (256 - 8 - (pos & ~7)) + (pos & 7), lin)
    mb = (nmb - 1 - lin // nbh) if causal else lin // nbh
    tiles = 2 * (mb + 1) if causal else np.full(nwg, S // 64)
    per_tile = {int(m): round(float((loop[mb == m] / tiles[mb == m]).mean()), 3) for m in range(nmb)}
    print(json.dumps({"shape": [B, S, H, D], "causal": causal, "workgroups": int(nwg), "span_us": round(span, 2),
                      "prologue_us": round(pro.mean(), 2), "loop_us": round(loop.mean(), 2),
                      "epilogue_us": round(epi.mean(), 2), "loop_share_of_wg_time": round(loop.sum() / life.sum(), 3),
                      "mean_resident": round(float(np.mean(resident)), 1), "resident_profile": resident[::10],
                      "last_start_us": round(st[:, 0].max(), 2), "loop_us_per_tile_by_block": per_tile,
                      "end_us_by_block": {int(m): round(float(st[mb == m, 3].mean()), 2) for m in range(nmb)}}))


if __name__ == "__main__":
    main()
