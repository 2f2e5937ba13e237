"""Per-phase cycle anatomy of attn_fwdp_kernel from the PICO_FWDP_STAMP diagnostic build (C2 causal by default;
PICO_TL_SHAPE=B,S,H,D[,causal]): every wave accumulates s_memtime deltas (shader clock) per phase of its tiles.
Prints the mean cycles per active tile and phase, the per-item prologue / epilogue and the wave lifetime.

  PICO_LIB_PATH=picotron_amd/lib/variants/fwdpstamp.so python scripts/fwdp_stamps.py
"""
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

NAMES = ["Ph1", "Ph2", "Ph3", "dma_wait", "barrier", "dma_issue", "Ph4", "idle_tiles", "item_prologue",
         "epilogue", "b_tail", "active_tiles", "lifetime"]


def main():
    sh = [int(x) for x in os.environ.get("PICO_TL_SHAPE", "4,1024,32,64,1").split(",")]
    B, S, H, D = sh[:4]
    causal = bool(sh[4]) if len(sh) > 4 else True
    torch.manual_seed(0)
    q, k, v = [torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16) for _ in range(3)]
    o = torch.empty_like(q)
    lse = torch.empty(B, H, S, device="cuda", dtype=torch.float32)
    a = ops._attn_args(q, k, v, o, lse, 1 / math.sqrt(D), causal)
    ws = torch.zeros(65536 * 4 * 16 * 8, dtype=torch.uint8, device="cuda")
    a.workspace = L.ptr(ws)
    lib = L.load()
    for _ in range(20):
        L.check(lib.pico_attn_fwd(ctypes.byref(a), L.stream_of(q)), "fwd")
    torch.cuda.synchronize()
    st = ws.cpu().numpy().view(np.uint64).astype(np.float64).reshape(-1, 4, 16)
    live = st[:, 0, 12] > 0
    st = st[live]
    nt = st[:, :, 11].sum()
    res = {"shape": [B, S, H, D, causal], "workgroups": int(st.shape[0])}
    for i, n in enumerate(NAMES[:11]):
        tot = st[:, :, i].sum()
        res[n + "_per_tile" if i < 7 or i == 10 else n + "_per_wave"] = round(tot / nt if i < 7 or i == 10 else tot / st[:, :, 0].size, 1)
    res["active_tiles_per_wave"] = round(nt / st[:, :, 0].size, 2)
    res["lifetime_cycles_mean"] = round(float(st[:, :, 12].mean()), 0)
    rt = (st[:, :, 14] - st[:, :, 13]) / 100.0  # us
    res["lifetime_us_mean"] = round(float(rt.mean()), 2)
    res["clock_ghz"] = round(float((st[:, :, 12] / (rt * 1e3)).mean()), 3)
    t0 = st[:, :, 13].min()
    res["span_us"] = round(float((st[:, :, 14].max() - t0) / 100.0), 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
