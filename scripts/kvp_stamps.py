"""Per-phase cycle anatomy of attn_bwd_kvp_kernel from the PICO_KVP_STAMP diagnostic build (C2 causal by default;
PICO_TL_SHAPE=B,S,H,D): every wave accumulates s_memtime deltas per tile phase — vmcnt wait, barrier, DMA issue +
cursor, M1(A) slots, M1(B) slots, M2(A) slots, M2(B) slots — which are ISSUE times (an MFMA is counted when it
issues, not when it completes). Prints the mean cycles per 64-row tile and phase, overall and by the workgroup's
dispatch class (block group g -> g * nbh / CUs: oldest first). The stamps cost ~10 % themselves.

  PICO_LIB_PATH=picotron_amd/lib/variants/kvpstamp.so PICO_ATTN_KVP=1 python scripts/kvp_stamps.py
(PICO_KVP_WAVES=8 for the 8-wave workgroups: the stamps are 16 words per wave at (block * NW + wave) * 16.)
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

PHASES = ["wait", "barrier", "issue", "M1A", "M1B", "M2A", "M2B"]


def main():
    B, S, H, D = (int(x) for x in os.environ.get("PICO_TL_SHAPE", "4,1024,32,64").split(","))
    torch.manual_seed(0)
    q, k, v, do = [torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16) for _ in range(4)]
    o, lse = ops.attention_block_fwd(q, k, v, 1 / math.sqrt(D), True)
    dq, dk, dv = (torch.empty_like(q) for _ in range(3))
    a = ops._attn_args(q, k, v, o, lse, 1 / math.sqrt(D), True)
    a.dout = L.ptr(do)
    a.do_strides = L.i64x3(do.stride()[:3])
    a.dq, a.dk, a.dv = L.ptr(dq), L.ptr(dk), L.ptr(dv)
    a.dq_strides, a.dk_strides, a.dv_strides = (L.i64x3(t.stride()[:3]) for t in (dq, dk, dv))
    lib = L.load()
    nbytes = lib.pico_attn_bwd_workspace_bytes(ctypes.byref(a))
    ws = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    a.workspace = L.ptr(ws)
    for _ in range(20):
        ws[nbytes - 65536 * 4 * 8:].zero_()
        L.check(lib.pico_attn_bwd(ctypes.byref(a), L.stream_of(q)), "bwd")
    torch.cuda.synchronize()
    nw = 8 if os.environ.get("PICO_KVP_WAVES") == "8" else 4  # waves per workgroup of the launch
    st = ws[nbytes - 65536 * 4 * 8:].cpu().numpy().view(np.uint64).astype(np.float64).reshape(-1, nw, 16)
    live = st[:, 0, 7] > 0
    st = st[live]
    nwg = st.shape[0]
    rt0, rt1 = st[:, :, 10], st[:, :, 11]  # s_memrealtime, 100 MHz
    clk = (st[:, :, 13] - st[:, :, 12]) / ((rt1 - rt0) / 100e6) / 1e9  # GHz per wave
    t0 = rt0.min()
    life_us = (rt1 - rt0) / 100.0
    tiles = st[:, :, 7:8]
    per_tile = st[:, :, :7] / np.maximum(tiles, 1)
    out = {"workgroups": int(nwg), "tiles_per_wave_mean": round(float(tiles.mean()), 2),
           "cycles_per_tile": {p: round(float((st[:, :, i].sum()) / tiles.sum()), 1) for i, p in enumerate(PHASES)}}
    out["cycles_per_tile"]["total"] = round(float(st[:, :, :7].sum() / tiles.sum()), 1)
    span = (rt1.max() - t0) / 100.0
    loop_cyc = st[:, :, :7].sum(axis=2)
    out["span_us"] = round(float(span), 2)
    out["clock_GHz_median"] = round(float(np.median(clk)), 3)
    out["wave_life_us_mean"] = round(float(life_us.mean()), 2)
    out["wave_life_us_max"] = round(float(life_us.max()), 2)
    # shares of a wave's lifetime (cycles): the tile loop, the blocks' prologues and epilogues, the rest (the
    # group's block switches, the kernel entry before the first block)
    life_cyc = st[:, :, 13] - st[:, :, 12]
    out["share_of_wave_life"] = {"loop": round(float(loop_cyc.sum() / life_cyc.sum()), 3),
                                 "prologue": round(float(st[:, :, 8].sum() / life_cyc.sum()), 3),
                                 "epilogue": round(float(st[:, :, 9].sum() / life_cyc.sum()), 3)}
    out["prologue_us_per_wave_mean"] = round(float((st[:, :, 8] / np.maximum(clk, 1e-3) / 1e3).mean()), 2)
    ends = (rt1.max(axis=1) - t0) / 100.0
    out["wg_end_us_percentiles"] = [round(float(np.percentile(ends, p)), 2) for p in (0, 10, 50, 90, 100)]
    nbh = B * H
    cus = 256
    cls = (np.arange(nwg) // nbh) * nbh // cus
    out["by_class"] = {}
    for c in sorted(set(cls.tolist())):
        m = cls == c
        out["by_class"][int(c)] = {p: round(float(st[m][:, :, i].sum() / st[m][:, :, 7].sum()), 1)
                                   for i, p in enumerate(PHASES)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
