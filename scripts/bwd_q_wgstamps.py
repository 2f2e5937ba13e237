"""Workgroup timeline of attn_bwd_q_kernel from the PICO_BWDQ_WGSTAMP diagnostic build (C2 causal):
per workgroup s_memrealtime (100 MHz) at entry, loop start, loop end, stores drained. Prints the kernel
span, mean prologue / loop / epilogue per workgroup, the loop share of the summed workgroup time, and the
mean number of workgroups resident over the span. PICO_LIB_PATH=picotron_amd/lib/variants/qstamp.so."""
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
    B, S, H, D = (int(x) for x in os.environ.get("PICO_TL_SHAPE", "4,1024,32,64").split(","))  # C4: 2,1024,16,128
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
        L.check(lib.pico_attn_bwd(ctypes.byref(a), L.stream_of(q)), "bwd")
    torch.cuda.synchronize()
    off = nbytes - 65536 * 4 * 8
    st = ws[off:].cpu().numpy().view(np.uint64).astype(np.int64).reshape(-1, 4)
    nwg = (S // 128) * B * H
    st = st[:nwg].astype(np.float64) / 100.0  # us
    t0 = st[:, 0].min()
    st -= t0
    span = st[:, 3].max()
    pro, loop, epi = st[:, 1] - st[:, 0], st[:, 2] - st[:, 1], st[:, 3] - st[:, 2]
    life = st[:, 3] - st[:, 0]
    ts = np.linspace(0, span, 200)
    resident = [int(((st[:, 0] <= t) & (st[:, 3] > t)).sum()) for t in ts]
    nmb = S // 128
    front = int(os.getenv("QFRONT", "2"))  # the kernel's q_front (C2 on 256 CUs: 2)
    gi = np.arange(nwg) // (B * H)
    mb = np.where(gi < front, gi, nmb - 1 - (gi - front))
    by_kb = {int(k): {"start": round(float(st[mb == k, 0].mean()), 2), "end": round(float(st[mb == k, 3].mean()), 2),
                      "pro": round(float(pro[mb == k].mean()), 2),
                      "loop_per_tile": round(float(loop[mb == k].mean()) / (2 * (k + 1)), 3)}
             for k in range(nmb)}
    print(json.dumps({"workgroups": int(nwg), "span_us": round(span, 2), "prologue_us": round(pro.mean(), 2),
                      "by_query_block": by_kb,
                      "loop_us": round(loop.mean(), 2), "epilogue_us": round(epi.mean(), 2),
                      "loop_share_of_wg_time": round(loop.sum() / life.sum(), 3),
                      "mean_resident": round(float(np.mean(resident)), 1), "resident_profile": resident[::10],
                      "last_start_us": round(st[:, 0].max(), 2)}))


if __name__ == "__main__":
    main()
