"""Phase timeline of attn_bwd_kv_kernel from the PICO_BWDKV_STAMP diagnostic build (workgroup 0 = key
block 0 of (b 0, kv-head 0): 32 query tiles at S 1024 causal). Per phase, the median cycles over tiles and
waves: 0->1 vmcnt wait + barrier, 1->2 DMA issue, 2->3 Q/dO reads + S/dP MFMAs (issue), 3->4 softmax +
dV/dK (issue), 4->next 0 loop overhead. Use with PICO_LIB_PATH=picotron_amd/lib/variants/stamp.so."""
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

TILES, PH = 48, 5


def main():
    B, S, H, D = 4, 1024, 32, 64
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
    off = nbytes - 8 * TILES * PH * 8
    st = ws[off:].cpu().numpy().view(np.uint64).astype(np.int64).reshape(-1, TILES, PH)
    ntiles = 32
    st = st[:, :ntiles]
    phases = [("wait+barrier", 0, 1), ("issue", 1, 2), ("tile", 2, 4), ("loop", 4, None)]
    out = {}
    for name, p0, p1 in phases:
        nxt = st[:, :, p1] if p1 is not None else np.concatenate([st[:, 1:, 0], st[:, -1:, 0]], 1)
        d = (nxt - st[:, :, p0])[:, 8: ntiles - 1]  # steady state: every wave active
        out[name] = [float(np.median(d[w])) for w in range(st.shape[0])]
    tot = (st[:, -1, 0] - st[:, 0, 0]) / (ntiles - 1)
    out["per_tile_total"] = [float(x) for x in tot]
    print(json.dumps(out))
    for w in range(st.shape[0]):
        print(w, (st[w, 16, [0, 1, 2, 4]] - st[w, 16, 0]).tolist(), "next", int(st[w, 17, 0] - st[w, 16, 0]))


if __name__ == "__main__":
    main()
