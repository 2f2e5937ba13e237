"""Per-wave phase cycles of attn_fwd64_kernel from the PICO_FWD64_STAMP diagnostic build (s_memtime sums per
phase: prologue, mask + max phase, main block, tile wait + barrier, DMA issue, S-only segments, epilogue,
total). Prints the mean per wave over all waves, and per softmax segment.
PICO_LIB_PATH=picotron_amd/lib/variants/stamp.so python scripts/fwd64_stamps.py [--full]"""
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

NAMES = ["prologue", "max_phase", "main_block", "wait_barrier", "dma_issue", "s_only", "epilogue", "total"]


def main():
    causal = "--full" not in sys.argv
    B, S, H, D = 4, 1024, 32, 64
    torch.manual_seed(0)
    q, k, v = [torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16) for _ in range(3)]
    o = torch.empty_like(q)
    lse = torch.empty(B, H, S, device="cuda", dtype=torch.float32)
    a = ops._attn_args(q, k, v, o, lse, 1 / math.sqrt(D), causal)
    nwg = (S // 256) * B * H
    st_buf = torch.zeros(nwg * 4 * 8, dtype=torch.int64, device="cuda")
    a.workspace = L.ptr(st_buf)
    lib = L.load()
    for _ in range(20):
        L.check(lib.pico_attn_fwd(ctypes.byref(a), L.stream_of(q)), "fwd")
    torch.cuda.synchronize()
    st = st_buf.cpu().numpy().reshape(nwg * 4, 8).astype(np.float64)
    # softmax segments per wave: tiles 0..last per half (64-row waves): causal wave w of block mb sees
    # 4 mb + w + 1 tiles per half
    wave = np.tile(np.arange(4), nwg)
    lin = np.repeat(np.arange(nwg), 4)
    nbh = B * H
    if causal:
        rnd, pos = lin // 256, lin % 256
        odd = ((rnd & 1) == 1) & ((rnd + 1) * 256 <= nwg)
        lin = np.where(odd, rnd * 256 + (256 - 8 - (pos & ~7)) + (pos & 7), lin)
        mb = (S // 256 - 1) - lin // nbh
        segs = 2 * (4 * mb + wave + 1)
    else:
        segs = np.full(nwg * 4, 2 * S // 64)
    mean = {n: round(float(st[:, i].mean()), 1) for i, n in enumerate(NAMES)}
    per_seg = {n: round(float((st[:, i] / segs).mean()), 1) for i, n in enumerate(NAMES)}
    print(json.dumps({"causal": causal, "waves": int(nwg * 4), "mean_cycles_per_wave": mean,
                      "mean_cycles_per_softmax_segment": per_seg}))


if __name__ == "__main__":
    main()
