"""Where the step's small device copies and fills come from: one eager C2 micro-batch (forward + backward) under
torch.profiler with Python stacks; prints, for every memcpy / memset / fill / copy kernel, the innermost
picotron_amd frame that issued it (or the ATen op), with counts.

  python scripts/trace_small_ops.py [--layers 15]
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=15)
    args = ap.parse_args()
    import socket
    import torch.distributed as dist
    import bench
    from picotron_amd import _lib
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.train import _micro_batch
    _lib.load()
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=1, dp_size=1)
    dev = torch.device("cuda", 0)
    cfg, model, opt, loader, _ = bench.setup(args.layers, 32, 1, dev)
    for p in model.parameters():
        p.grad = torch.zeros_like(p)
    b = next(loader)
    for _ in range(2):
        _micro_batch(model, b["input_ids"], b["target_ids"], 32)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        _micro_batch(model, b["input_ids"], b["target_ids"], 32)
        torch.cuda.synchronize()
    counts = collections.Counter()
    small = ("fillbuffer", "copybuffer", "fill", "memset", "memcpy", "copy")
    for ev in prof.events():
        if ev.device_type.name != "CPU":
            continue
        for k in ev.kernels:
            if any(t in k.name.lower() for t in small):
                frames = [f for f in (ev.stack or []) if "picotron_amd" in f or "bench.py" in f]
                counts[(k.name[:40], ev.name[:40], frames[0] if frames else "-")] += 1
    gpu = collections.Counter(ev.name[:60] for ev in prof.events() if ev.device_type.name != "CPU"
                              and any(t in ev.name.lower() for t in small))
    print("GPU small-op kernels:", dict(gpu))
    for (kname, op, where), c in counts.most_common(40):
        print(f"{c:4d}  {kname:40s}  {op:40s}  {where}")


if __name__ == "__main__":
    main()
