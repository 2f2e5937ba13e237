"""Host-side cost of the C2 training step's phases (TrainingStep, pipelined graph): how long the host takes to
issue each phase, from an idle device (a synchronisation before each measured step, so no phase waits on a
full launch queue). One JSON line per step after warm-up, then the medians.

  python scripts/host_step_probe.py [--steps 4] [--layers 15]
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--layers", type=int, default=15)
    args = ap.parse_args()
    import bench
    from picotron_amd import _lib, ops
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.train import TrainingStep
    _lib.load()
    import socket
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=1, dp_size=1)
    cfg, model, opt, loader, _ = bench.setup(args.layers, 32, 1, dev)
    step = TrainingStep(model, opt, loader, dev)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    g = step.graphs
    orig_run = g.run
    t = {}

    def timed_run(batches):
        t0 = time.perf_counter()
        ops.refresh_weight_transposes()
        t["refresh_ms"] = 1e3 * (time.perf_counter() - t0)
        t1 = time.perf_counter()
        orig_run(batches)  # (refreshes again: a no-op now) copies + replay
        t["copies_replay_ms"] = 1e3 * (time.perf_counter() - t1)

    g.run = timed_run
    rows = []
    for _ in range(args.steps):
        torch.cuda.synchronize()
        t.clear()
        a = time.perf_counter()
        step.zero()
        b = time.perf_counter()
        loss = step.micro_batches(sync_loss=False)
        c = time.perf_counter()
        step.optimizer_step()
        d = time.perf_counter()
        step.reset()
        e = time.perf_counter()
        rows.append({"zero_ms": 1e3 * (b - a), "micro_batches_ms": 1e3 * (c - b), "optimizer_ms": 1e3 * (d - c),
                     "reset_ms": 1e3 * (e - d), **t})
        print(json.dumps({k: round(v, 3) for k, v in rows[-1].items()}), flush=True)
    torch.cuda.synchronize()
    med = {k: round(statistics.median(r[k] for r in rows), 3) for k in rows[0]}
    print(json.dumps({"median": med, "loss": float(loss)}), flush=True)


if __name__ == "__main__":
    main()
