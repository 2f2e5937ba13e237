"""Where the DataParallelBucket step's extra time goes (RCCL W = 1): host issue time vs device time of the syncing
micro-batch's forward (issued beside the graph tail) and backward (hooks launching the bucket all-reduces), from a
wrapped Tensor.backward / train._forward_loss. One JSON line: per phase, host ms (perf_counter around the issue)
and device ms (HIP events on the issuing stream), mean over the timed steps.

  python scripts/dp_sync_probe.py [--steps 4] [--layers 15] [--grad-acc 32]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--layers", type=int, default=15)
    ap.add_argument("--grad-acc", type=int, default=32)
    args = ap.parse_args()
    import torch.distributed as dist
    import bench
    from picotron_amd import process_group_manager as pgm
    from picotron_amd import train as T
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29533"), RANK="0",
                      WORLD_SIZE="1", LOCAL_RANK="0")
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    pgm.setup_process_group_manager(1, 1, 1, 1)
    cfg, model, opt, loader, _ = bench.setup(args.layers, args.grad_acc, 1, dev, dp_bucket=True)
    step = T.TrainingStep(model, opt, loader, dev, graphs=True)
    rec = {"fwd": [], "bwd": [], "graph_run": []}
    live = [False]

    orig_fwd = T._forward_loss

    def fwd(*a, **k):
        if not (live[0] and model.require_backward_grad_sync):
            return orig_fwd(*a, **k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        out = orig_fwd(*a, **k)
        e1.record()
        rec["fwd"].append((time.perf_counter() - t0, e0, e1))
        return out
    T._forward_loss = fwd

    orig_bwd = torch.Tensor.backward

    def bwd(self, *a, **k):
        if not (live[0] and model.require_backward_grad_sync and torch.cuda.is_current_stream_capturing() is False):
            return orig_bwd(self, *a, **k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        out = orig_bwd(self, *a, **k)
        e1.record()
        rec["bwd"].append((time.perf_counter() - t0, e0, e1))
        return out
    torch.Tensor.backward = bwd

    orig_run = T.PipelinedMicroBatchGraph.run

    def run(self, batches, between=None):
        if not live[0]:
            return orig_run(self, batches, between)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        out = orig_run(self, batches, between)
        e1.record()
        rec["graph_run"].append((time.perf_counter() - t0, e0, e1))
        return out
    T.PipelinedMicroBatchGraph.run = run

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    live[0] = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(sync_loss=False)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.steps
    out = {"step_ms": round(1e3 * wall, 2), "tail_overlap": T.tail_overlap_enabled()}
    for k, v in rec.items():
        if v:
            out[k + "_host_ms"] = round(1e3 * sum(x[0] for x in v) / len(v), 2)
            out[k + "_device_ms"] = round(sum(x[1].elapsed_time(x[2]) for x in v) / len(v), 2)
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
