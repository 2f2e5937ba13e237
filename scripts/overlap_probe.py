"""Probe: how much does overlapping micro-batch i+1's forward with micro-batch i's backward (two HIP streams)
gain over the serial grad-accumulation loop (ref train.py:33-51), eagerly, at the C2 shape?

  python scripts/overlap_probe.py [--layers 15] [--n 16] [--reps 3] [--graph]

--graph captures each order once as a HIP graph and times its replays (the bench's form: eagerly the host
issue rate, not the device, bounds a micro-batch).

Serial: fwd(i), bwd(i) for i in 0..n-1 on one stream. Overlapped: fwd(i) on stream i % 2; bwd(i - 1) is issued
before fwd(i) and runs on its forward's stream (autograd); bwd(i) waits for bwd(i - 1) (the gradient buffers
accumulate in micro-batch order, as in the serial loop). Prints one JSON line with ms per micro-batch and the
max |grad difference| between the two orders (the accumulation order is the same, so 0 expected).
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
    ap.add_argument("--layers", type=int, default=15)
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--graph", action="store_true")
    args = ap.parse_args()
    from picotron_amd import _lib, ops
    from picotron_amd.model import build_llama, smollm_1_7b
    _lib.load()
    dev = torch.device("cuda", 0)
    cfg = smollm_1_7b(num_hidden_layers=args.layers, seq_length=1024)
    torch.manual_seed(42)
    model = build_llama(cfg, device=dev)
    with torch.no_grad():
        model.final_proj.weight.normal_(0, 0.02)
    g = torch.Generator().manual_seed(3)
    toks = [torch.randint(0, cfg.vocab_size, (4, 1025), generator=g).to(dev) for _ in range(args.n)]
    head = model.final_proj
    n = args.n

    def fwd(i):
        h = model(input_ids=toks[i][:, :-1], return_hidden=True)
        return ops.lm_head_cross_entropy(h, head.weight, toks[i][:, 1:].reshape(-1), grad_scale=1.0 / n)

    for p in model.parameters():
        p.grad = torch.zeros_like(p)

    def zero():
        for p in model.parameters():
            p.grad.zero_()

    def serial():
        for i in range(n):
            fwd(i).backward()

    s = [torch.cuda.Stream(), torch.cuda.Stream()]

    def overlapped():
        main = torch.cuda.current_stream()
        for st in s:
            st.wait_stream(main)
        losses = [None] * n
        done = None  # event: the previous micro-batch's backward finished
        fdone = None  # event: the previous micro-batch's forward finished
        for i in range(n + 1):
            if i >= 1:  # backward of micro-batch i - 1, on its forward's stream, after the one before it
                st = s[(i - 1) % 2]
                with torch.cuda.stream(st):
                    if done is not None:
                        st.wait_event(done)
                    losses[i - 1].backward()
                    done = torch.cuda.Event()
                    done.record(st)
                losses[i - 1] = None
            if i < n:  # forward of micro-batch i after forward i - 1 (the chunked LM-head CE accumulates dW there)
                st = s[i % 2]
                with torch.cuda.stream(st):
                    if fdone is not None:
                        st.wait_event(fdone)
                    losses[i] = fwd(i)
                    fdone = torch.cuda.Event()
                    fdone.record(st)
        for st in s:
            main.wait_stream(st)

    def graphed(body):
        ops.refresh_weight_transposes()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            body()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            body()
        torch.cuda.synchronize()
        return g.replay

    res = {}
    grads = {}
    params = list(model.parameters())
    check = params[:8] + params[-2:]
    orders = {"serial": serial, "overlap": overlapped}
    if args.graph:
        orders = {k: graphed(v) for k, v in orders.items()}
    for name, fn in (("serial", orders["serial"]), ("overlap", orders["overlap"]), ("serial2", orders["serial"]),
                     ("overlap2", orders["overlap"])):
        zero()
        fn()  # warm-up (and the gradients of one pass, for the comparison)
        torch.cuda.synchronize()
        grads[name] = [p.grad.float().clone() for p in check]
        ts = []
        for _ in range(args.reps):
            zero()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        res[name] = round(1e3 * min(ts) / n, 3)
    diff = max(float((a - b).abs().max()) for a, b in zip(grads["serial"], grads["overlap"]))
    print(json.dumps({"ms_per_microbatch": res, "max_grad_diff": diff, "layers": args.layers, "n": n,
                      "graph": args.graph}), flush=True)


if __name__ == "__main__":
    main()
