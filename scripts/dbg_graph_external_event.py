"""Probe: does an event recorded inside a captured HIP graph (torch.cuda.Event(external=True)) fire at its place in
the replay, so that work outside the graph can wait for the middle of it? A graph of [fill a, long matmul chain]
with the event after the fill; after replay a side stream waits on the event and copies a. If the copy finishes long
before the graph, the event fired mid-graph."""
import time

import torch


def main():
    dev = torch.device("cuda", 0)
    a = torch.zeros(1 << 20, device=dev)
    x = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    y = torch.empty_like(x)
    ev = torch.cuda.Event(external=True)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up
        a.fill_(1.0)
        for _ in range(4):
            torch.mm(x, x, out=y)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        a.fill_(2.0)
        ev.record()
        for _ in range(200):
            torch.mm(x, x, out=y)
    torch.cuda.synchronize()
    side = torch.cuda.Stream(device=dev)
    b = torch.empty_like(a)
    t_side, t_main = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = torch.cuda.Event(enable_timing=True)
    t0.record()
    g.replay()
    side.wait_event(ev)
    with torch.cuda.stream(side):
        b.copy_(a)
        t_side.record()
    t_main.record()
    torch.cuda.synchronize()
    print({"side_done_ms": t0.elapsed_time(t_side), "graph_done_ms": t0.elapsed_time(t_main),
           "b_value": float(b[0]), "mid_graph": t0.elapsed_time(t_side) < 0.5 * t0.elapsed_time(t_main)})


if __name__ == "__main__":
    main()
