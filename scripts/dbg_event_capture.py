"""Debug: the two-stream micro-batch pipeline's event pattern under graph capture, with plain tensor ops.

  python scripts/dbg_event_capture.py [--keep-events] [--relay] [--k 4]

Forward i (stream i % 2) waits an event recorded after forward i - 1; backward i - 1 (issued before forward i, on
forward i - 1's stream) waits an event recorded after backward i - 2. --keep-events holds every event object
until the capture has ended (otherwise each is destroyed once replaced, inside the capture). --relay carries
each dependency through a relay stream instead (wait_stream only: every event is waited right after it is
recorded, before its stream captures anything else).
"""
import argparse
import json

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--keep-events", action="store_true")
    ap.add_argument("--relay", action="store_true")
    ap.add_argument("--prealloc", action="store_true", help="no allocation inside the capture (in-place ops)")
    ap.add_argument("--origin-slot", action="store_true", help="pipeline slot 0 = the capture stream itself")
    ap.add_argument("--sibling", action="store_true", help="minimal: forked B waits forked A, nothing else")
    args = ap.parse_args()
    x = torch.randn(1 << 20, device="cuda")
    acc = torch.zeros_like(x)
    streams = (torch.cuda.Stream(), torch.cuda.Stream())
    keep = []
    bufs = [torch.empty_like(x) for _ in range(args.k)]
    tmp = [torch.empty_like(x) for _ in range(2)]
    relay_f, relay_b = torch.cuda.Stream(), torch.cuda.Stream()

    def body_relay():
        cur = torch.cuda.current_stream()
        for st in streams + (relay_f, relay_b):
            st.wait_stream(cur)
        acts = [None] * args.k
        for i in range(args.k + 1):
            if i >= 1:
                st = streams[(i - 1) % 2]
                with torch.cuda.stream(st):
                    if i >= 2:
                        st.wait_stream(relay_b)
                    acc.add_(acts[i - 1] * 0.5)
                relay_b.wait_stream(st)
                acts[i - 1] = None
            if i < args.k:
                st = streams[i % 2]
                with torch.cuda.stream(st):
                    if i >= 1:
                        st.wait_stream(relay_f)
                    acts[i] = (x * (i + 1)).sin()
                relay_f.wait_stream(st)
        for st in streams + (relay_f, relay_b):
            cur.wait_stream(st)

    def body_sibling():
        cur = torch.cuda.current_stream()
        a, b = streams
        a.wait_stream(cur)
        b.wait_stream(cur)
        with torch.cuda.stream(a):
            torch.mul(x, 2, out=tmp[0])
        b.wait_stream(a)
        with torch.cuda.stream(b):
            torch.add(tmp[0], 1, out=tmp[1])
        cur.wait_stream(a)
        cur.wait_stream(b)

    def body():
        nonlocal streams
        cur = torch.cuda.current_stream()
        if args.origin_slot:
            streams = (cur, streams[1])
        for st in streams:
            if st is not cur:
                st.wait_stream(cur)
        acts = [None] * args.k
        bwd_done = fwd_done = None
        for i in range(args.k + 1):
            if i >= 1:
                st = streams[(i - 1) % 2]
                with torch.cuda.stream(st):
                    if bwd_done is not None:
                        st.wait_event(bwd_done)
                    if args.prealloc:
                        acc.add_(acts[i - 1], alpha=0.5)
                    else:
                        acc.add_(acts[i - 1] * 0.5)
                    bwd_done = torch.cuda.Event()
                    bwd_done.record(st)
                    if args.keep_events:
                        keep.append(bwd_done)
                acts[i - 1] = None
            if i < args.k:
                st = streams[i % 2]
                with torch.cuda.stream(st):
                    if fwd_done is not None:
                        st.wait_event(fwd_done)
                    if args.prealloc:
                        torch.mul(x, i + 1, out=bufs[i])
                        bufs[i].sin_()
                        acts[i] = bufs[i]
                    else:
                        acts[i] = (x * (i + 1)).sin()
                    fwd_done = torch.cuda.Event()
                    fwd_done.record(st)
                    if args.keep_events:
                        keep.append(fwd_done)
        for st in streams:
            if st is not cur:
                cur.wait_stream(st)

    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        (body_sibling if args.sibling else body_relay if args.relay else body)()
    print(json.dumps({"phase": "captured"}), flush=True)
    acc.zero_()
    g.replay()
    torch.cuda.synchronize()
    ref = x * 0 if args.sibling else sum((x * (i + 1)).sin() * 0.5 for i in range(args.k))
    print(json.dumps({"phase": "replayed", "keep_events": args.keep_events, "relay": args.relay, "prealloc": args.prealloc, "k": args.k,
                      "max_err": float((acc - ref).abs().max())}), flush=True)


if __name__ == "__main__":
    main()
