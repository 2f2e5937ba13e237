"""Debug: the pipelined micro-batch graph's event pattern with a third stream for the weight-gradient GEMMs,
under graph capture, with plain tensor ops.

  python scripts/dbg_wstream_capture.py [--k 8]

Slots as in PipelinedMicroBatchGraph: slot 0 = the capture stream, slot 1 forked; forward i on slot i % 2 after
forward i - 1, backward i - 1 on its forward's slot after backward i - 2. Forward i writes its half of a pair
buffer set ("x^T", sets alternating per pair), backward i its half of the one "dy" set; the second backward of
a pair hands the pair's product to stream W (W waits an event recorded on slot 1), which adds it into `acc`
in pair order and records an event per pair. A writer on slot 0 (the capture stream) waits for the W event of
the last reader of the half it overwrites; a writer on slot 1 waits for nothing from W directly (it follows
slot 0's writer of the same set through the fwd / bwd event chain). The graph's end joins W and slot 1.
"""
import argparse
import json

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--n", type=int, default=1 << 20)
    args = ap.parse_args()
    k, n = args.k, args.n
    dev = "cuda"
    x = torch.randn(n, device=dev)
    acc = torch.zeros(n, device=dev)
    xt = [[torch.empty(n, device=dev) for _ in range(2)] for _ in range(2)]  # [set][half]
    dy = [torch.empty(n, device=dev) for _ in range(2)]  # [half]
    s1 = torch.cuda.Stream()
    W = torch.cuda.Stream()
    xt_reader = {}  # set -> W event of the pair that last read it
    dy_reader = [None]

    def body():
        cur = torch.cuda.current_stream()
        streams = (cur, s1)
        s1.wait_stream(cur)
        W.wait_stream(cur)
        bwd_done = fwd_done = None
        for i in range(k + 1):
            if i >= 1:
                j = i - 1
                st = streams[j % 2]
                with torch.cuda.stream(st):
                    if bwd_done is not None:
                        st.wait_event(bwd_done)
                    if st is cur and dy_reader[0] is not None:
                        st.wait_event(dy_reader[0])
                    torch.mul(xt[(j // 2) % 2][j % 2], 0.5 + j, out=dy[j % 2])  # "dy" of micro-batch j
                    if j % 2 == 1:  # the pair's product on W
                        ev = torch.cuda.Event()
                        ev.record(st)
                        W.wait_event(ev)
                        with torch.cuda.stream(W):
                            s = (j // 2) % 2
                            acc.add_(dy[0] * xt[s][0] + dy[1] * xt[s][1])
                            done = torch.cuda.Event()
                            done.record(W)
                        xt_reader[s] = done
                        dy_reader[0] = done
                    bwd_done = torch.cuda.Event()
                    bwd_done.record(st)
            if i < k:
                st = streams[i % 2]
                with torch.cuda.stream(st):
                    if fwd_done is not None:
                        st.wait_event(fwd_done)
                    s = (i // 2) % 2
                    if st is cur and xt_reader.get(s) is not None:
                        st.wait_event(xt_reader[s])
                    torch.mul(x, i + 1, out=xt[s][i % 2])
                    xt[s][i % 2].sin_()
                    fwd_done = torch.cuda.Event()
                    fwd_done.record(st)
        cur.wait_stream(s1)
        cur.wait_stream(W)

    ref = torch.zeros_like(acc)
    for p in range(k // 2):
        a, b = 2 * p, 2 * p + 1
        xa, xb = (x * (a + 1)).sin(), (x * (b + 1)).sin()
        ref += xa * (0.5 + a) * xa + xb * (0.5 + b) * xb
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    print(json.dumps({"phase": "captured"}), flush=True)
    errs = []
    for _ in range(3):
        acc.zero_()
        g.replay()
        torch.cuda.synchronize()
        errs.append(float((acc - ref).abs().max() / ref.abs().max()))
    print(json.dumps({"phase": "replayed", "k": k, "rel_err": errs}), flush=True)
    assert max(errs) < 1e-5, errs


if __name__ == "__main__":
    main()
