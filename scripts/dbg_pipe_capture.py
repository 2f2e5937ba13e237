"""Debug: capture PipelinedMicroBatchGraph on a 2-layer model (the graph-replay test's geometry) and replay it
once; prints one JSON line. Environment knobs select the variant (PICO_WGRAD_CONC=none: no side streams).

  python scripts/dbg_pipe_capture.py [--k 3] [--serial-streams]

--serial-streams: both pipeline slots on ONE stream (the pipelined code path, no second stream).
--on-current: both slots on the stream the body is called on (the capture stream itself: nothing forked).
--fork-plain: no pipeline: each micro-batch's forward + backward (train._micro_batch) on one stream forked
from the capture stream, no events (is a backward on a forked capture stream the problem?).
--fork-fwd-only: the forwards on the forked stream, the backwards on the capture stream.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--serial-streams", action="store_true")
    ap.add_argument("--on-current", action="store_true")
    ap.add_argument("--fork-plain", action="store_true")
    ap.add_argument("--fork-fwd-only", action="store_true")
    args = ap.parse_args()
    from picotron_amd import _lib
    from picotron_amd.model import LlamaConfig, build_llama
    from picotron_amd.train import PipelinedMicroBatchGraph
    _lib.load()
    cfg = LlamaConfig(hidden_size=256, intermediate_size=512, num_attention_heads=4, num_key_value_heads=4,
                      num_hidden_layers=2, vocab_size=1024, max_position_embeddings=128)
    torch.manual_seed(7)
    m = build_llama(cfg, "cuda", torch.bfloat16)
    for p in m.parameters():
        p.grad = torch.zeros_like(p)

    def zero():
        for p in m.parameters():
            p.grad.zero_()

    g = PipelinedMicroBatchGraph(m, args.k, zero)
    if args.serial_streams:
        s = torch.cuda.Stream()
        g.streams = (s, s)  # (slot 0 is always the calling stream now: this only affects slot 1)
    if args.on_current:
        body = g._body

        def on_current(inp, tgt):
            cur = torch.cuda.current_stream()
            g.streams = (cur, cur)
            body(inp, tgt)
        g.streams = (torch.cuda.current_stream(),) * 2
        g._body = on_current
    if args.fork_plain or args.fork_fwd_only:
        from picotron_amd import train

        def plain(inp, tgt):
            cur = torch.cuda.current_stream()
            s = torch.cuda.Stream()
            s.wait_stream(cur)
            for i in range(inp.shape[0]):
                if args.fork_plain:
                    with torch.cuda.stream(s):
                        train._micro_batch(m, inp[i], tgt[i], args.k, g.loss_acc)
                else:
                    with torch.cuda.stream(s):
                        loss, folded = train._forward_loss(m, inp[i], tgt[i], args.k, g.loss_acc)
                    cur.wait_stream(s)
                    loss.backward()
                    s.wait_stream(cur)
            cur.wait_stream(s)
        g._body = plain
    gen = torch.Generator().manual_seed(1)
    batches = [(torch.randint(0, cfg.vocab_size, (2, 128), generator=gen).cuda(),
                torch.randint(0, cfg.vocab_size, (2, 128), generator=gen).cuda()) for _ in range(args.k)]
    print("capturing", flush=True)
    g.run(batches)
    torch.cuda.synchronize()
    print("replayed", flush=True)
    loss = float(g.take_loss())
    print(json.dumps({"ok": True, "k": args.k, "serial_streams": args.serial_streams,
                      "conc": os.getenv("PICO_WGRAD_CONC", "gu,lm"), "loss": loss}), flush=True)


if __name__ == "__main__":
    main()
