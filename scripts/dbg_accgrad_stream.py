"""Which parameters' gradients reach an AccumulateGrad node through autograd in the pipelined micro-batch graph
(torch's "AccumulateGrad node's stream does not match ..." warning in
test_wgrad_pairs_match_unpaired[4-False-True]). The test's model and step (4 micro-batches, no DP, pipelined graph):
every parameter gets a tensor hook (called with the incoming gradient; None ones are skipped) that records the parameter, the
micro-batch announced to wgrad_pair and the current stream; warnings are recorded per step."""
import os
import sys
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from picotron_amd import wgrad_pair as WP
    from picotron_amd.data import SyntheticDataLoader
    from picotron_amd.model import LlamaConfig, build_llama
    from picotron_amd.train import PipelinedMicroBatchGraph, train_step
    cfg = LlamaConfig(hidden_size=1024, intermediate_size=2048, num_attention_heads=16, num_key_value_heads=16,
                      num_hidden_layers=2, vocab_size=512, max_position_embeddings=128)
    n = 4
    torch.manual_seed(7)
    m = build_llama(cfg, "cuda", torch.bfloat16)
    with torch.no_grad():
        m.final_proj.weight.normal_(0, 0.02, generator=torch.Generator("cuda").manual_seed(1))
    loader = SyntheticDataLoader(2, 128, n, cfg.vocab_size, seed=5, num_batches=n, device="cuda")
    for p in m.parameters():
        p.grad = torch.zeros_like(p)
    seen = []
    for name, p in m.named_parameters():
        def hook(g, name=name):
            if g is not None:
                seen.append((name, WP._CTX["i"], torch.cuda.current_stream().stream_id, tuple(g.shape)))
            return g
        p.register_hook(hook)

    def zero():
        for p in m.parameters():
            if p.grad is not None:
                p.grad.zero_()
    g = PipelinedMicroBatchGraph(m, n, zero)
    for step in range(2):
        seen.clear()
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            zero()
            train_step(m, loader, "cuda", graphs=g)
            torch.cuda.synchronize()
        msgs = sorted({str(x.message)[:90] for x in w})
        print(f"step {step}: {len(w)} warnings {msgs}")
        names = {}
        for nm, i, sid, shp in seen:
            names.setdefault(nm, []).append((i, sid))
        print(f"step {step}: {len(names)} parameters received a defined gradient through autograd:")
        for nm, v in names.items():
            print(f"   {nm}: (micro-batch, stream id) {v[:8]}")


if __name__ == "__main__":
    main()
