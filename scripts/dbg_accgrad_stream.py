"""Which parameters' gradients reach their AccumulateGrad node through autograd (a DEFINED gradient) in the
pipelined micro-batch graph — VERDICT r04 item 5: torch's "AccumulateGrad node's stream does not match ..." warning
in test_wgrad_pairs_match_unpaired[4-False-True].

Probed with pre-hooks on the AccumulateGrad NODES (tensor hooks would count as parameter hooks and switch the
fused weight-gradient paths off). Three set-ups, two steps each (capture + replay), 4 micro-batches:
  test  — the test's: every p.grad pre-allocated separately (torch.zeros_like per parameter);
  bench — bench.py's: no gradients before the first step (the fused producers create them, stacked weights'
          gradients as row blocks of one buffer), then zero_grad(set_to_none=False);
  dp    — DataParallelBucket (RCCL, W = 1): fp32 main_grad views of the bucket buffers.
"""
import os
import sys
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(setup):
    import torch.distributed as dist
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.data import SyntheticDataLoader
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    from picotron_amd.model import LlamaConfig, build_llama
    from picotron_amd.train import PipelinedMicroBatchGraph, train_step
    cfg = LlamaConfig(hidden_size=1024, intermediate_size=2048, num_attention_heads=16, num_key_value_heads=16,
                      num_hidden_layers=2, vocab_size=512, max_position_embeddings=128)
    n = 4
    torch.manual_seed(7)
    m = build_llama(cfg, "cuda", torch.bfloat16)
    with torch.no_grad():
        m.final_proj.weight.normal_(0, 0.02, generator=torch.Generator("cuda").manual_seed(1))
    model = m
    if setup == "dp":
        model = DataParallelBucket(m, bucket_cap_mb=1)
    loader = SyntheticDataLoader(2, 128, n, cfg.vocab_size, seed=5, num_batches=n, device="cuda")
    if setup == "test":
        for p in m.parameters():
            p.grad = torch.zeros_like(p)
    elif setup == "bench":  # one eager step creates the gradient buffers the way the fused producers lay them out
        train_step(model, loader, "cuda", graphs=None)
    seen = {}
    nodes = []
    for name, p in m.named_parameters():
        node = p.view_as(p).grad_fn.next_functions[0][0]  # the parameter's AccumulateGrad node (kept alive here)
        nodes.append(node)

        def pre(grads, name=name):
            if grads and grads[0] is not None:
                seen[name] = seen.get(name, 0) + 1
        node.register_prehook(pre)

    def zero():
        for p in m.parameters():
            if p.grad is not None:
                p.grad.zero_()
        if setup == "dp":
            model.bucket_manager.reset()
    g = PipelinedMicroBatchGraph(model, n, zero)
    for step in range(2):
        seen.clear()
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            zero()
            train_step(model, loader, "cuda", graphs=g)
            torch.cuda.synchronize()
        print(f"[{setup}] step {step}: {len(w)} warnings; defined gradients into AccumulateGrad "
              f"(python runs only while capturing / eager): {dict(sorted(seen.items())) or 'none'}", flush=True)
    del nodes


def main():
    import torch.distributed as dist
    from picotron_amd import process_group_manager as pgm
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29731", RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    pgm.setup_process_group_manager(1, 1, 1, 1)
    for setup in sys.argv[1:] or ["test", "bench", "dp"]:
        run(setup)
    pgm.process_group_manager = None
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
