"""One process, one set-up: does the two-stream pipelined micro-batch graph hand any gradient to autograd's
AccumulateGrad across streams? Prints the number of torch "AccumulateGrad node's stream does not match" warnings
over two steps (capture + replay). TORCH_WARN_ONCE is per process, hence one set-up per process
(tests/test_model_gpu.py::test_pipelined_graph_no_accumulategrad_stream_sync runs the three).

  python scripts/accgrad_warn_probe.py {bench|zeros|dp}
    bench — no gradients before the first step (the fused producers create them), as bench.py;
    zeros — every p.grad pre-allocated separately (torch.zeros_like per parameter), as the wgrad-pair test;
    dp    — DataParallelBucket over RCCL at W = 1.
"""
import os
import sys
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    setup = sys.argv[1]
    import torch.distributed as dist
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.data import SyntheticDataLoader
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    from picotron_amd.model import LlamaConfig, build_llama
    from picotron_amd.train import PipelinedMicroBatchGraph, train_step
    if setup == "dp":
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("PROBE_PORT", "29733"), RANK="0",
                          WORLD_SIZE="1", LOCAL_RANK="0")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        pgm.setup_process_group_manager(1, 1, 1, 1)
    cfg = LlamaConfig(hidden_size=1024, intermediate_size=2048, num_attention_heads=16, num_key_value_heads=16,
                      num_hidden_layers=2, vocab_size=512, max_position_embeddings=128)
    n = 4
    torch.manual_seed(7)
    m = build_llama(cfg, "cuda", torch.bfloat16)
    model = DataParallelBucket(m, bucket_cap_mb=1) if setup == "dp" else m
    loader = SyntheticDataLoader(2, 128, n, cfg.vocab_size, seed=5, num_batches=n, device="cuda")
    if setup == "zeros":
        for p in m.parameters():
            p.grad = torch.zeros_like(p)
    elif setup == "bench":
        train_step(model, loader, "cuda", graphs=None)

    def zero():
        for p in m.parameters():
            if p.grad is not None:
                p.grad.zero_()
        if setup == "dp":
            model.bucket_manager.reset()
    g = PipelinedMicroBatchGraph(model, n, zero)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        for _ in range(2):
            zero()
            train_step(model, loader, "cuda", graphs=g)
        torch.cuda.synchronize()
    hits = [x for x in w if "AccumulateGrad node's stream" in str(x.message)]
    print(f"ACCGRAD_STREAM_WARNINGS {setup} {len(hits)}", flush=True)
    if setup == "dp":
        pgm.process_group_manager = None
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
