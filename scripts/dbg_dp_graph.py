"""Debug: trace DP bucket readiness and grad hooks through MicroBatchGraph capture/replay (W = 1)."""
import os
import sys
import traceback

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import process_group_manager as pgm  # noqa: E402
from picotron_amd.data import SyntheticDataLoader  # noqa: E402
from picotron_amd.data_parallel import bucket as B  # noqa: E402
from picotron_amd.data_parallel.data_parallel import DataParallelBucket  # noqa: E402
from picotron_amd.model import LlamaConfig, build_llama  # noqa: E402
from picotron_amd.train import MicroBatchGraph, train_step  # noqa: E402


def main():
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533", RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    pgm.setup_process_group_manager(1, 1, 1, 1)
    cfg = LlamaConfig(hidden_size=256, intermediate_size=512, num_attention_heads=4, num_key_value_heads=2,
                      num_hidden_layers=2, vocab_size=512, max_position_embeddings=128)
    m = build_llama(cfg, "cuda", torch.bfloat16)
    names = {id(p): n for n, p in m.named_parameters()}
    orig = B.Bucket.mark_param_as_ready

    def mark(self, param, prescaled=False):
        print("ready", names[id(param)], flush=True)
        return orig(self, param, prescaled)
    B.Bucket.mark_param_as_ready = mark
    ddp = DataParallelBucket(m, bucket_cap_mb=1)
    for n, p in m.named_parameters():
        p.register_post_accumulate_grad_hook(
            lambda q, n=n: print("hook", n, q.grad is None, getattr(q, "_pico_fused_pending", None), flush=True))
    opt = torch.optim.AdamW(ddp.parameters(), lr=1e-3)
    loader = SyntheticDataLoader(2, 128, 3, cfg.vocab_size, seed=5, num_batches=3, device="cuda")

    def zero():
        for p in m.parameters():
            if p.grad is not None:
                p.grad.zero_()
        ddp.bucket_manager.reset()
    g = MicroBatchGraph(ddp, 3, zero)
    for step in range(2):
        print("=== step", step, flush=True)
        opt.zero_grad(set_to_none=False)
        try:
            train_step(ddp, loader, "cuda", graphs=g)
        except Exception:  # noqa: BLE001
            traceback.print_exc()
            break
        opt.step()
        ddp.reset()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
