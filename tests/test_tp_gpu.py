"""The hot path under tensor parallelism: tp = 2 ranks sharing this GPU (gloo; RCCL refuses two ranks on
one device) run picotron_amd.tensor_parallel.apply_tensor_parallel (ref picotron/tensor_parallel/
tensor_parallel.py:9-51: q/k/v/up/gate column-parallel, out/down row-parallel, vocab-parallel embedding,
gathered LM head) on a model built with the same weights as an unsharded one (shard_weights=True), with
the fused q|k|v + RoPE + attention and gate|up + SwiGLU paths on the local shards (one f region each) and
with the unfused per-projection path (PICO_UNFUSED=1). Forward logits, loss and every gradient must match
the unsharded model.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, unfused):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ["PICO_UNFUSED"] = "1" if unfused else "0"
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.model import LlamaConfig, build_llama
    pgm.setup_process_group_manager(tp_size=world, cp_size=1, pp_size=1, dp_size=1)
    bf = torch.bfloat16
    cfg = LlamaConfig(hidden_size=256, intermediate_size=512, num_attention_heads=4, num_key_value_heads=2,
                      num_hidden_layers=2, vocab_size=512, max_position_embeddings=128)
    # unsharded model (built as at tp = 1) and the tp model (built under tp = world: local head counts)
    tp_size = pgm.tp_world_size
    pgm.tp_world_size = lambda: 1
    torch.manual_seed(42)
    full = build_llama(cfg, device="cuda", dtype=bf)
    pgm.tp_world_size = tp_size
    torch.manual_seed(42)
    tpm = build_llama(cfg, device="cuda", dtype=bf)
    g = torch.Generator(device="cpu").manual_seed(3)
    with torch.no_grad():
        full.final_proj.weight.copy_((torch.randn(full.final_proj.weight.shape, generator=g) * 0.02).to(bf))
        for pf, pt in zip(full.parameters(), tpm.parameters()):
            pt.copy_(pf)
    from picotron_amd.tensor_parallel.tensor_parallel import apply_tensor_parallel
    apply_tensor_parallel(tpm, shard_weights=True)
    if os.environ.get("PICO_UNFUSED", "0") != "1":  # the fused paths take the column-parallel shards
        assert tpm.decoder_layers[0].attention._fusable() == "tp"
    toks = torch.randint(0, cfg.vocab_size, (2, 129), generator=g).to("cuda")

    def run(m):
        logits = m(toks[:, :-1])
        loss = torch.nn.functional.cross_entropy(logits.reshape(-1, cfg.vocab_size).float(), toks[:, 1:].reshape(-1))
        loss.backward()
        return logits.float(), float(loss)

    lf_, loss_f = run(full)
    lt_, loss_t = run(tpm)
    torch.cuda.synchronize()

    def rel(a, b):
        a, b = a.double(), b.double()
        return float((a - b).norm() / b.norm().clamp_min(1e-30))

    errs = {"logits": rel(lt_, lf_), "loss": abs(loss_t - loss_f)}
    for (nf, pf), (nt, pt) in zip(full.named_parameters(), tpm.named_parameters()):
        gf = pf.grad
        shape = tuple(pt.shape)
        if shape != tuple(pf.shape):  # sharded: column (rows) or row (columns) parallel
            if shape[0] != pf.shape[0]:
                n = shape[0]
                gf = gf[rank * n:(rank + 1) * n]
            else:
                n = shape[1]
                gf = gf[:, rank * n:(rank + 1) * n]
        errs["grad:" + nt] = rel(pt.grad, gf)
    bad = {k: v for k, v in errs.items() if not v < (2e-2 if k != "loss" else 5e-3)}
    dist.barrier()
    dist.destroy_process_group()
    if bad:
        raise AssertionError(f"rank {rank}: {bad}")


@pytest.mark.parametrize("unfused", [False, True])
def test_tensor_parallel_drop_in(unfused):
    mp.start_processes(_worker, args=(2, _free_port(), unfused), nprocs=2, join=True, start_method="spawn")
