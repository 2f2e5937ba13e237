"""The hot path as a drop-in under pipeline parallelism: pp = 2 stages sharing this GPU (gloo, host-staged
P2P; RCCL refuses two ranks on one device). Each stage owns the reference's split of the model
(ref picotron/pipeline_parallel/pipeline_parallel.py:9-42: embedding on the first stage, a contiguous run
of decoder layers each, final_norm + final_proj on the last; layers called as `layer(x, position_ids=...)`),
and the schedule's forward send / backward recv (ref :44-142, here one micro-batch, all-forward-all-
backward) is restated test-side: the wrapper is a caller, not rebuilt. Every stage's gradients must
match the unsplit model's on the same weights and tokens.
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


def _worker(rank, world, port):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.model import LlamaConfig, build_llama
    pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=world, dp_size=1)
    bf = torch.bfloat16
    cfg = LlamaConfig(hidden_size=256, intermediate_size=512, num_attention_heads=4, num_key_value_heads=2,
                      num_hidden_layers=4, vocab_size=512, max_position_embeddings=128)
    torch.manual_seed(42)
    full = build_llama(cfg, device="cuda", dtype=bf)
    torch.manual_seed(42)
    stage = build_llama(cfg, device="cuda", dtype=bf)
    g = torch.Generator(device="cpu").manual_seed(5)
    with torch.no_grad():
        full.final_proj.weight.copy_((torch.randn(full.final_proj.weight.shape, generator=g) * 0.02).to(bf))
        stage.final_proj.weight.copy_(full.final_proj.weight)
    toks = torch.randint(0, cfg.vocab_size, (2, 129), generator=g).to("cuda")
    lo, hi = rank * cfg.num_hidden_layers // world, (rank + 1) * cfg.num_hidden_layers // world
    first, last = rank == 0, rank == world - 1
    B, S, H = 2, 128, cfg.hidden_size

    def send(t, dst):
        dist.send(t.detach().float().cpu().contiguous(), dst)

    def recv(src):
        buf = torch.empty((B, S, H), dtype=torch.float32)
        dist.recv(buf, src)
        return buf.to("cuda").to(bf)

    # forward: this stage's share of the model
    if first:
        x_in = None
        x = stage.embedding(toks[:, :-1])
    else:
        x_in = recv(rank - 1).requires_grad_(True)
        x = x_in
    for i in range(lo, hi):
        x = stage.decoder_layers[i](x, position_ids=None)
    if last:
        logits = stage.final_proj(stage.final_norm(x))
        loss = torch.nn.functional.cross_entropy(logits.reshape(-1, cfg.vocab_size).float(), toks[:, 1:].reshape(-1))
        loss.backward()
    else:
        send(x, rank + 1)
        torch.autograd.backward(x, recv(rank + 1))
    if not first:
        send(x_in.grad, rank - 1)
    # the unsplit model
    logits_f = full(toks[:, :-1])
    torch.nn.functional.cross_entropy(logits_f.reshape(-1, cfg.vocab_size).float(), toks[:, 1:].reshape(-1)).backward()
    torch.cuda.synchronize()

    def rel(a, b):
        a, b = a.double(), b.double()
        return float((a - b).norm() / b.norm().clamp_min(1e-30))

    mine = {f"decoder_layers.{i}." for i in range(lo, hi)}
    errs = {}
    for (n, pf), (_, ps) in zip(full.named_parameters(), stage.named_parameters()):
        owned = any(n.startswith(p) for p in mine) or (first and n.startswith("embedding.")) or \
            (last and n.startswith(("final_norm.", "final_proj.")))
        if owned:
            errs[n] = rel(ps.grad, pf.grad)
        else:
            assert ps.grad is None, n  # other stages' parameters see no gradient here
    assert errs
    bad = {k: v for k, v in errs.items() if not v < 2e-2}
    dist.barrier()
    dist.destroy_process_group()
    if bad:
        raise AssertionError(f"stage {rank}: {bad}")


def test_pipeline_parallel_drop_in():
    mp.start_processes(_worker, args=(2, _free_port()), nprocs=2, join=True, start_method="spawn")
