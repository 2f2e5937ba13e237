"""Multi-process (world size 2, gloo, CPU) tests of the data-parallel host path:
picotron_amd's DataParallelBucket / BucketManager with the oracle's CPU device-op table, on the
oracle Llama, against the reference's own DataParallelBucket run (tests/golden/dp_w2_tiny.safetensors).
"""
import os
import socket
from types import SimpleNamespace

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, ROOT

TINY_DP = dict(hidden_size=128, intermediate_size=256, num_attention_heads=2, num_key_value_heads=1,
               num_hidden_layers=2, vocab_size=256, max_position_embeddings=64, rms_norm_eps=1e-5, rope_theta=10000.0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, outdir):
    import sys
    sys.path.insert(0, ROOT)
    torch.set_num_threads(1)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from safetensors.torch import load_file, save_file
    from oracle import hotpath as H
    from oracle import model as OM
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.data import synth_tokens
    from picotron_amd.data_parallel import bucket as B
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=1, dp_size=world)
    B.set_kernels(H.CpuBucketKernels())
    cfg = SimpleNamespace(**TINY_DP)
    model = OM.Llama(cfg)
    gold = load_file(os.path.join(GOLDEN, "dp_w2_tiny.safetensors"))
    model.load_state_dict({k[5:]: v for k, v in gold.items() if k.startswith("init.")}, strict=True)
    ddp = DataParallelBucket(model, bucket_cap_mb=0.05)
    out = {}
    if mode == "golden":
        gen = torch.Generator().manual_seed(7 + rank)
        ga = 3
        for i in range(ga):
            toks = synth_tokens(2, cfg.max_position_embeddings + 1, cfg.vocab_size, gen, "arith")
            ddp.require_backward_grad_sync = i == ga - 1
            logits = ddp(input_ids=toks[:, :-1])
            loss = torch.nn.functional.cross_entropy(logits.reshape(-1, cfg.vocab_size), toks[:, 1:].reshape(-1)) / ga
            loss.backward()
        for n, p in model.named_parameters():
            out["main_grad." + n] = p.main_grad.clone()
            out["grad." + n] = p.grad.clone()
    elif mode == "semantics":
        gen = torch.Generator().manual_seed(11 + rank)
        toks = synth_tokens(2, cfg.max_position_embeddings + 1, cfg.vocab_size, gen, "arith")
        # no_sync: accumulate only, no bucket fires, no .grad handed out
        with ddp.no_sync():
            ddp(input_ids=toks[:, :-1]).float().mean().backward()
        assert all(b.handle is None for b in ddp.bucket_manager.buckets)
        assert all(p.grad is None for p in model.parameters())
        local = {n: p.main_grad.clone() for n, p in model.named_parameters()}
        # syncing backward: every bucket fires once; main_grad = (local + g) / W summed over ranks
        ddp(input_ids=toks[:, :-1]).float().mean().backward()
        assert all(b.handle is not None for b in ddp.bucket_manager.buckets)
        for n, p in model.named_parameters():
            out["main_grad." + n] = p.main_grad.clone()
            out["local." + n] = local[n]
            assert torch.equal(p.grad, p.main_grad.to(p.dtype))
        # reset zeroes every bucket and clears readiness
        ddp.reset()
        assert all(float(b.grad_data.abs().sum()) == 0 and not b.params_with_grad_ready
                   for b in ddp.bucket_manager.buckets)
        assert all(float(p.main_grad.abs().sum()) == 0 for p in model.parameters())
    save_file({k: v.contiguous() for k, v in out.items()}, os.path.join(outdir, f"rank{rank}.safetensors"))
    dist.barrier()
    dist.destroy_process_group()


def _run(mode, tmp_path):
    mp.start_processes(_worker, args=(2, _free_port(), mode, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    from safetensors.torch import load_file
    return [load_file(os.path.join(tmp_path, f"rank{r}.safetensors")) for r in range(2)]


def test_dp_bucket_matches_reference_golden(tmp_path):
    from safetensors.torch import load_file
    gold = load_file(os.path.join(GOLDEN, "dp_w2_tiny.safetensors"))
    r0, r1 = _run("golden", tmp_path)
    n = 0
    for k, v in gold.items():
        if not k.startswith("main_grad."):
            continue
        name = k[len("main_grad."):]
        # both ranks hold the same averaged gradient
        assert torch.equal(r0[k], r1[k]), name
        assert torch.allclose(r0[k], v, rtol=1e-5, atol=1e-7), (name, float((r0[k] - v).abs().max()))
        assert torch.equal(r0["grad." + name], r0[k])  # fp32 params: .grad == main_grad
        n += 1
    assert n == 21


def test_dp_sync_semantics(tmp_path):
    r0, r1 = _run("semantics", tmp_path)
    for k in r0:
        if k.startswith("main_grad."):
            name = k[len("main_grad."):]
            assert torch.equal(r0[k], r1[k]), name
            assert float(r0["local." + name].abs().sum()) > 0


def _fused_worker(rank, world, port, outdir):
    """A producer that accumulates into main_grad itself and calls param._pico_wgrad_ready() (as the fused
    wgrad GEMMs do), next to a plain parameter on the hook path, with persistent .grad buffers
    (set_to_none=False, as under HIP-graph replay): each param is marked ready exactly once per syncing
    backward and main_grad holds the micro-batch sum."""
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import hotpath as H
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.data_parallel import bucket as B
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=1, dp_size=world)
    B.set_kernels(H.CpuBucketKernels())

    class FusedMul(torch.autograd.Function):  # y = x * w; dw goes straight into w.main_grad
        @staticmethod
        def forward(ctx, x, w):
            ctx.save_for_backward(x)
            ctx.w = w
            return x * w

        @staticmethod
        def backward(ctx, g):
            (x,) = ctx.saved_tensors
            w = ctx.w
            sync, W = w._pico_wgrad_sync()
            w.main_grad.add_((g * x).sum(0))
            if sync:
                w.main_grad.div_(W)
            w._pico_wgrad_ready()
            return g * w, None

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Parameter(torch.ones(4))
            self.b = torch.nn.Parameter(torch.full((4,), 2.0))

        def forward(self, x):
            return FusedMul.apply(x, self.a) * self.b

    m = DataParallelBucket(M(), bucket_cap_mb=1)
    for step in range(2):
        for p in m.parameters():  # persistent .grad from the second step on
            if p.grad is not None:
                p.grad.zero_()
        # step 1: one syncing micro-batch straight after the persistent .grad views were installed (the
        # eager micro-batch after graph replays): the hook sees a non-None .grad for the fused param
        xs = [torch.full((3, 4), float(i + 1 + rank)) for i in range(3 if step == 0 else 1)]
        for i, x in enumerate(xs):
            m.require_backward_grad_sync = i == len(xs) - 1
            m(x).sum().backward()
        torch.save({"a": m.module.a.main_grad.clone(), "b": m.module.b.main_grad.clone()},
                   os.path.join(outdir, f"s{step}_r{rank}.pt"))
        m.reset()
    dist.destroy_process_group()


def test_fused_ready_with_persistent_grads(tmp_path):
    world = 2
    mp.start_processes(_fused_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    # d/da sum(x a b) = sum_rows(x) * b = 3 x b; d/db = 3 x a; x = i + 1 + rank, a = 1, b = 2
    for step in range(2):
        n = 3 if step == 0 else 1
        sa = sum(3 * (i + 1 + r) * 2.0 for i in range(n) for r in range(world)) / world
        sb = sum(3 * (i + 1 + r) * 1.0 for i in range(n) for r in range(world)) / world
        for r in range(world):
            got = torch.load(tmp_path / f"s{step}_r{r}.pt", weights_only=True)
            assert torch.allclose(got["a"], torch.full((4,), sa)), (step, r, got["a"])
            assert torch.allclose(got["b"], torch.full((4,), sb)), (step, r, got["b"])


def _defer_worker(rank, world, port, outdir):
    """DataParallelBucket(defer_grad_cast=True) under a torch.optim optimizer: the deferred fp32 ->
    .grad cast is run by the bucket's global step pre-hook before torch.optim.AdamW steps, so the step equals the
    eager-cast run's bit for bit; only picotron_amd.optim.AdamW (which reads main_grad itself) skips it."""
    import sys
    sys.path.insert(0, ROOT)
    torch.set_num_threads(1)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from safetensors.torch import load_file
    from oracle import hotpath as H
    from oracle import model as OM
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.data import synth_tokens
    from picotron_amd.data_parallel import bucket as B
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=1, dp_size=world)
    B.set_kernels(H.CpuBucketKernels())
    cfg = SimpleNamespace(**TINY_DP)
    gold = load_file(os.path.join(GOLDEN, "dp_w2_tiny.safetensors"))
    init = {k[5:]: v for k, v in gold.items() if k.startswith("init.")}
    res = {}
    for defer in (False, True):
        model = OM.Llama(cfg)
        model.load_state_dict(init, strict=True)
        ddp = DataParallelBucket(model, bucket_cap_mb=0.05, defer_grad_cast=defer)
        for go in ddp.bucket_manager.grad_out_list:
            go.fill_(float("nan"))  # what an unrun cast would leave visible
        opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
        gen = torch.Generator().manual_seed(5 + rank)
        for step in range(2):
            opt.zero_grad(set_to_none=False)
            for i in range(2):
                toks = synth_tokens(2, cfg.max_position_embeddings + 1, cfg.vocab_size, gen, "arith")
                ddp.require_backward_grad_sync = i == 1
                logits = ddp(input_ids=toks[:, :-1])
                loss = torch.nn.functional.cross_entropy(logits.reshape(-1, cfg.vocab_size), toks[:, 1:].reshape(-1))
                (loss / 2).backward()
            opt.step()
            for p in model.parameters():
                assert torch.equal(p.grad, p.main_grad), "the optimizer stepped on an un-cast .grad"
                assert not getattr(p, "_pico_grad_deferred", False)
            ddp.reset()
        res[defer] = {n: p.detach().clone() for n, p in model.named_parameters()}
    for n in res[False]:
        assert torch.equal(res[False][n], res[True][n]), n
    torch.save({"ok": True}, os.path.join(outdir, f"defer_r{rank}.pt"))
    dist.destroy_process_group()


def test_deferred_cast_materialized_for_torch_optimizers(tmp_path):
    world = 2
    mp.start_processes(_defer_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        assert torch.load(tmp_path / f"defer_r{r}.pt", weights_only=True)["ok"]
