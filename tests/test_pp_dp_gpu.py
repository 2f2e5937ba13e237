"""The hot path under pipeline x data parallelism (config C1's composition, dp 2 x pp 2, here on one GPU:
four gloo ranks, host-staged P2P; RCCL refuses several ranks on one device). Each rank holds its pipeline
stage — the reference's layer split, ref picotron/pipeline_parallel/pipeline_parallel.py:8-52, restated
test-side because the PP wrapper is a hosted caller, not rebuilt — wrapped in picotron_amd's
DataParallelBucket, and runs the reference's 1F1B schedule (ref :85-145): warm-up forwards, steady-state
one-forward-one-backward through `model.backward(input, output, output_grad)` (= DataParallelBucket.backward,
ref picotron/data_parallel/data_parallel.py:90-91), `require_backward_grad_sync` forced False and set True
only for the last backward (ref :113-114, :125-126, :137-139), cool-down backwards.

Checks: (1) every stage parameter's averaged gradient (.grad bf16 and main_grad fp32) equals half the
gradient sum of the unsplit model over both DP ranks' micro-batches (within bf16 forward rounding);
(2) the two DP replicas of each stage hold identical gradients (one all-reduce, after the last backward);
(3) no bucket was marked ready twice and none was left unsynchronised (DataParallelBucket asserts).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu

GRAD_ACC, B, S = 3, 2, 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    import torch.nn as nn
    import torch.nn.functional as F
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    from picotron_amd.model import LlamaConfig, build_llama
    m = pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=2, dp_size=2)
    bf = torch.bfloat16
    cfg = LlamaConfig(hidden_size=256, intermediate_size=512, num_attention_heads=4, num_key_value_heads=2,
                      num_hidden_layers=4, vocab_size=512, max_position_embeddings=S)
    torch.manual_seed(42)
    full = build_llama(cfg, device="cuda", dtype=bf)
    g = torch.Generator().manual_seed(5)
    with torch.no_grad():
        full.final_proj.weight.copy_((torch.randn(full.final_proj.weight.shape, generator=g) * 0.02).to(bf))
    ref_grads = {n: torch.zeros_like(p, dtype=torch.float32) for n, p in full.named_parameters()}
    data = {d: torch.randint(0, cfg.vocab_size, (GRAD_ACC, B, S + 1), generator=torch.Generator().manual_seed(100 + d))
            for d in range(2)}

    # --- reference: the unsplit model, layer by layer as the stages call it, over both DP ranks' micro-batches
    # (weight-gradient fusion off: the fused GEMMs accumulate into .grad and hand autograd.grad nothing)
    os.environ["PICO_WGRAD_FUSION"] = "0"
    for d in range(2):
        for mb in range(GRAD_ACC):
            toks = data[d][mb].cuda()
            x = full.embedding(toks[:, :-1])
            for layer in full.decoder_layers:
                x = layer(x, position_ids=None)
            logits = full.final_proj(full.final_norm(x))
            loss = F.cross_entropy(logits.transpose(1, 2), toks[:, 1:], reduction="mean")  # ref :98 (no / grad_acc)
            gs = torch.autograd.grad(loss, list(full.parameters()), allow_unused=True)
            for (n, _), gr in zip(full.named_parameters(), gs):
                if gr is not None:
                    ref_grads[n] += gr.float()

    os.environ["PICO_WGRAD_FUSION"] = "1"
    # --- the stage (ref pipeline_parallel.py:8-52; layer split :26-29)
    pp_rank, pp_size = m.pp_rank, m.pp_world_size
    per = [cfg.num_hidden_layers // pp_size + (1 if i < cfg.num_hidden_layers % pp_size else 0) for i in range(pp_size)]
    start = sum(per[:pp_rank])
    layers = list(range(start, start + per[pp_rank]))
    first, last = m.pp_is_first_stage, m.pp_is_last_stage

    class Stage(nn.Module):
        def __init__(self):
            super().__init__()
            self.embedding = full.embedding if first else nn.Identity()
            self.decoder_layers = nn.ModuleDict({str(i): full.decoder_layers[i] for i in layers})
            self.final_norm = full.final_norm if last else nn.Identity()
            self.final_proj = full.final_proj if last else nn.Identity()

        def forward(self, input_ids, position_ids, hidden_states):
            x = hidden_states if hidden_states is not None else input_ids
            x = self.embedding(x)
            for layer in self.decoder_layers.values():
                x = layer(x, position_ids=position_ids)
            x = self.final_norm(x)
            return self.final_proj(x)

        def backward(self, input_tensor, output_tensor, output_tensor_grad):
            if input_tensor is not None:
                input_tensor.retain_grad()
            if output_tensor_grad is None:
                output_tensor_grad = torch.ones_like(output_tensor, memory_format=torch.preserve_format)
            torch.autograd.backward(output_tensor, grad_tensors=output_tensor_grad, retain_graph=False,
                                    create_graph=False)
            return input_tensor.grad if input_tensor is not None else None

    for p in full.parameters():
        p.grad = None
    model = DataParallelBucket(Stage())
    shape = (B, S, cfg.hidden_size)

    # host-staged P2P (gloo): the reference's pipeline_communicate / bidirectional_pipeline_communicate
    def p2p(send=None, dst=None, recv=False, src=None):
        ops, buf = [], None
        if send is not None:
            ops.append(dist.P2POp(dist.isend, send.detach().float().cpu().contiguous(), dst))
        if recv:
            buf = torch.empty(shape, dtype=torch.float32)
            ops.append(dist.P2POp(dist.irecv, buf, src))
        for r in dist.batch_isend_irecv(ops):
            r.wait()
        return buf.cuda().to(bf).requires_grad_(True) if buf is not None else None

    mbs = iter(data[m.dp_rank])

    def forward_step(input_tensor):
        toks = next(mbs).cuda()
        out = model.forward(input_ids=toks[:, :-1], position_ids=None, hidden_states=input_tensor)
        if last:
            out = F.cross_entropy(out.transpose(1, 2), toks[:, 1:], reduction="mean")
        return out

    # ---- 1F1B (ref :85-145)
    warm = min(pp_size - pp_rank - 1, GRAD_ACC)
    remaining = GRAD_ACC - warm
    ins, outs = [], []
    nxt, prv = m.pp_next_rank, m.pp_prev_rank
    for _ in range(warm):
        inp = None if first else p2p(recv=True, src=prv)
        out = forward_step(inp)
        if not last:
            p2p(send=out, dst=nxt)
        ins.append(inp)
        outs.append(out)
    inp = None
    if remaining > 0 and not first:
        inp = p2p(recv=True, src=prv)
    model.require_backward_grad_sync = False
    for i in range(remaining):
        is_last = i == remaining - 1
        out = forward_step(inp)
        out_grad = None if last else p2p(send=out, dst=nxt, recv=True, src=nxt)
        ins.append(inp)
        outs.append(out)
        inp, out = ins.pop(0), outs.pop(0)
        if warm == 0 and is_last:
            model.require_backward_grad_sync = True
        in_grad = model.backward(inp, out, out_grad)
        if is_last:
            inp = None
            if not first:
                p2p(send=in_grad, dst=prv)
        else:
            inp = None if first else p2p(send=in_grad, dst=prv, recv=True, src=prv)
    for j in range(warm):
        model.require_backward_grad_sync = j == warm - 1
        inp, out = ins.pop(0), outs.pop(0)
        out_grad = None if last else p2p(recv=True, src=nxt)
        in_grad = model.backward(inp, out, out_grad)
        if not first:
            p2p(send=in_grad, dst=prv)
    torch.cuda.synchronize()

    names = dict((id(p), n) for n, p in full.named_parameters())
    res, errs = {}, {}
    for p in model.module.parameters():
        n = names[id(p)]
        ref = ref_grads[n] / 2
        assert p.grad is not None, n
        res[n] = (p.main_grad.detach().cpu().clone(), p.grad.detach().cpu().clone())
        den = float(ref.norm().clamp_min(1e-30))
        errs[n] = (float((p.main_grad - ref).norm()) / den, float((p.grad.float() - ref).norm()) / den)
    torch.save(res, os.path.join(out_dir, f"pp{pp_rank}_dp{m.dp_rank}.pt"))
    bad = {k: v for k, v in errs.items() if not (v[0] < 2e-2 and v[1] < 2e-2)}
    dist.barrier()
    dist.destroy_process_group()
    if bad:
        raise AssertionError(f"rank {rank} (pp {pp_rank}, dp {m.dp_rank}): {bad}")


def test_pp2_dp2_1f1b_data_parallel_bucket(tmp_path):
    mp.start_processes(_worker, args=(4, _free_port(), str(tmp_path)), nprocs=4, join=True, start_method="spawn")
    for pp in range(2):
        a = torch.load(tmp_path / f"pp{pp}_dp0.pt", weights_only=True)
        b = torch.load(tmp_path / f"pp{pp}_dp1.pt", weights_only=True)
        assert a.keys() == b.keys() and a
        for n in a:  # one all-reduce: both replicas hold the same average
            assert torch.equal(a[n][0], b[n][0]), n
            assert torch.equal(a[n][1], b[n][1]), n
