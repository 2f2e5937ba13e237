"""The hot path under the reference's whole 3-D grid (VERDICT r02 missing 1 / next 1a-b): data x tensor x
pipeline parallelism composed on the product path, ranks sharing this one GPU over gloo (RCCL refuses several
ranks on one device; the TP / DP collectives take the gloo branch of tp_communications / bucket.py, P2P is
host-staged).

  * C1 (BASELINE configs[0]): SmolLM-1.7B geometry, 5 layers, dp 2 x tp 2 x pp 2, micro-batch 4, seq 128,
    grad_acc 2 — eight ranks;
  * C4 variant: Llama-2-7B geometry (Hd 4096, I 11008 -> 5504 per tp rank, 32 heads -> 16, D = 128,
    V 32000) reduced to 2 layers, at the reference's micro-batch 4 and seq 1024 (ref README.md:34), dp 2 x tp 2 x
    pp 2 — eight ranks (the reference's dp 4 would be sixteen processes on this one GPU).

Each rank: the grid of ref picotron/process_group_manager.py:13-23 (picotron_amd.process_group_manager);
apply_tensor_parallel (ref picotron/tensor_parallel/tensor_parallel.py:9-52: column q/k/v/up/gate, row
out/down, vocab-parallel embedding, gathered column-parallel LM head) converting a model that holds the
unsplit model's weights, so the fused q|k|v + RoPE + attention and gate|up + SwiGLU ops run on the local
shards with one f region each; the rank's pipeline stage of the reference's layer split (ref
picotron/pipeline_parallel/pipeline_parallel.py:8-52, restated test-side: the PP wrapper is a hosted caller);
DataParallelBucket over cp_dp_group (ref picotron/data_parallel/data_parallel.py:62-171) with the weight
gradients fused into the fp32 main_grad (1/W folded into the syncing GEMMs); the reference's 1F1B schedule
(ref pipeline_parallel.py:85-145) with require_backward_grad_sync False until the last backward.

Checks per rank: every parameter's main_grad (fp32) and .grad (bf16) equal the rank's tensor-parallel shard of
(sum over the dp ranks' micro-batches of the unsplit model's gradient) / dp — within bf16 forward rounding;
the dp replicas of a (pp, tp) position hold identical gradients (one all-reduce).
"""
import json
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


# relative L2 bound on every sharded gradient vs the unsplit HIP model's (bf16 activations, different
# reduction orders under TP / PP / DP). Measured worst on MI355X: 1.04e-2 (c1_smollm_5l), 7.3e-3
# (c4_llama2_7b_2l); the bound was 2.5e-2 until those were recorded ("loose").
COMP_TOL = float(os.environ.get("PICO_COMP_TOL", "1.5e-2"))

GEOMETRY = {
    # name: (config kwargs, mbs, seq, grad_acc)
    "c1_smollm_5l": (dict(hidden_size=2048, intermediate_size=8192, num_attention_heads=32, num_key_value_heads=32,
                          num_hidden_layers=5, vocab_size=49152), 4, 128, 2),
    "c4_llama2_7b_2l": (dict(hidden_size=4096, intermediate_size=11008, num_attention_heads=32,
                             num_key_value_heads=32, num_hidden_layers=2, vocab_size=32000), 4, 1024, 2),
}


def _worker(rank, world, port, geom, tp, pp, dp, out_dir):
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
    from picotron_amd.tensor_parallel.tensor_parallel import apply_tensor_parallel
    m = pgm.setup_process_group_manager(tp_size=tp, cp_size=1, pp_size=pp, dp_size=dp)
    kw, B, S, GA = GEOMETRY[geom]
    cfg = LlamaConfig(max_position_embeddings=S, **kw)
    bf = torch.bfloat16

    # the unsplit model (built as at tp = 1) and the model to shard (built under tp: local head counts), same
    # weights; a nonzero LM head so every gradient below it is nonzero
    tp_size_fn = pgm.tp_world_size
    pgm.tp_world_size = lambda: 1
    torch.manual_seed(42)
    full = build_llama(cfg, device="cuda", dtype=bf)
    pgm.tp_world_size = tp_size_fn
    torch.manual_seed(42)
    tpm = build_llama(cfg, device="cuda", dtype=bf)
    g = torch.Generator().manual_seed(5)
    with torch.no_grad():
        full.final_proj.weight.copy_((torch.randn(full.final_proj.weight.shape, generator=g) * 0.02).to(bf))
        for pf, pt in zip(full.parameters(), tpm.parameters()):
            pt.copy_(pf)
    data = {d: torch.randint(0, cfg.vocab_size, (GA, B, S + 1), generator=torch.Generator().manual_seed(100 + d))
            for d in range(dp)}

    # --- reference gradients: the unsplit model over every dp rank's micro-batches, loss as the reference's
    # last stage computes it (ref pipeline_parallel.py:98, mean CE, no / grad_acc); fusion off so autograd.grad
    # sees every gradient
    os.environ["PICO_WGRAD_FUSION"] = "0"
    ref = {n: torch.zeros_like(p, dtype=torch.float32) for n, p in full.named_parameters()}
    for d in range(dp):
        for mb in range(GA):
            toks = data[d][mb].cuda()
            x = full.embedding(toks[:, :-1])
            for layer in full.decoder_layers:
                x = layer(x, position_ids=None)
            logits = full.final_proj(full.final_norm(x))
            loss = F.cross_entropy(logits.transpose(1, 2), toks[:, 1:], reduction="mean")
            for (n, _), gr in zip(full.named_parameters(), torch.autograd.grad(loss, list(full.parameters()))):
                ref[n] += gr.float()
    shapes = {n: tuple(p.shape) for n, p in full.named_parameters()}
    del full
    torch.cuda.empty_cache()
    os.environ["PICO_WGRAD_FUSION"] = "1"

    apply_tensor_parallel(tpm, shard_weights=True)
    assert tpm.decoder_layers[0].attention._fusable() == "tp" and tp > 1

    # --- this rank's pipeline stage (ref pipeline_parallel.py:8-52; layer split :26-29)
    pp_rank, pp_size = m.pp_rank, m.pp_world_size
    L = cfg.num_hidden_layers
    per = [L // pp_size + (1 if i < L % pp_size else 0) for i in range(pp_size)]
    start = sum(per[:pp_rank])
    layers = list(range(start, start + per[pp_rank]))
    first, last = m.pp_is_first_stage, m.pp_is_last_stage

    class Stage(nn.Module):
        def __init__(self):
            super().__init__()
            self.embedding = tpm.embedding if first else nn.Identity()
            self.decoder_layers = nn.ModuleDict({str(i): tpm.decoder_layers[i] for i in layers})
            self.final_norm = tpm.final_norm if last else nn.Identity()
            self.final_proj = tpm.final_proj if last else nn.Identity()

        def forward(self, input_ids, position_ids, hidden_states):
            x = hidden_states if hidden_states is not None else input_ids
            x = self.embedding(x)
            for layer in self.decoder_layers.values():
                x = layer(x, position_ids=position_ids)
            return self.final_proj(self.final_norm(x))

        def backward(self, input_tensor, output_tensor, output_tensor_grad):  # ref pipeline_parallel.py:46-52
            if input_tensor is not None:
                input_tensor.retain_grad()
            if output_tensor_grad is None:
                output_tensor_grad = torch.ones_like(output_tensor, memory_format=torch.preserve_format)
            torch.autograd.backward(output_tensor, grad_tensors=output_tensor_grad, retain_graph=False,
                                    create_graph=False)
            return input_tensor.grad if input_tensor is not None else None

    stage = Stage()
    names = {id(p): n for n, p in tpm.named_parameters()}
    model = DataParallelBucket(stage)
    assert model.bucket_manager.process_group_size == dp
    shape = (B, S, cfg.hidden_size)

    def p2p(send=None, dst=None, recv=False, src=None):  # host-staged batch_isend_irecv (ref pp_communications.py)
        ops_, buf = [], None
        if send is not None:
            ops_.append(dist.P2POp(dist.isend, send.detach().float().cpu().contiguous(), dst))
        if recv:
            buf = torch.empty(shape, dtype=torch.float32)
            ops_.append(dist.P2POp(dist.irecv, buf, src))
        for r in dist.batch_isend_irecv(ops_):
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
    warm = min(pp_size - pp_rank - 1, GA)
    remaining = GA - warm
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

    # --- gradients vs the unsplit model's, sharded like the parameter
    tr = m.tp_rank
    res, errs = {}, {}
    for p in stage.parameters():
        n = names[id(p)]
        want = ref[n] / dp
        if tuple(p.shape) != shapes[n]:  # column (rows) / vocab (rows) or row (columns) parallel
            if p.shape[0] != shapes[n][0]:
                k = p.shape[0]
                want = want[tr * k:(tr + 1) * k]
            else:
                k = p.shape[1]
                want = want[:, tr * k:(tr + 1) * k]
        assert p.grad is not None and p.main_grad is not None, n
        den = float(want.norm().clamp_min(1e-30))
        errs[n] = (float((p.main_grad - want).norm()) / den, float((p.grad.float() - want).norm()) / den)
        res[n] = (p.main_grad.detach().cpu().clone(), p.grad.detach().cpu().clone())
        assert torch.equal(p.grad, p.main_grad.to(bf)), n  # .grad = bf16 cast of the averaged main_grad
    torch.save(res, os.path.join(out_dir, f"pp{pp_rank}_tp{tr}_dp{m.dp_rank}.pt"))
    with open(os.path.join(out_dir, f"errs_pp{pp_rank}_tp{tr}_dp{m.dp_rank}.json"), "w") as f:
        json.dump(errs, f)
    bad = {k: v for k, v in errs.items() if not (v[0] < COMP_TOL and v[1] < COMP_TOL)}
    dist.barrier()
    dist.destroy_process_group()
    if bad:
        raise AssertionError(f"rank {rank} (pp {pp_rank}, tp {tr}, dp {m.dp_rank}) {geom}: {bad}")


@pytest.mark.parametrize("geom,tp,pp,dp", [("c1_smollm_5l", 2, 2, 2), ("c4_llama2_7b_2l", 2, 2, 2)])
def test_dp_tp_pp_1f1b_composition(geom, tp, pp, dp, tmp_path):
    world = tp * pp * dp
    mp.start_processes(_worker, args=(world, _free_port(), geom, tp, pp, dp, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    worst = max(max(v) for f in tmp_path.glob("errs_*.json") for v in json.load(open(f)).values())
    print(f"[composition {geom}] worst gradient rel-L2 vs the unsplit model: {worst:.3e} (bound {COMP_TOL})")
    if dp > 1:
        for p in range(pp):
            for t in range(tp):
                a = torch.load(tmp_path / f"pp{p}_tp{t}_dp0.pt", weights_only=True)
                for d in range(1, dp):
                    b = torch.load(tmp_path / f"pp{p}_tp{t}_dp{d}.pt", weights_only=True)
                    assert a.keys() == b.keys() and a
                    for n in a:
                        assert torch.equal(a[n][0], b[n][0]), n
                        assert torch.equal(a[n][1], b[n][1]), n
