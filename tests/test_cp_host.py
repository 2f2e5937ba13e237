"""Context-parallel host logic on CPU (no GPU): the zig-zag layout, its load balance, the loader / RoPE
slicing that follow it, and the ring algorithm itself (RingAttentionFunc, contiguous and zig-zag) over
gloo with the attention block ops replaced by the fp64 oracle (oracle/hotpath.py attention_fwd/_bwd and
update_out_and_lse, ref picotron/context_parallel/context_parallel.py:112-187) — so the ring's block
schedule, merges and dK/dV hand-offs are checked independently of the HIP kernels, against whole-sequence
causal attention."""
import os
import socket
from types import SimpleNamespace

import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("S,n", [(16, 2), (64, 4), (256, 8)])
def test_zigzag_positions_partition(S, n):
    from picotron_amd.context_parallel.context_parallel import zigzag_positions
    c = S // (2 * n)
    seen = []
    for r in range(n):
        p = zigzag_positions(S, r, n)
        assert p.numel() == S // n
        assert torch.all(p[1:] > p[:-1])  # increasing: the local causal mask is the global one
        assert p[0] == r * c and p[c] == (2 * n - 1 - r) * c
        seen.append(p)
    assert torch.equal(torch.sort(torch.cat(seen))[0], torch.arange(S))
    with pytest.raises(AssertionError):
        zigzag_positions(S + 2, 0, n)


def _causal_pairs(qpos, kpos):
    return int((kpos[None, :] <= qpos[:, None]).sum())


@pytest.mark.parametrize("n", [2, 4, 8])
def test_zigzag_balances_causal_work(n):
    """Visible (query, key) pairs each rank computes over the ring: equal on every rank with the zig-zag
    split, r + 1/2 blocks' worth on rank r with the reference's contiguous split (rank cp - 1 ~ 2 cp x
    rank 0). Per ring step after the first, every zig-zag rank computes exactly c x 2c pairs."""
    from picotron_amd.context_parallel.context_parallel import zigzag_positions
    S = 64 * n
    c = S // (2 * n)
    zz = [zigzag_positions(S, r, n) for r in range(n)]
    cont = [torch.arange(r * S // n, (r + 1) * S // n) for r in range(n)]
    work_zz = [sum(_causal_pairs(zz[r], zz[(r - s) % n]) for s in range(n)) for r in range(n)]
    work_ct = [sum(_causal_pairs(cont[r], cont[(r - s) % n]) for s in range(n)) for r in range(n)]
    assert len(set(work_zz)) == 1
    assert work_ct[-1] > 1.8 * work_ct[0] and sum(work_ct) == sum(work_zz)
    for r in range(n):
        for s in range(1, n):
            assert _causal_pairs(zz[r], zz[(r - s) % n]) == c * 2 * c


def test_loader_and_rope_follow_zigzag(monkeypatch):
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.context_parallel import context_parallel as CP
    from picotron_amd.data import SyntheticDataLoader
    S, n, r = 32, 4, 1
    monkeypatch.setenv("PICO_CP_ZIGZAG", "1")
    monkeypatch.setattr(pgm, "process_group_manager",
                        SimpleNamespace(dp_world_size=1, dp_rank=0, cp_world_size=n, cp_rank=r))
    dl = SyntheticDataLoader(2, S, 1, 1000, seed=3, kind="arith")
    toks = dl._make()
    b = dl.collate(toks)
    pos = CP.zigzag_positions(S, r, n)
    assert torch.equal(b["input_ids"], toks[:, pos]) and torch.equal(b["target_ids"], toks[:, pos + 1])
    assert torch.equal(b["position_ids"][0], pos)
    cos = torch.arange(S * 4, dtype=torch.float32).view(S, 4)
    c2, s2 = CP.update_rope_for_context_parallel(cos, -cos)
    assert torch.equal(c2, cos[pos]) and torch.equal(s2, -cos[pos])
    monkeypatch.setenv("PICO_CP_ZIGZAG", "0")
    b = dl.collate(toks)
    assert torch.equal(b["input_ids"], toks[:, r * S // n:(r + 1) * S // n])


def test_apply_context_parallel_reslices_built_model_rope(monkeypatch):
    """the reference builds the model first and applies CP afterwards (ref train.py:175-188).
    apply_context_parallel(model, zigzag=True) on an already built model must re-slice every decoder layer's
    RoPE tables to the zig-zag positions (and back to the contiguous slice with zigzag=False); checked against
    the fp64 oracle's tables (oracle.hotpath.get_cos_sin, ref picotron/model.py:21-30) at those positions."""
    from oracle import hotpath as H
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.context_parallel import context_parallel as CP
    from picotron_amd.model import Llama, LlamaConfig
    S, n, r = 64, 4, 2
    monkeypatch.setenv("DEVICE", "cpu")
    monkeypatch.setenv("PICO_CP_ZIGZAG", "0")
    monkeypatch.setattr(pgm, "process_group_manager",
                        SimpleNamespace(tp_world_size=1, dp_world_size=1, dp_rank=0, cp_world_size=n, cp_rank=r))
    cfg = LlamaConfig(hidden_size=128, intermediate_size=256, num_attention_heads=2, num_key_value_heads=2,
                      num_hidden_layers=2, vocab_size=64, max_position_embeddings=S)
    with torch.device("meta"):
        model = Llama(cfg)
    cos_ref, sin_ref = H.get_cos_sin(S, 64, cfg.rope_theta)
    contiguous = torch.arange(r * S // n, (r + 1) * S // n)
    zig = CP.zigzag_positions(S, r, n)
    assert not torch.equal(contiguous, zig)

    def check(pos):
        for layer in model.decoder_layers:
            assert layer.cos.shape == (S // n, 64)
            assert torch.equal(layer.cos.double(), cos_ref[pos].double())
            assert torch.equal(layer.sin.double(), sin_ref[pos].double())

    check(contiguous)  # built under the contiguous layout
    CP.apply_context_parallel(model, zigzag=True)
    assert os.environ["PICO_CP_ZIGZAG"] == "1" and os.environ["CONTEXT_PARALLEL"] == "1"
    check(zig)
    CP.apply_context_parallel(model, zigzag=False)
    check(contiguous)


def _oracle_ops(CP, H):
    """attention_block_fwd/_bwd and update_out_and_lse on [B, S, H, D] tensors, computed by the oracle."""
    def fwd(q, k, v, scale, causal):
        o, lse = H.attention_fwd(q.transpose(1, 2).double(), k.transpose(1, 2).double(), v.transpose(1, 2).double(),
                                 scale, causal)
        return o.transpose(1, 2).to(q.dtype), lse.float()

    def bwd(dout, q, k, v, o, lse, scale, causal, dq_accum=None):
        t = lambda x: x.transpose(1, 2).double()
        dq, dk, dv = H.attention_bwd(t(dout), t(q), t(k), t(v), t(o), lse.double(), scale, causal)
        dq, dk, dv = (x.transpose(1, 2) for x in (dq, dk, dv))
        if dq_accum is not None:
            dq_accum += dq.to(dq_accum.dtype)
            dq = dq_accum
        return dq, dk.to(k.dtype), dv.to(v.dtype)

    def merge(out, lse, bo, bl):
        o2 = None if out is None else out.transpose(1, 2)
        l2 = None if lse is None else lse.unsqueeze(-1)
        o, l = H.update_out_and_lse(o2, l2, bo.transpose(1, 2), bl)
        return o.transpose(1, 2).contiguous(), l.squeeze(-1).contiguous()

    CP.ops.attention_block_fwd = fwd
    CP.ops.attention_block_bwd = bwd
    CP._merge_bshd = merge


def _ring_worker(rank, world, port, zigzag, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ["PICO_CP_ZIGZAG"] = "1" if zigzag else "0"
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import hotpath as H
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.context_parallel import context_parallel as CP
    pgm.setup_process_group_manager(tp_size=1, cp_size=world, pp_size=1, dp_size=1)
    _oracle_ops(CP, H)
    B, S, Hh, D = 1, 16 * world, 2, 8
    g = torch.Generator().manual_seed(4)
    q, k, v, do = [torch.randn(B, Hh, S, D, generator=g) for _ in range(4)]  # [B, H, S, D] like the reference
    pos = CP.zigzag_positions(S, rank, world) if zigzag else torch.arange(rank * S // world, (rank + 1) * S // world)
    ql, kl, vl = [t[:, :, pos].clone().requires_grad_(True) for t in (q, k, v)]
    ol = CP.ring_attention(ql, kl, vl, D ** -0.5, True)
    ol.backward(do[:, :, pos])
    torch.save({"pos": pos, "o": ol.detach(), "dq": ql.grad, "dk": kl.grad, "dv": vl.grad},
               os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,zigzag", [(2, False), (4, False), (2, True), (4, True)])
def test_ring_attention_host_algorithm(world, zigzag, tmp_path):
    mp.start_processes(_ring_worker, args=(world, _free_port(), zigzag, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    import sys
    sys.path.insert(0, ROOT)
    from oracle import hotpath as H
    B, S, Hh, D = 1, 16 * world, 2, 8
    g = torch.Generator().manual_seed(4)
    q, k, v, do = [torch.randn(B, Hh, S, D, generator=g) for _ in range(4)]
    qd, kd, vd = [t.double().requires_grad_(True) for t in (q, k, v)]
    o, _ = H.attention_fwd(qd, kd, vd, D ** -0.5, True)
    o.backward(do.double())
    for r in range(world):
        res = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        p = res["pos"]
        for name, ref in (("o", o.detach()), ("dq", qd.grad), ("dk", kd.grad), ("dv", vd.grad)):
            got = res[name].double()
            err = float((got - ref[:, :, p]).abs().max())
            assert err < 1e-5, (r, name, err)
