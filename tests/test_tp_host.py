"""Tensor-parallel layers on CPU over gloo (world 2 and 4): apply_tensor_parallel(shard_weights=True) on a
small model skeleton, then every parallel layer against its unsharded nn.Linear / nn.Embedding on the
same weights — forward values and input / weight gradients — including the async input-gradient
all-reduce of ColumnParallelLinear, the gathered LM head and the vocab-parallel embedding
(ref picotron/tensor_parallel/tensor_parallel.py:9-270, tp_communications.py:19-108)."""
import os
import socket

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


def _worker(rank, world, port):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import torch.nn as nn
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.tensor_parallel import tensor_parallel as TP
    pgm.setup_process_group_manager(tp_size=world, cp_size=1, pp_size=1, dp_size=1)
    torch.manual_seed(0)
    H, I, V, T = 16, 32, 64, 6

    class Attn(nn.Module):
        def __init__(self):
            super().__init__()
            self.q_proj, self.k_proj, self.v_proj = (nn.Linear(H, H, bias=False) for _ in range(3))
            self.out_proj = nn.Linear(H, H, bias=False)

    class Mlp(nn.Module):
        def __init__(self):
            super().__init__()
            self.up_proj, self.gate_proj = nn.Linear(H, I, bias=False), nn.Linear(H, I, bias=False)
            self.down_proj = nn.Linear(I, H, bias=False)

    class Layer(nn.Module):
        def __init__(self):
            super().__init__()
            self.attention, self.mlp = Attn(), Mlp()

    class Skel(nn.Module):
        def __init__(self):
            super().__init__()
            self.embedding = nn.Embedding(V, H)
            self.decoder_layers = nn.ModuleList([Layer()])
            self.final_proj = nn.Linear(H, V, bias=False)

    full = Skel().double()
    tp = Skel().double()
    tp.load_state_dict(full.state_dict())
    TP.apply_tensor_parallel(tp, shard_weights=True)
    lt, lf = tp.decoder_layers[0], full.decoder_layers[0]
    assert isinstance(lt.attention.q_proj, TP.ColumnParallelLinear) and isinstance(lt.mlp.down_proj, TP.RowParallelLinear)
    assert isinstance(tp.embedding, TP.VocabParallelEmbedding) and tp.final_proj.gather_output
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(0, V, (2, T), generator=g)
    errs = {}

    def close(name, a, b):
        errs[name] = float((a - b).abs().max())

    # embedding (vocab-parallel) -> column (q) with async all-reduce -> row (out) -> gathered LM head
    lt.attention.q_proj.async_all_reduce = True
    xf = full.embedding(ids)
    xt = tp.embedding(ids)
    close("embedding", xt, xf)
    xf2, xt2 = xf.detach().requires_grad_(True), xt.detach().requires_grad_(True)
    hf = lf.attention.out_proj(lf.attention.q_proj(xf2))
    ht = lt.attention.out_proj(lt.attention.q_proj(xt2))
    close("q->out", ht, hf)
    yf, yt = torch.tanh(hf) @ torch.ones(H, 1, dtype=torch.float64), torch.tanh(ht) @ torch.ones(H, 1, dtype=torch.float64)
    logits_f = full.final_proj(lf.mlp.down_proj(lf.mlp.up_proj(hf) * lf.mlp.gate_proj(hf)))
    logits_t = tp.final_proj(lt.mlp.down_proj(lt.mlp.up_proj(ht) * lt.mlp.gate_proj(ht)))
    close("logits", logits_t, logits_f)
    (logits_f.square().mean() + yf.sum()).backward()
    (logits_t.square().mean() + yt.sum()).backward()
    close("dx", xt2.grad, xf2.grad)
    n = world
    for name, mf, mt, style in (("q", lf.attention.q_proj, lt.attention.q_proj, "col"),
                                ("out", lf.attention.out_proj, lt.attention.out_proj, "row"),
                                ("up", lf.mlp.up_proj, lt.mlp.up_proj, "col"), ("gate", lf.mlp.gate_proj, lt.mlp.gate_proj, "col"),
                                ("down", lf.mlp.down_proj, lt.mlp.down_proj, "row"), ("lm", full.final_proj, tp.final_proj, "col")):
        gfull = mf.weight.grad
        if style == "col":
            k = gfull.shape[0] // n
            ref = gfull[rank * k:(rank + 1) * k]
        else:
            k = gfull.shape[1] // n
            ref = gfull[:, rank * k:(rank + 1) * k]
        close("dW " + name, mt.weight.grad, ref)
    xe = tp.embedding(ids)
    (xe * torch.arange(H, dtype=torch.float64)).sum().backward()
    full.embedding.weight.grad = None
    (full.embedding(ids) * torch.arange(H, dtype=torch.float64)).sum().backward()
    k = V // n
    close("dW embedding", tp.embedding.weight.grad, full.embedding.weight.grad[rank * k:(rank + 1) * k])
    bad = {kk: e for kk, e in errs.items() if not e < 1e-10}
    dist.barrier()
    dist.destroy_process_group()
    if bad:
        raise AssertionError(f"rank {rank}: {bad}")


@pytest.mark.parametrize("world", [2, 4])
def test_tensor_parallel_layers_match_unsharded(world):
    mp.start_processes(_worker, args=(world, _free_port()), nprocs=world, join=True, start_method="spawn")
