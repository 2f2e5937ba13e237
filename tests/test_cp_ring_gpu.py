"""Context-parallel ring attention across ranks on the GPU: RingAttentionFunc (ref
picotron/context_parallel/context_parallel.py:17-110) with cp = 2 and 4 ranks sharing this one GPU,
forward and backward on the gfx950 kernels, against whole-sequence attention on the same inputs.

RCCL refuses two ranks on one device, so the ring's P2P runs over gloo with each transfer staged
through host memory (a test-only ContextCommunicate; the product class is plain RCCL
batch_isend_irecv). Every other piece — block kernels, LSE merge kernel, fp32 dQ accumulation, the
dK/dV rotation order — is the product path.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _staged_comm_class(base):
    import torch.distributed as dist

    class HostStagedCommunicate(base):
        """Same ring protocol as the product's ContextCommunicate; buffers cross over host memory."""

        def send_recv(self, tensor_to_send, recv_tensor=None):
            result = (torch.empty(tensor_to_send.shape, dtype=tensor_to_send.dtype, device=tensor_to_send.device)
                      if recv_tensor is None else recv_tensor)
            host_send = tensor_to_send.detach().contiguous().cpu()
            host_recv = torch.empty(result.shape, dtype=result.dtype)
            self._pending.append(dist.P2POp(dist.isend, host_send, self.send_rank, group=self.group))
            self._pending.append(dist.P2POp(dist.irecv, host_recv, self.recv_rank, group=self.group))
            self._landing = getattr(self, "_landing", []) + [(host_recv, result)]
            return result

        def wait(self):
            super().wait()
            for host, dev in self._landing:
                dev.copy_(host)
            self._landing = []

    return HostStagedCommunicate


def _worker(rank, world, port, causal, zigzag=False, S=1024, B=2, Hq=4, rope=False):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from picotron_amd import ops
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.context_parallel import context_parallel as CP
    pgm.setup_process_group_manager(tp_size=1, cp_size=world, pp_size=1, dp_size=1)
    os.environ["PICO_CP_ZIGZAG"] = "1" if zigzag else "0"
    CP.ContextCommunicate = _staged_comm_class(CP.ContextCommunicate)

    dev = "cuda:0"
    D = 64
    g = torch.Generator(device="cpu").manual_seed(21)  # identical full tensors on every rank
    q, k, v, do = [torch.randn(B, S, Hq, D, generator=g).to(BF).to(dev) for _ in range(4)]
    scale = D ** -0.5
    # rope: q and k rotated before attention with the whole-sequence tables, and on each rank with the tables
    # update_rope_for_context_parallel slices for it (ref picotron/context_parallel/context_parallel.py:189-195,
    # ref picotron/model.py:135-136) — at C5 that is positions up to 32,767
    if rope:
        from picotron_amd.model import get_cos_sin
        cos, sin = get_cos_sin(S, D, base=10000.0)
        cos, sin = cos.to(dev), sin.to(dev)
        cosl, sinl = CP.update_rope_for_context_parallel(cos, sin)
        rot = lambda x, c, s_: ops.apply_rotary_emb(x, c[:, : D // 2], s_[:, : D // 2])  # noqa: E731
    # whole-sequence reference through the same kernels (pinned to the fp64 oracle by test_kernels_gpu)
    qf, kf, vf = [t.clone().requires_grad_(True) for t in (q, k, v)]
    qa, ka = (rot(qf, cos, sin), rot(kf, cos, sin)) if rope else (qf, kf)
    of = ops.flash_attn_func(qa, ka, vf, softmax_scale=scale, causal=causal)
    of.backward(do)
    n = S // world
    # this rank's rows: contiguous chunk (reference split) or the zig-zag pair of chunks
    sl = CP.zigzag_positions(S, rank, world).to(dev) if zigzag else slice(rank * n, (rank + 1) * n)
    ql, kl, vl = [t[:, sl].contiguous().requires_grad_(True) for t in (q, k, v)]
    qla, kla = (rot(ql, cosl, sinl), rot(kl, cosl, sinl)) if rope else (ql, kl)
    # exactly the reference's call (ref picotron/model.py:139-150): [B, S, H, D] projections transposed to
    # [B, H, S, D], ring_attention, output transposed back to [B, S, H, D]
    ol = CP.ring_attention(qla.transpose(1, 2), kla.transpose(1, 2), vl.transpose(1, 2), scale, causal).transpose(1, 2)
    assert ol.shape == ql.shape
    ol.backward(do[:, sl].contiguous())
    torch.cuda.synchronize()

    def rel(a, b):
        a, b = a.double(), b.double()
        return float((a - b).norm() / b.norm())

    errs = {"out": rel(ol, of[:, sl]), "dq": rel(ql.grad, qf.grad[:, sl]), "dk": rel(kl.grad, kf.grad[:, sl]),
            "dv": rel(vl.grad, vf.grad[:, sl])}
    # bf16 outputs of two differently-blocked fp32 computations: within a few bf16 roundings
    tol = {"out": 4e-3, "dq": 8e-3, "dk": 8e-3, "dv": 8e-3}
    bad = {kk: e for kk, e in errs.items() if not e < tol[kk]}
    dist.barrier()
    dist.destroy_process_group()
    if bad:
        raise AssertionError(f"rank {rank} cp={world} causal={causal} zigzag={zigzag}: {bad} (all: {errs})")


@pytest.mark.parametrize("world,causal,zigzag,S,B,Hq,rope", [
    (2, True, False, 1024, 2, 4, False), (4, True, False, 1024, 2, 4, False), (2, False, False, 1024, 2, 4, False),
    (2, True, True, 1024, 2, 4, False), (4, True, True, 1024, 2, 4, True), (8, True, False, 2048, 2, 4, False),
    (8, True, True, 2048, 2, 4, False),
    # config 5 itself (BASELINE configs[4]): cp = 8 at S = 32768, S_local = 4096 — the last rank's eight-block chain of
    # 4096-row blocks and the RoPE tables sliced per rank at positions up to 32,767; B = 1, 2 heads
    (8, True, False, 32768, 1, 2, True), (8, True, True, 32768, 1, 2, True)])
def test_ring_attention_multi_rank(world, causal, zigzag, S, B, Hq, rope):
    """Contiguous (reference) split, and the zig-zag split (PICO_CP_ZIGZAG=1: rank r holds chunks r and
    2 cp - 1 - r; every rank does equal block work), against whole-sequence attention at the rows each
    rank holds. cp = 8 (C5's ring size): the 8-step ring loop, and the zig-zag split
    into 2 cp = 16 chunks, at S = 2048 and at C5's own S = 32768."""
    mp.start_processes(_worker, args=(world, _free_port(), causal, zigzag, S, B, Hq, rope), nprocs=world, join=True,
                       start_method="spawn")
