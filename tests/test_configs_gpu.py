"""Kernel parity at the BASELINE configs' own shapes (VERDICT r01 "configs untested"), against an fp32
torch reference computed on the GPU on the same bf16 inputs (north_star: "fp32 reference, max-abs and
relative error reported"). Tolerances as DESIGN.md §3 / tests/test_kernels_gpu.py: attention output
rel-L2 <= 4e-3 and LSE max-abs <= 2e-3, attention gradients rel-L2 <= 1e-2, norm / SwiGLU rel-L2 <= 4e-3.

  C2  SmolLM-1.7B, micro-batch 4, S 1024: attention (B 4, S 1024, 32 heads, D 64) fwd + bwd, whole shape.
  C4  Llama-2-7B per tensor-parallel rank (tp 2): attention at the reference's micro-batch (B 4, S 1024, 16 heads,
      D 128; ref README.md:34 `--mbs 4 --seq_len 1024`) and at B 2 (the grid of one 256-CU round), RMSNorm
      [4096 x 4096] (residual form), SwiGLU with I / tp = 5504 on the strided halves of one gate|up GEMM.
  C5  SmolLM-1.7B cp 8 at S 32768 -> 4096-row blocks (B 1, 32 heads, D 64): the ring's block forward
      (causal diagonal + full off-diagonal), the 3-block LSE merge, and block backwards from the GLOBAL
      O / LSE with fp32 dQ accumulation (ref picotron/context_parallel/context_parallel.py:17-155).
Errors are printed (pytest -s) so the GPUTEST log carries them.
"""
import math

import pytest
import torch

from conftest import max_abs, rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def _report(tag, **errs):
    print(f"[config-parity] {tag}: " + ", ".join(f"{k}={v:.3e}" for k, v in errs.items()), flush=True)


def _attn_ref(q, k, v, do, scale, causal, q_offset=0):
    """fp32 attention on the GPU: q [B,Sq,Hq,D], k/v [B,Sk,Hkv,D] (bf16) -> out [B,Sq,Hq,D], lse [B,Hq,Sq],
    grads (dq, dk, dv) in the input layouts. Causal with q_offset: query i sees keys <= q_offset + i."""
    Hq, Hkv = q.shape[2], k.shape[2]
    qf, kf, vf = [t.float().transpose(1, 2).detach().requires_grad_(True) for t in (q, k, v)]
    kr = kf.repeat_interleave(Hq // Hkv, 1)
    vr = vf.repeat_interleave(Hq // Hkv, 1)
    s = (qf @ kr.transpose(-1, -2)) * scale
    if causal:
        Sq, Sk = s.shape[-2:]
        i = torch.arange(Sq, device=DEV)[:, None] + q_offset
        j = torch.arange(Sk, device=DEV)[None, :]
        s = s.masked_fill(j > i, float("-inf"))
    lse = torch.logsumexp(s, -1)
    out = torch.softmax(s, -1) @ vr
    gq, gk, gv = torch.autograd.grad(out, (qf, kf, vf), do.float().transpose(1, 2))
    tr = lambda t: t.transpose(1, 2)
    return tr(out).detach(), lse.detach(), (tr(gq), tr(gk), tr(gv))


@pytest.mark.parametrize("tag,B,S,Hq,Hkv,D", [("C2", 4, 1024, 32, 32, 64), ("C4-tp2-mbs4", 4, 1024, 16, 16, 128),
                                               ("C4-tp2-mbs2", 2, 1024, 16, 16, 128)])
def test_attention_full_config_shape(tag, B, S, Hq, Hkv, D):
    from picotron_amd import ops
    torch.manual_seed(S + Hq + D)
    q = torch.randn(B, S, Hq, D, dtype=BF, device=DEV)
    k = torch.randn(B, S, Hkv, D, dtype=BF, device=DEV)
    v = torch.randn(B, S, Hkv, D, dtype=BF, device=DEV)
    do = torch.randn(B, S, Hq, D, dtype=BF, device=DEV)
    sc = 1.0 / math.sqrt(D)
    o, lse = ops.attention_block_fwd(q, k, v, sc, True)
    dq, dk, dv = ops.attention_block_bwd(do, q, k, v, o, lse, sc, True)
    O, L, (gq, gk, gv) = _attn_ref(q, k, v, do, sc, True)
    e = dict(out=rel_l2(o.float(), O), out_maxabs=max_abs(o.float(), O), lse_maxabs=max_abs(lse, L),
             dq=rel_l2(dq.float(), gq), dk=rel_l2(dk.float(), gk), dv=rel_l2(dv.float(), gv),
             dq_maxabs=max_abs(dq.float(), gq))
    _report(f"{tag} attention {B}x{S}x{Hq}/{Hkv}x{D}", **e)
    assert e["out"] < 4e-3 and e["lse_maxabs"] < 2e-3
    assert e["dq"] < 1e-2 and e["dk"] < 1e-2 and e["dv"] < 1e-2


def test_rmsnorm_llama7b_hidden():
    """C4: RMSNorm over [micro-batch 4 x 1024 tokens, 4096] in the residual (prenorm) form the model uses."""
    from picotron_amd import ops
    torch.manual_seed(4096)
    x = (torch.randn(4096, 4096, device=DEV) * 2).to(BF).requires_grad_(True)
    res = torch.randn(4096, 4096, device=DEV).to(BF).requires_grad_(True)
    w = (1 + 0.1 * torch.randn(4096, device=DEV)).to(BF).requires_grad_(True)
    y, r = ops.rms_norm(x, w, 1e-5, residual=res, prenorm=True)
    dy, dr = torch.randn_like(y), torch.randn_like(r)
    torch.autograd.backward((y, r), (dy, dr))
    xs = (x.detach().float() + res.detach().float()).to(BF).float().requires_grad_(True)  # x_eff in bf16
    wf = w.detach().float().requires_grad_(True)
    yf = xs * torch.rsqrt(xs.pow(2).mean(-1, keepdim=True) + 1e-5) * wf
    gx, gw = torch.autograd.grad(yf, (xs, wf), dy.float())
    gx = gx + dr.float()
    e = dict(y=rel_l2(y.float(), yf), res_out=max_abs(r.float(), xs), dx=rel_l2(x.grad.float(), gx),
             dres=rel_l2(res.grad.float(), gx), dw=rel_l2(w.grad.float(), gw))
    _report("C4 rmsnorm 4096x4096 residual", **e)
    assert e["y"] < 4e-3 and e["res_out"] == 0.0
    assert e["dx"] < 4e-3 and e["dres"] < 4e-3 and e["dw"] < 4e-3


def test_swiglu_llama7b_tp2_strided_halves():
    """C4: I / tp = 5504, SwiGLU on the two column halves of one [T, 2I] gate|up GEMM output (row stride 2I),
    forward (with the h^T by-product) and backward into the halves of one [T, 2I] gradient."""
    from picotron_amd import ops
    torch.manual_seed(5504)
    T, Hd, I = 2048, 512, 5504
    x = (torch.randn(T, Hd, device=DEV) * 0.5).to(BF).requires_grad_(True)
    wg = (torch.randn(I, Hd, device=DEV) / math.sqrt(Hd)).to(BF).requires_grad_(True)
    wu = (torch.randn(I, Hd, device=DEV) / math.sqrt(Hd)).to(BF).requires_grad_(True)
    h = ops.gate_up_swiglu(x, wg, wu)
    ht = getattr(h, "_pico_t", None)
    dh = torch.randn_like(h)
    h.backward(dh)
    # reference on the same bf16 GEMM outputs (the GEMM is hipBLASLt in both; the kernel is the epilogue)
    gu = (x.detach() @ torch.cat([wg.detach(), wu.detach()], 0).t())
    g, u = gu[:, :I].float().requires_grad_(True), gu[:, I:].float().requires_grad_(True)
    href = torch.nn.functional.silu(g) * u
    dg, du = torch.autograd.grad(href, (g, u), dh.float())
    dgu = torch.cat([dg, du], 1)
    dx_ref = dgu @ torch.cat([wg.detach(), wu.detach()], 0).float()
    e = dict(h=rel_l2(h.float(), href), dx=rel_l2(x.grad.float(), dx_ref),
             dwg=rel_l2(wg.grad.float(), dg.t() @ x.detach().float()),
             dwu=rel_l2(wu.grad.float(), du.t() @ x.detach().float()))
    _report("C4 swiglu T2048 I5504 strided", **e)
    assert e["h"] < 4e-3 and e["dx"] < 1e-2 and e["dwg"] < 1e-2 and e["dwu"] < 1e-2
    if ht is not None:
        assert torch.equal(ht, h.detach().t())


def test_ring_blocks_cp8_local_4096():
    """C5: the last cp rank's view of 3 ring steps at S_local 4096 — its query block against its own KV block
    (causal) and two earlier blocks (full) — merged in fp32 (3-block update_out_and_lse), then each block's
    backward fed the GLOBAL O / LSE with dQ accumulated in fp32, vs whole-sequence fp32 attention."""
    from picotron_amd import ops
    from picotron_amd.context_parallel.context_parallel import _merge_bshd
    torch.manual_seed(32768)
    B, n, H, D, nb = 1, 4096, 32, 64, 3
    sc = 1.0 / math.sqrt(D)
    q = torch.randn(B, n, H, D, dtype=BF, device=DEV)
    ks = [torch.randn(B, n, H, D, dtype=BF, device=DEV) for _ in range(nb)]
    vs = [torch.randn(B, n, H, D, dtype=BF, device=DEV) for _ in range(nb)]
    do = torch.randn(B, n, H, D, dtype=BF, device=DEV)
    out = lse = None
    for j in range(nb):  # ring order: own block (causal) first, then the earlier ones
        src = nb - 1 - j
        bo, bl = ops.attention_block_fwd(q, ks[src], vs[src], sc, src == nb - 1)
        out, lse = _merge_bshd(out, lse, bo, bl)
    o = out.to(BF)
    kcat, vcat = torch.cat(ks, 1), torch.cat(vs, 1)
    O, L, (gq, gk, gv) = _attn_ref(q, kcat, vcat, do, sc, True, q_offset=(nb - 1) * n)
    dq = torch.zeros(q.shape, dtype=torch.float32, device=DEV)
    dks, dvs = [], []
    for src in range(nb):
        _, dk, dv = ops.attention_block_bwd(do, q, ks[src], vs[src], o, lse, sc, src == nb - 1, dq_accum=dq)
        dks.append(dk)
        dvs.append(dv)
    e = dict(out=rel_l2(o.float(), O), lse_maxabs=max_abs(lse, L), dq=rel_l2(dq, gq),
             dk=rel_l2(torch.cat(dks, 1).float(), gk), dv=rel_l2(torch.cat(dvs, 1).float(), gv))
    _report("C5 ring blocks 3 x 4096 (B1 H32 D64)", **e)
    assert e["out"] < 4e-3 and e["lse_maxabs"] < 2e-3
    assert e["dq"] < 1e-2 and e["dk"] < 1e-2 and e["dv"] < 1e-2
