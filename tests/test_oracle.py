"""Pin the CPU oracle (oracle/) to golden vectors produced by the reference itself
(tests/golden/make_golden.py, run in the build container). CPU only."""
import math
from types import SimpleNamespace

import pytest
import torch

from conftest import max_abs, rel_l2
from oracle import hotpath as H
from oracle import model as OM


def test_rmsnorm_eager_bit_exact(golden_kernels):
    g = golden_kernels
    y = H.rmsnorm_eager(g["rms.x"], g["rms.w"], 1e-5)
    assert torch.equal(y, g["rms.y_eager_bf16"])


def test_rmsnorm_grads(golden_kernels):
    g = golden_kernels
    # the reference module normalises in fp32 even for fp64 inputs (ref model.py:82), so its
    # "f64" goldens carry fp32 rounding: compare at fp32 resolution
    dx, dw = H.rmsnorm_grads(g["rms.x"], g["rms.w"], 1e-5, g["rms.dy"])
    assert rel_l2(dx, g["rms.dx_f64"]) < 1e-6
    assert rel_l2(dw, g["rms.dw_f64"]) < 1e-6
    y, _ = H.rmsnorm_fused(g["rms.x"].double(), g["rms.w"].double(), 1e-5)
    assert rel_l2(y, g["rms.y_f64"]) < 1e-6


def test_cos_sin_tables_bit_exact(golden_kernels):
    g = golden_kernels
    c, s = H.get_cos_sin(64, 64, base=10000.0)
    assert torch.equal(c, g["rope.cos"]) and torch.equal(s, g["rope.sin"])
    c, s = H.get_cos_sin(1024, 64, base=10000.0)
    assert torch.equal(c, g["rope.cos_1024"]) and torch.equal(s, g["rope.sin_1024"])


def test_rope(golden_kernels):
    g = golden_kernels
    q, c, s = g["rope.q"], g["rope.cos"], g["rope.sin"]
    assert torch.equal(H.rope_eager(q, c, s), g["rope.out_eager_bf16"])
    # fused (flash-attn) numerics in fp64 == the reference formula in fp64
    out = H.rope_fused(q.double().transpose(1, 2), c.double(), s.double()).transpose(1, 2)
    assert max_abs(out, g["rope.out_f64"]) < 1e-12
    # backward = rotation by -theta
    dx = H.rope_fused(g["rope.dy"].double().transpose(1, 2), c.double(), s.double(), conjugate=True).transpose(1, 2)
    assert max_abs(dx, g["rope.dx_f64"]) < 1e-12


@pytest.mark.parametrize("tag", ["causal", "full"])
def test_attention_block(golden_kernels, tag):
    g = golden_kernels
    p = lambda n: g[f"attn.{tag}.{n}"]
    sc = 1.0 / math.sqrt(64)
    O, L = H.attention_fwd(p("q"), p("k"), p("v"), sc, tag == "causal")
    assert max_abs(O, p("o")) < 1e-6 and max_abs(L, p("lse")) < 1e-6
    assert max_abs(O, p("sdpa")) < 1e-5
    dq, dk, dv = H.attention_bwd(p("do"), p("q"), p("k"), p("v"), p("o"), p("lse"), sc, tag == "causal")
    for a, b in ((dq, "dq"), (dk, "dk"), (dv, "dv")):
        assert max_abs(a, p(b)) < 1e-5


def test_attention_gqa_matches_expanded():
    torch.manual_seed(0)
    q = torch.randn(2, 4, 32, 64, dtype=torch.float64)
    k = torch.randn(2, 2, 32, 64, dtype=torch.float64)
    v = torch.randn(2, 2, 32, 64, dtype=torch.float64)
    do = torch.randn(2, 4, 32, 64, dtype=torch.float64)
    O, L = H.attention_fwd(q, k, v, 0.125, True)
    qq, kk, vv = [t.clone().requires_grad_(True) for t in (q, k, v)]
    ref = torch.nn.functional.scaled_dot_product_attention(qq, kk.repeat_interleave(2, 1), vv.repeat_interleave(2, 1),
                                                           is_causal=True, scale=0.125)
    ref.backward(do)
    assert max_abs(O, ref) < 1e-12
    dq, dk, dv = H.attention_bwd(do, q, k, v, O, L, 0.125, True)
    assert max_abs(dq, qq.grad) < 1e-10 and max_abs(dk, kk.grad) < 1e-10 and max_abs(dv, vv.grad) < 1e-10


def test_update_out_and_lse(golden_kernels):
    g = golden_kernels
    out = lse = None
    for i in range(3):
        out, lse = H.update_out_and_lse(out, lse, g[f"merge.block_out{i}"], g[f"merge.block_lse{i}"])
    assert torch.equal(out, g["merge.out"]) and torch.equal(lse.squeeze(-1), g["merge.lse"])


def test_swiglu(golden_kernels):
    g = golden_kernels
    h = H.swiglu(g["swiglu.g"].double(), g["swiglu.u"].double())
    assert max_abs(h, g["swiglu.h_f64"]) < 1e-12
    assert torch.equal(torch.nn.functional.silu(g["swiglu.g"]) * g["swiglu.u"], g["swiglu.h_eager_bf16"])
    dg, du = H.swiglu_grads(g["swiglu.g"], g["swiglu.u"], g["swiglu.dh"])
    assert max_abs(dg, g["swiglu.dg_f64"]) < 1e-12 and max_abs(du, g["swiglu.du_f64"]) < 1e-12


def test_bucket_layouts_bit_exact(golden_layouts):
    """oracle restatement AND the product's host-side layout == the reference's BucketManager."""
    from picotron_amd.data_parallel.bucket import BucketManager
    for name, lay in golden_layouts.items():
        rg = [True] * len(lay["numels"])
        locs, sizes = H.bucket_layout(lay["numels"], rg, lay["bucket_size"])
        assert [list(l) for l in locs] == lay["locations"], name
        assert sizes == lay["bucket_sizes"], name
        locs2, sizes2 = BucketManager.compute_layout(lay["numels"], rg, lay["bucket_size"])
        assert [list(l) for l in locs2] == lay["locations"], name
        assert sizes2 == lay["bucket_sizes"], name
    assert len(golden_layouts["smollm_1.7b_15l"]["bucket_sizes"]) == 108
    assert sum(golden_layouts["smollm_1.7b_15l"]["numels"]) == 1_208_023_040


def test_bucket_layout_edge_cases():
    # param larger than the cap opens its own bucket; frozen params are skipped; empty model
    locs, sizes = H.bucket_layout([5, 100, 3, 2, 1], [True, True, False, True, True], 10)
    assert locs == [(0, 5, 0), (0, 100, 1), None, (0, 2, 2), (2, 3, 2)]
    assert sizes == [5, 100, 3]
    assert H.bucket_layout([], [], 10) == ([], [])
    assert H.bucket_layout([4], [False], 10) == ([None], [])


def _tiny_cfg(golden_loss):
    return SimpleNamespace(**golden_loss["config"])


def test_oracle_init_matches_reference(golden_loss, golden_init_fp):
    torch.manual_seed(golden_loss["seed"])
    m = OM.build(_tiny_cfg(golden_loss))
    sd = m.state_dict()
    assert set(sd) == set(golden_init_fp)
    for k, fp in golden_init_fp.items():
        v = sd[k].double()
        assert float(v.sum()) == pytest.approx(fp["sum"], rel=1e-9, abs=1e-9), k
        assert [float(x) for x in sd[k].flatten()[:16]] == fp["head"], k
    # final_proj is zero at step 0 (ref checkpoint.py:88-91 + model.py:262 quirk)
    assert golden_init_fp["final_proj.weight"]["abs_sum"] == 0.0


def test_oracle_loss_curve_matches_reference(golden_loss):
    """Oracle train loop (fp32 CPU) reproduces the reference's 200-step curve."""
    from picotron_amd.data import synth_tokens
    torch.manual_seed(golden_loss["seed"])
    cfg = _tiny_cfg(golden_loss)
    m = OM.build(cfg)
    opt = torch.optim.AdamW(m.parameters(), lr=golden_loss["lr"])
    gen = torch.Generator().manual_seed(1234)
    mbs, seq, ga = golden_loss["mbs"], golden_loss["seq"], golden_loss["grad_acc"]
    batches = [synth_tokens(mbs, seq + 1, cfg.vocab_size, gen, "arith") for _ in range(16)]
    steps = 60
    k = 0
    for step in range(steps):
        opt.zero_grad()
        mb = []
        for _ in range(ga):
            t = batches[k % 16]
            k += 1
            mb.append((t[:, :-1], t[:, 1:]))
        loss = OM.train_step(m, mb, ga)
        opt.step()
        ref = golden_loss["losses"][step]
        assert abs(loss - ref) < 2e-4 * max(1.0, abs(ref)), (step, loss, ref)
    assert golden_loss["losses"][0] == pytest.approx(math.log(cfg.vocab_size), abs=1e-4)
