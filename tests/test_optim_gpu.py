"""pico_adamw_bf16 (picotron_amd.optim.AdamW) against torch.optim.AdamW(fused=True), the reference's
optimizer (ref train.py:204-209), on bf16 parameters: same arguments, same steps, same gradients; each
step is compared from identical states (1-ulp bf16 differences would otherwise compound over steps)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _ulp_diff(a, b):
    ai = a.view(torch.int16).to(torch.int32)
    bi = b.view(torch.int16).to(torch.int32)
    return (ai - bi).abs()


@pytest.mark.parametrize("wd,lr", [(0.01, 3e-4), (0.0, 1e-2), (0.1, 1e-3)])
def test_adamw_matches_torch_fused(wd, lr):
    from picotron_amd.optim import AdamW
    torch.manual_seed(0)
    shapes = [(2048,), (6144, 2048), (1000, 3), (7,), (65536 + 8,), (3, 5, 40)]
    base = [torch.randn(s, device="cuda").to(BF) for s in shapes]
    big = torch.randn(1 + 6000, device="cuda").to(BF)
    base.append(big[1:])  # a view whose storage offset is not 16-byte aligned (scalar path)
    ours = [torch.nn.Parameter(t.clone()) for t in base]
    ref = [torch.nn.Parameter(t.clone()) for t in base]
    o1 = AdamW(ours, lr=lr, weight_decay=wd)
    o2 = torch.optim.AdamW(ref, lr=lr, weight_decay=wd, fused=True)
    for step in range(4):
        for a, b in zip(ours, ref):
            g = (torch.randn(a.shape, device="cuda") * (10.0 ** (step - 2))).to(BF)
            a.grad = g.clone()
            b.grad = g.clone()
        o1.step()
        o2.step()
        for a, b in zip(ours, ref):
            for x, y in ((a, b), (o1.state[a]["exp_avg"], o2.state[b]["exp_avg"]),
                         (o1.state[a]["exp_avg_sq"], o2.state[b]["exp_avg_sq"])):
                d = _ulp_diff(x.detach(), y.detach())
                # <= 1 bf16 ulp, except where the moment update cancels to rounding noise (|m| ~ 1e-19
                # from b1 m + (1 - b1) g with b1 m ~ -(1 - b1) g: double vs fp32 FMA order decides)
                bad = (d > 1) & ((x.detach().float() - y.detach().float()).abs() > 1e-12)
                assert not bool(bad.any()), (step, tuple(a.shape), int(d.max()))
                assert float((d > 0).float().mean()) < 1e-3, (step, tuple(a.shape))
                with torch.no_grad():  # re-sync, so each step is compared from identical states
                    x.copy_(y)
    assert set(o1.state[ours[0]]) == set(o2.state[ref[0]])
    assert float(o1.state[ours[0]]["step"]) == 4.0


def test_adamw_rejects_non_bf16():
    from picotron_amd.optim import AdamW
    p = torch.nn.Parameter(torch.randn(16, device="cuda"))
    p.grad = torch.randn(16, device="cuda")
    with pytest.raises(TypeError):
        AdamW([p]).step()


def test_adamw_per_parameter_step_counts():
    """A parameter without a gradient on some steps (frozen for a while, an idle pipeline stage) keeps its
    own step count, as torch.optim.AdamW does: same result as torch's fused AdamW."""
    from picotron_amd.optim import AdamW
    torch.manual_seed(1)
    base = [torch.randn(s, device="cuda").to(BF) for s in [(512,), (64, 32), (300,)]]
    ours = [torch.nn.Parameter(t.clone()) for t in base]
    ref = [torch.nn.Parameter(t.clone()) for t in base]
    o1 = AdamW(ours, lr=1e-2, weight_decay=0.01)
    o2 = torch.optim.AdamW(ref, lr=1e-2, weight_decay=0.01, fused=True)
    for step in range(5):
        for i, (a, b) in enumerate(zip(ours, ref)):
            if i == 1 and step in (0, 2):  # parameter 1 idles on steps 0 and 2
                a.grad = b.grad = None
                continue
            g = torch.randn(a.shape, device="cuda").to(BF)
            a.grad = g.clone()
            b.grad = g.clone()
        o1.step()
        o2.step()
        for a, b in zip(ours, ref):
            d = _ulp_diff(a.detach(), b.detach())
            bad = (d > 1) & ((a.detach().float() - b.detach().float()).abs() > 1e-12)
            assert not bool(bad.any()), (step, tuple(a.shape), int(d.max()))
            with torch.no_grad():
                a.copy_(b)
                if b in o2.state:
                    o1.state[a]["exp_avg"].copy_(o2.state[b]["exp_avg"])
                    o1.state[a]["exp_avg_sq"].copy_(o2.state[b]["exp_avg_sq"])
    assert [float(o1.state[p]["step"]) for p in ours] == [5.0, 3.0, 5.0]
    assert [float(o2.state[p]["step"]) for p in ref] == [5.0, 3.0, 5.0]


def test_adamw_bad_step_leaves_state_untouched():
    from picotron_amd.optim import AdamW
    p = torch.nn.Parameter(torch.randn(16, device="cuda").to(BF))
    q = torch.nn.Parameter(torch.randn(16, device="cuda"))  # fp32: rejected
    p.grad = torch.randn(16, device="cuda").to(BF)
    q.grad = torch.randn(16, device="cuda")
    opt = AdamW([p, q])
    with pytest.raises(TypeError):
        opt.step()
    assert not opt.state[p]  # nothing was initialised or incremented
