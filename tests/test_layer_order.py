"""Host logic of picotron_amd.layer_order (CPU): the layer-boundary identity is a no-op outside a schedule and an
identity autograd node inside one. Its ordering effect (backward waits on device events) is GPU-only:
tests/test_model_gpu.py::test_layer_ordered_backwards_match."""
import torch

from picotron_amd import layer_order as LO


def test_boundary_is_a_no_op_without_a_schedule():
    d = torch.randn(4, 8, requires_grad=True)
    r = torch.randn(4, 8, requires_grad=True)
    d2, r2 = LO.boundary(d, r, 3)
    assert d2 is d and r2 is r
    d2, r2 = LO.boundary(d, None, 0)
    assert d2 is d and r2 is None


def test_boundary_under_a_schedule_is_an_identity_node():
    sched = LO.Schedule()
    d = torch.randn(4, 8, requires_grad=True)
    r = torch.randn(4, 8, requires_grad=True)
    with sched.forward(5):
        d2, r2 = LO.boundary(d, r, 2)
        e2, none = LO.boundary(d, None, 0)
    assert LO._ACTIVE is None  # the context restores the inactive state
    assert torch.equal(d2, d) and torch.equal(r2, r) and torch.equal(e2, d) and none is None
    assert d2.grad_fn is not None and "Boundary" in type(d2.grad_fn).__name__
    assert e2.grad_fn is not None and "BoundaryFirst" in type(e2.grad_fn).__name__
    with sched.forward(0), torch.no_grad():  # no autograd node when gradients are off
        d3, r3 = LO.boundary(d, r, 1)
    assert d3 is d and r3 is r
