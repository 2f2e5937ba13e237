"""Layer-granular ordering of consecutive micro-batches' backward passes (the pipelined micro-batch graph,
train.PipelinedMicroBatchGraph).

The graph's backwards must accumulate every gradient in micro-batch order (results equal to the serial loop bit
for bit). Waiting for the whole previous backward before starting the next one does that, but leaves one stream
alone for the part of each backward that outlasts the other stream's forward. Every gradient accumulation of this
model happens inside one decoder layer's backward (the projections' wgrad GEMMs and groups, the chained norm dw
reductions) or in the embedding's backward after the last layer, so it is enough that micro-batch i enters the
backward of layer b after micro-batch i - 1 has left it: `boundary()` puts an identity on the (delta, residual)
pair at every layer boundary, whose backward records where this micro-batch is and makes its stream wait for
the previous micro-batch's event one boundary further down (for boundary 0, the previous backward's end).

Only active between `Schedule.forward(i)` enter / exit (the model's forward of micro-batch i); otherwise
`boundary()` returns its inputs unchanged and adds no autograd node.
"""
import contextlib

import torch

_ACTIVE = None  # (Schedule, micro-batch index) while a scheduled forward is being issued


class Schedule:
    """Host-side book of one graph body's events: (micro-batch, boundary) -> event recorded when that micro-batch's
    backward passed the boundary; `done[i]`: micro-batch i's whole backward (recorded by the caller)."""

    def __init__(self):
        self.passed = {}
        self.done = {}

    @contextlib.contextmanager
    def forward(self, i):
        global _ACTIVE
        prev, _ACTIVE = _ACTIVE, (self, i)
        try:
            yield
        finally:
            _ACTIVE = prev

    def backward_done(self, i, event):
        self.done[i] = event

    def _pass(self, i, b):
        st = torch.cuda.current_stream()
        ev = torch.cuda.Event()
        ev.record(st)
        self.passed[(i, b)] = ev
        # micro-batch i is about to run layer b - 1's backward (or, at b = 0, the embedding's): micro-batch i - 1
        # must have left it
        prev = self.passed.get((i - 1, b - 1)) if b > 0 else self.done.get(i - 1)
        if prev is not None:
            st.wait_event(prev)


class _Boundary(torch.autograd.Function):
    @staticmethod
    def forward(ctx, sched, i, b, delta, residual):
        ctx.sched, ctx.i, ctx.b = sched, i, b
        return delta.view_as(delta), residual.view_as(residual)

    @staticmethod
    def backward(ctx, g_delta, g_residual):
        ctx.sched._pass(ctx.i, ctx.b)
        return None, None, None, g_delta, g_residual


class _BoundaryFirst(torch.autograd.Function):
    """Boundary 0 (no residual yet: the embedding output is the first layer's only input)."""

    @staticmethod
    def forward(ctx, sched, i, delta):
        ctx.sched, ctx.i = sched, i
        return delta.view_as(delta)

    @staticmethod
    def backward(ctx, g_delta):
        ctx.sched._pass(ctx.i, 0)
        return None, None, g_delta


def boundary(delta, residual, b):
    """The layer-boundary pair, unchanged; under an active schedule, through the ordering identity."""
    if _ACTIVE is None or not torch.is_grad_enabled():
        return delta, residual
    sched, i = _ACTIVE
    if residual is None:
        return _BoundaryFirst.apply(sched, i, delta), None
    return _Boundary.apply(sched, i, b, delta, residual)
