"""Paired weight gradients: the wgrad GEMMs of two consecutive micro-batches as ONE GEMM over both.

The reference accumulates every projection's weight gradient once per micro-batch (ref train.py:33-51: one
backward per micro-batch, AccumulateGrad / main_grad.add_ per parameter). Here the producers of a projection's
two wgrad operands — its input x (kept as x^T: the RMSNorm's y^T, the attention's O^T, the SwiGLU's h^T) and its
output gradient dy (the attention backward's dq|dk|dv, the SwiGLU backward's dgate|dup, the RMSNorm backward's
dx) — write straight into per-projection pair buffers, micro-batch i into half i % 2:

    x^T pair  [K, 2T]  (two sets, alternating per pair: the forward of pair p + 1 may run beside the backward
                        of pair p in the pipelined graph, so it must not overwrite pair p's x^T)
    dy pair   [2T, N]  (one set: the backwards run in micro-batch order)

The first micro-batch of a pair then skips its wgrad GEMM and the second runs dW (+)= dy_pair^T x_pair over
K = 2T tokens — hipBLASLt runs the doubled-K GEMM 3-17 % faster than two GEMMs (scripts/gemm_wgrad_k_probe.py),
with no copy: the operands are already adjacent. dW is the same sum, accumulated in one fp32 GEMM instead of two
(one bf16 rounding of the .grad accumulate per pair instead of per micro-batch). A micro-batch without a partner
(the last of an odd grad_acc) runs its own GEMM, as does a first half whose operands are not in its pair halves
(the pairing is verified per GEMM by pointer, never assumed); a second half whose own operands are elsewhere while
its first half is pending copies them in and runs the pair GEMM.

Active only inside train.train_step / PipelinedMicroBatchGraph, which announce each micro-batch
(`micro_batch(i, n)`), and with PICO_WGRAD_PAIR != 0. Not under MicroBatchGraph: its one captured micro-batch
is replayed for every index.
"""
import contextlib
import os
import weakref

import torch

_CTX = {"i": None, "n": None}  # the micro-batch being issued (forward or backward), or None: pairing off
STATS = {"deferred": 0, "paired": 0}  # GEMM decisions since import (tests)
_BUFS = {}  # id(weight Parameter) -> (weakref to it, PairBuf); the entry goes with the weight


def _get(weight):
    e = _BUFS.get(id(weight))
    return e[1] if e is not None and e[0]() is weight else None


def _put(weight, b):
    key = id(weight)
    _BUFS[key] = (weakref.ref(weight, lambda _r, k=key: _BUFS.pop(k, None)), b)


def enabled():
    return os.getenv("PICO_WGRAD_PAIR", "1") != "0"


@contextlib.contextmanager
def micro_batch(i, n):
    """Announce micro-batch i of n (forward and backward issue both run inside it)."""
    prev = (_CTX["i"], _CTX["n"])
    _CTX["i"], _CTX["n"] = (i, n) if enabled() else (None, None)
    try:
        yield
    finally:
        _CTX["i"], _CTX["n"] = prev


def active():
    return _CTX["i"] is not None


def begin_step():
    """Drop any half-pair a previous step left pending (a step that raised between a pair's two backwards)."""
    for _, b in list(_BUFS.values()):
        b.pending = None


def pending_state():
    """{PairBuf: pending set} — what a captured graph leaves deferred at its end (restored after each replay: the
    replay runs no Python, so the eager micro-batch after it must be told its first half is pending)."""
    return {b: b.pending for _, b in list(_BUFS.values()) if b.pending is not None}


def restore_pending(state):
    for b, v in state.items():
        b.pending = v


class PairBuf:
    """The pair buffers of one projection (weight [N, K]) for T tokens per micro-batch."""

    def __init__(self, N, K, T, dtype, device):
        self.N, self.K, self.T = N, K, T
        self.xt = [torch.empty((K, 2 * T), dtype=dtype, device=device) for _ in range(2)]
        self.dy = torch.empty((2 * T, N), dtype=dtype, device=device)
        self.pending = None  # the x^T set of a first half whose GEMM was deferred to the second

    def xt_slot(self, i):
        """Micro-batch i's x^T: [K, T] view, row stride 2T, in set (i // 2) % 2, columns of half i % 2."""
        h = i % 2
        return self.xt[(i // 2) % 2][:, h * self.T:(h + 1) * self.T]

    def dy_slot(self, i):
        h = i % 2
        return self.dy[h * self.T:(h + 1) * self.T]


def buf(weight, N, K, T, dtype, device):
    """The pair buffers of `weight` (created on first use; recreated if the shape changed)."""
    b = _get(weight)
    if b is None or (b.N, b.K, b.T) != (N, K, T) or b.dy.dtype != dtype or b.dy.device != device:
        if b is not None and b.pending is not None:
            raise RuntimeError("paired weight gradients (wgrad_pair) need the micro-batches of a pair to have one "
                               "shape; a first half is pending in buffers of another shape (PICO_WGRAD_PAIR=0 "
                               "turns the pairing off)")
        b = PairBuf(N, K, T, dtype, device)
        _put(weight, b)
    return b


def xt_out(weight, N, K, T, dtype, device):
    """Where the producer of `weight`'s input should write x^T for the current micro-batch ([K, T] view with row
    stride 2T), or None when pairing is off."""
    if not active() or weight is None:
        return None
    return buf(weight, N, K, T, dtype, device).xt_slot(_CTX["i"])


def dy_out(weight, N, K, T, dtype, device):
    """Where the producer of `weight`'s output gradient should write dy for the current micro-batch ([T, N],
    contiguous), or None when pairing is off."""
    if not active() or weight is None:
        return None
    return buf(weight, N, K, T, dtype, device).dy_slot(_CTX["i"])


def dy_out_existing(weight, N, K, T, dtype, device):
    """dy_out, but only into pair buffers that already exist with this shape (created by the forward's x^T
    producer); None otherwise — a backward never creates the buffers for a projection the forward did not pair."""
    if not active() or weight is None:
        return None
    b = _get(weight)
    if b is None or (b.N, b.K, b.T) != (N, K, T) or b.dy.dtype != dtype or b.dy.device != device:
        return None
    return b.dy_slot(_CTX["i"])


def footprint_bytes():
    """Bytes held by every live pair buffer: per projection (weight [N, K], T tokens per micro-batch) two x^T sets
    [K, 2T] and one dy [2T, N] — (4 K T + 2 T N) elements; SmolLM-1.7B at T = 4096: about 0.9 GB per layer."""
    return sum(sum(x.numel() * x.element_size() for x in b.xt) + b.dy.numel() * b.dy.element_size()
               for _, b in list(_BUFS.values()))


def release():
    """Free every pair buffer (after training; a graph captured on them must not be replayed afterwards)."""
    for _, b in list(_BUFS.values()):
        if b.pending is not None:
            raise RuntimeError("wgrad_pair.release: a deferred first half is still pending")
    _BUFS.clear()


def dy_out_if_paired(weight, x2, N, K, T, dtype, device):
    """dy_out, but only when this micro-batch's x^T of `weight` (x2, the [T, K] view its backward saved) sits in the
    weight's pair buffer — i.e. the forward paired it; otherwise None (no buffers created for unpaired paths)."""
    if not active() or weight is None:
        return None
    b = _get(weight)
    if b is None or (b.N, b.K, b.T) != (N, K, T) or x2.data_ptr() != b.xt_slot(_CTX["i"]).data_ptr():
        return None
    return b.dy_slot(_CTX["i"])


def plan(weight, dy2, x2):
    """How the wgrad of `weight` runs for the current micro-batch: ('skip',) — first half, deferred; or
    ('gemm', dy, x) — one GEMM over (dy, x): the pair, or this micro-batch alone. A second half whose own operands
    are not in the pair buffers while its first half is pending copies them there (a fallback: the producers
    normally write them in place)."""
    b = _get(weight) if active() else None
    if b is None:
        return ("gemm", dy2, x2)
    i, n = _CTX["i"], _CTX["n"]
    T = b.T
    h = i % 2
    mine = (dy2.data_ptr() == b.dy_slot(i).data_ptr() and tuple(dy2.shape) == (T, b.N)
            and x2.data_ptr() == b.xt_slot(i).data_ptr() and tuple(x2.shape) == (T, b.K) and x2.stride() == (1, 2 * T))
    if h == 0:
        if mine and i + 1 < n:
            b.pending = (i // 2) % 2
            STATS["deferred"] += 1
            return ("skip",)
        return ("gemm", dy2, x2)
    s = (i // 2) % 2
    if b.pending is not None and b.pending == s:
        b.pending = None
        if not mine:
            b.dy_slot(i).copy_(dy2)
            b.xt_slot(i).copy_(x2.t())
        STATS["paired"] += 1
        return ("gemm", b.dy, b.xt[s].t())
    return ("gemm", dy2, x2)
