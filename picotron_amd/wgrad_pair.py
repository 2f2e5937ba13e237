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

Groups of G micro-batches (group_size(): 4, or 8 under DataParallelBucket; PICO_WGRAD_GROUP overrides) generalise
the pairs (slot i % G, x^T set (i // G) % 2): the first G - 1 defer and the last runs one GEMM over K = G T tokens —
and, under DataParallelBucket, one fp32 read-modify-write of main_grad per G micro-batches instead of per two.

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


def group_size(weight=None):
    """Micro-batches per weight-gradient GEMM: PICO_WGRAD_GROUP (2 = pairs .. 8) when set; else 8 for a weight
    whose gradient accumulates into DataParallelBucket's fp32 main_grad, 4 otherwise. C2 step, same box, 3
    alternating rounds (profiles/r05_ab_wgrad_group.jsonl): 4 vs 2 — 823.7 -> 818.9 ms, under DataParallelBucket
    854.3 -> 837.3 ms (half the fp32 main_grad read-modify-writes); 8 vs 4 under DataParallelBucket (RCCL W = 1,
    2 alternating rounds, profiles/r06_ab_dp_group.jsonl): 844.5 / 844.3 -> 840.8 / 840.8 ms (plain step 826.8 /
    828.0), group buffers 28.9 -> 57.8 GB; without main_grad 8 measured neutral (round 5)."""
    env = os.getenv("PICO_WGRAD_GROUP")
    if env is None:
        mg = getattr(weight, "main_grad", None)
        return 8 if mg is not None and mg.dtype == torch.float32 else 4
    g = int(env)
    if g < 2 or g > 8:
        raise ValueError(f"PICO_WGRAD_GROUP={g}: 2..8 micro-batches per weight-gradient GEMM")
    return g


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
    """The group buffers of one projection (weight [N, K]) for T tokens per micro-batch and G micro-batches per
    GEMM (G = 2: the pairs)."""

    def __init__(self, N, K, T, dtype, device, G=2):
        self.N, self.K, self.T, self.G = N, K, T, G
        self.xt = [torch.empty((K, G * T), dtype=dtype, device=device) for _ in range(2)]
        self.dy = torch.empty((G * T, N), dtype=dtype, device=device)
        # (x^T set, next slot) of a group whose first members deferred their GEMM to its last member, or None
        self.pending = None

    def xt_slot(self, i):
        """Micro-batch i's x^T: [K, T] view, row stride G T, in set (i // G) % 2, columns of slot i % G."""
        h = i % self.G
        return self.xt[(i // self.G) % 2][:, h * self.T:(h + 1) * self.T]

    def dy_slot(self, i):
        h = i % self.G
        return self.dy[h * self.T:(h + 1) * self.T]


def buf(weight, N, K, T, dtype, device):
    """The pair buffers of `weight` (created on first use; recreated if the shape changed)."""
    b = _get(weight)
    G = group_size(weight)
    if b is None or (b.N, b.K, b.T, b.G) != (N, K, T, G) or b.dy.dtype != dtype or b.dy.device != device:
        if b is not None and b.pending is not None:
            raise RuntimeError("paired weight gradients (wgrad_pair) need the micro-batches of a pair to have one "
                               "shape; a first half is pending in buffers of another shape (PICO_WGRAD_PAIR=0 "
                               "turns the pairing off)")
        b = PairBuf(N, K, T, dtype, device, G)
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
    """Bytes held by every live pair buffer: per projection (weight [N, K], T tokens per micro-batch, G per group)
    two x^T sets [K, G T] and one dy [G T, N] — G (2 K T + T N) elements; SmolLM-1.7B at T = 4096, G = 4: about
    1.8 GB per layer, plus the LM head's when its x^T is grouped (dy [4T, V]: 1.6 GB). bench.py reports it."""
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
    """How the wgrad of `weight` runs for the current micro-batch i: ('skip',) — deferred to the last member of
    its group (micro-batches g0 .. g0 + r - 1, g0 = i - i % G, r = min(G, n - g0)); or ('gemm', dy, x) — one GEMM
    over (dy, x): the group's first r slots, or this micro-batch alone. A member that continues a pending group
    while its own operands are not in its slot copies them there (a fallback: the producers normally write them in
    place); a member with no pending group before it runs its own GEMM."""
    b = _get(weight) if active() else None
    if b is None:
        return ("gemm", dy2, x2)
    i, n = _CTX["i"], _CTX["n"]
    T, G = b.T, b.G
    h = i % G
    s = (i // G) % 2
    r = min(G, n - (i - h))
    mine = (dy2.data_ptr() == b.dy_slot(i).data_ptr() and tuple(dy2.shape) == (T, b.N)
            and x2.data_ptr() == b.xt_slot(i).data_ptr() and tuple(x2.shape) == (T, b.K) and x2.stride() == (1, G * T))
    if b.pending is not None and b.pending != (s, h):
        raise RuntimeError(f"wgrad_pair: micro-batch {i} of {n} reached a projection whose group state is "
                           f"{b.pending} (x^T set, next slot): the deferred weight gradients of that group would be "
                           "lost; the micro-batches of a step must be issued in order (begin_step() drops a group a "
                           "failed step left)")
    if h > 0 and b.pending == (s, h):
        if not mine:
            b.dy_slot(i).copy_(dy2)
            b.xt_slot(i).copy_(x2.t())
        if h < r - 1:
            b.pending = (s, h + 1)
            STATS["deferred"] += 1
            return ("skip",)
        b.pending = None
        STATS["paired"] += 1
        return ("gemm", b.dy[:r * T], b.xt[s][:, :r * T].t())
    if h == 0 and mine and r > 1:
        b.pending = (s, 1)
        STATS["deferred"] += 1
        return ("skip",)
    return ("gemm", dy2, x2)
