"""Training step and loop — semantics of the reference train.py (train_step :29-55, loop :219-259),
on the gfx950 hot path. Data is synthetic (no network); the model is built by
picotron_amd.model.build_llama with the reference's init (seed first)."""
import contextlib
import os
import time

import torch
import torch.nn.functional as F

from . import process_group_manager as pgm
from . import wgrad_pair as WP

# MI355X bf16 dense MFMA peak: 256 CUs x 4096 FLOP/clk x 2.4 GHz (MI355X_MICROARCH.md; the H100
# constant of ref picotron/utils.py:42 is 989.5e12)
MI355X_BF16_PEAK = 256 * 4096 * 2.4e9


def _cross_entropy(outputs, targets):
    """F.cross_entropy (ref train.py:46-49) on the fused HIP kernel for bf16 logits on the GPU."""
    if outputs.is_cuda and outputs.dtype == torch.bfloat16 and outputs.shape[-1] % 8 == 0 and \
            os.getenv("PICO_UNFUSED", "0") != "1":
        from . import ops
        return ops.cross_entropy(outputs, targets)
    return F.cross_entropy(outputs, targets, reduction="mean")


def _fused_lm_head(model):
    """The LM head of `model` (or of the module a DP wrapper holds) when the fused LM head + CE applies:
    our Llama (forward(return_hidden=True)), a bias-free nn.Linear head, bf16 on a HIP device."""
    core = getattr(model, "module", model)
    head = getattr(core, "final_proj", None)
    if os.getenv("PICO_UNFUSED", "0") == "1" or os.getenv("PICO_FUSED_LM_CE", "1") == "0":
        return None
    if not hasattr(core, "decoder_layers") or type(head) is not torch.nn.Linear or head.bias is not None:
        return None
    w = head.weight
    if not w.is_cuda or w.dtype != torch.bfloat16 or w.shape[0] % 8 != 0:
        return None
    return head


def _forward_loss(model, input_ids, target_ids, grad_acc_steps, loss_acc=None):
    """One micro-batch forward to its mean CE / grad_acc (ref train.py:39-49): (loss, folded). folded: the loss
    was already added into loss_acc (fp32 device scalar) by the fused CE's mean launch (the chunked form)."""
    head = _fused_lm_head(model)
    folded = False
    if head is not None:  # fused LM head + cross-entropy: logits never re-read
        from . import ops
        h = model(input_ids=input_ids, return_hidden=True)
        if ops.ce_chunk_rows() > 0:  # chunked: 1 / grad_acc folded into the op (its dW is taken in the forward)
            loss = ops.lm_head_cross_entropy(h, head.weight, target_ids.reshape(-1), grad_scale=1.0 / grad_acc_steps,
                                             loss_acc=loss_acc)
            folded = loss_acc is not None
        else:
            loss = ops.lm_head_cross_entropy(h, head.weight, target_ids.reshape(-1)) / grad_acc_steps
    else:
        outputs = model(input_ids=input_ids)
        batch_size, seq_len = input_ids.shape
        outputs = outputs.view(seq_len * batch_size, -1)
        loss = _cross_entropy(outputs, target_ids.reshape(-1)) / grad_acc_steps
    return loss, folded


def _micro_batch(model, input_ids, target_ids, grad_acc_steps, loss_acc=None):
    """One micro-batch forward + backward (ref train.py:39-51); returns the detached loss. loss_acc (fp32 device
    scalar): += the loss — inside the fused CE's mean launch when the chunked form runs, else one add."""
    loss, folded = _forward_loss(model, input_ids, target_ids, grad_acc_steps, loss_acc)
    loss.backward()
    if loss_acc is not None and not folded:
        loss_acc += loss.detach()
    return loss.detach()


def train_step(model, data_loader, device, graphs=None, sync_loss=True):
    """ref train.py:29-55: grad-accumulation loop, DP sync only on the last micro-batch,
    mean CE / grad_acc_steps, returns the accumulated (python float) loss.
    `graphs` (a MicroBatchGraph) replays the micro-batches that do not sync DP gradients.
    sync_loss=False returns the loss as a device scalar instead: no host synchronisation in the step, so the
    host queues the optimizer step and the next step's launches while the device still runs this one."""
    m = pgm.process_group_manager
    # the reference toggles DP sync only when cp_dp_world_size > 1; a DP wrapper at W = 1 is toggled
    # too (identical sums: all-reducing once at the end == every micro-batch when W = 1)
    requires_grad_sync = (m is not None and m.cp_dp_world_size > 1) or hasattr(model, "require_backward_grad_sync")
    losses = []
    n = data_loader.grad_acc_steps
    grouped = graphs is not None and getattr(graphs, "grouped", False)
    # paired weight gradients (wgrad_pair) need every micro-batch announced with its index: eager micro-batches and
    # the pipelined graph do; MicroBatchGraph replays one captured micro-batch for every index, so not with it
    pair = graphs is None or grouped
    if grouped and getattr(graphs, "n", n) != n:
        # the graph's micro-batch indices (and its wgrad pairing decisions, fixed at capture) are those of n
        raise RuntimeError(f"train_step: the pipelined graph was built for grad_acc {graphs.n}, the loader has {n}")
    if pair:
        WP.begin_step()
    pending = []  # grouped graphs: the non-syncing micro-batches, replayed together before the syncing one

    def run_pending():
        if pending:
            if requires_grad_sync:
                model.require_backward_grad_sync = False
            graphs.run(pending)
            pending.clear()

    for i in range(n):
        batch = next(data_loader)
        input_ids = batch["input_ids"].to(device)
        target_ids = batch["target_ids"].to(device)
        sync = requires_grad_sync and i == n - 1
        if grouped and not sync:
            pending.append((input_ids, target_ids))
            continue
        if grouped and sync and pending and getattr(graphs, "tail_overlap", False) and tail_overlap_enabled():
            # the syncing micro-batch's forward runs beside the graph's last backward (bwd n - 2 on a side stream);
            # its backward, whose hooks launch the RCCL all-reduces, stays eager after both
            def fwd_sync(x=input_ids, y=target_ids, j=i):
                model.require_backward_grad_sync = True
                with (WP.micro_batch(j, n) if pair else contextlib.nullcontext()):
                    return _forward_loss(model, x, y, n)
            model.require_backward_grad_sync = False
            loss, folded = graphs.run(pending, between=fwd_sync)
            pending.clear()
            model.require_backward_grad_sync = True
            with (WP.micro_batch(i, n) if pair else contextlib.nullcontext()):
                loss.backward()
            losses.append(loss.detach())
            continue
        run_pending()
        if requires_grad_sync:
            model.require_backward_grad_sync = sync
        if graphs is not None and not sync:  # syncing micro-batches launch RCCL from hooks: eager
            graphs.replay(input_ids, target_ids)
        else:
            with (WP.micro_batch(i, n) if pair else contextlib.nullcontext()):
                losses.append(_micro_batch(model, input_ids, target_ids, n))
    run_pending()
    if pair and WP.pending_state():
        # a first half whose wgrad GEMM was deferred and never run: its weight gradients would be lost silently
        raise RuntimeError("train_step: paired weight gradients (wgrad_pair) left a deferred first half unconsumed "
                           "(pairing toggled between capture and replay?)")
    if graphs is not None:
        acc = graphs.take_loss()
        if acc is not None:  # None: no graph replay ran this step (e.g. grad_acc 1 under DP: the syncing one only)
            losses.append(acc)
    # one host sync per step instead of one per micro-batch (ref :53 calls .item() each time), or none
    total = torch.stack(losses).float().sum() if losses else torch.zeros((), device=device)
    if not sync_loss:
        return total
    value = float(total.item())
    from . import ops
    ops.check_lm_head_grad_scale()  # the host just synchronised: a free read of the chunked CE's contract flag
    return value


class MicroBatchGraph:
    """A training micro-batch (forward, mean CE / grad_acc, backward) captured once as a HIP graph
    and replayed: the ~330 kernels of a SmolLM-1.7B micro-batch then launch back to back instead of
    paying a host dispatch gap each. Inputs are copied into static buffers, the loss is accumulated
    on the device, and gradients accumulate into persistent buffers — so between steps gradients
    must be zeroed in place (`optimizer.zero_grad(set_to_none=False)`), never dropped. Micro-batches
    that sync DP gradients (RCCL all-reduces launched from hooks) are not replayed; train_step runs
    them eagerly. Capture happens on the first replay: two eager warm-up micro-batches on a side
    stream, then the capture; their effects on gradients / the loss are undone (zeroed), so call it
    at the start of a step (grads zero)."""

    def __init__(self, model, grad_acc_steps, zero_grads):
        self.model = model
        self.n = grad_acc_steps
        self.zero_grads = zero_grads  # callable zeroing every gradient buffer in place
        self.graph = None
        self.inp = self.tgt = None
        self.loss_acc = None

    def _fwd_bwd(self):
        _micro_batch(self.model, self.inp, self.tgt, self.n, loss_acc=self.loss_acc)

    def _capture(self, input_ids, target_ids):
        self.inp = input_ids.clone()
        self.tgt = target_ids.clone()
        self.loss_acc = torch.zeros((), dtype=torch.float32, device=input_ids.device)
        side = torch.cuda.Stream(device=input_ids.device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                self._fwd_bwd()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._fwd_bwd()
        torch.cuda.synchronize()
        self.zero_grads()
        self.loss_acc.zero_()

    def replay(self, input_ids, target_ids):
        from . import ops
        ops.refresh_weight_transposes()  # dgrad W^T copies are graph inputs: bring them up to date
        if self.graph is None:
            self._capture(input_ids, target_ids)
        self.inp.copy_(input_ids)
        self.tgt.copy_(target_ids)
        self.graph.replay()

    def take_loss(self):
        if self.loss_acc is None:
            return None
        out = self.loss_acc.clone()
        self.loss_acc.zero_()
        return out


class PipelinedMicroBatchGraph:
    """The non-syncing micro-batches of a step captured as ONE HIP graph, software-pipelined over two streams:
    the forward of micro-batch i runs beside the backward of micro-batch i - 1, so the GEMMs that cannot fill
    the chip alone (the 2048-wide out / down projections: 128 tiles of 256 x 256 for 256 CUs) and the HBM-bound
    kernels share it with the other micro-batch's work. Results are those of the serial loop bit for bit: the
    backwards stay in micro-batch order (backward i waits for backward i - 1, so every gradient accumulates in
    the same order) and so do the forwards (forward i waits for forward i - 1: the chunked LM-head CE adds its
    weight gradient and the loss in the forward). Same contract as MicroBatchGraph (persistent gradient
    buffers zeroed in place; capture at the start of a step), one replay per step instead of one per
    micro-batch; `train_step` hands it the step's non-syncing micro-batches together (`run`)."""

    grouped = True
    tail_overlap = True  # run(batches, between=...): the split head / tail capture

    def __init__(self, model, grad_acc_steps, zero_grads):
        self.model = model
        self.n = grad_acc_steps
        self.zero_grads = zero_grads
        self.graphs = {}  # number of micro-batches -> (graph, inputs [k, B, S], targets [k, B, S])
        self.loss_acc = None
        self.streams = None
        self.pair_latched = None
        self.tail_stream = None  # the split capture's tail replays here (run(between=...))
        self._tail_state = None

    @property
    def graph(self):
        return next(iter(self.graphs.values()))[0] if self.graphs else None

    def _body(self, inp, tgt, part="all"):
        """Issue the pipeline: part "all"; or "head" (everything but the last backward) then "tail" (that backward),
        captured as two graphs so that the syncing micro-batch's eager forward can run beside the tail (run)."""
        from . import ops
        model, n, acc = self.model, self.n, self.loss_acc
        cur = torch.cuda.current_stream()
        if part == "tail":
            st = self._tail_state
            self._tail_state = None
            k = inp.shape[0]
            s = (cur, self.streams[1])[(k - 1) % 2]
            if s is not cur:
                s.wait_stream(cur)
            st["bwd_done"] = None  # the head ran to its end before the tail starts (stream order)
            self._issue(k, k, model, n, acc, (cur, self.streams[1]), inp, tgt, st)
            if s is not cur:
                cur.wait_stream(s)
            return
        WP.begin_step()  # each run of the body (eager warm-up, capture) issues the step's micro-batches from 0
        # no dgrad / wgrad side-stream pairs (ops.dgrad_wgrad) inside the pipeline: a fork from slot 1's stream
        # crashes the capture (ops.no_side_streams), and on slot 0 alone they measured slower (C2 154.2 -> 152.2 K
        # tokens/s, profiles/r04_ab_pipeline_side0.jsonl): the other micro-batch already fills the chip.
        # Slot 0 runs on the capture stream itself, slot 1 on one stream forked from it: with BOTH slots on
        # forked streams (dependencies in both directions between two forked streams) hipStreamEndCapture
        # segfaults on this ROCm (scripts/dbg_event_capture.py reproduces it with plain tensor ops)
        streams = (cur, self.streams[1])
        streams[1].wait_stream(cur)
        # (a third stream for the grouped weight-gradient GEMMs, waits routed through the capture stream, measured
        # 4.7 % slower: DESIGN.md §4e)
        k = inp.shape[0]
        st = {"losses": [None] * k, "bwd_done": None, "fwd_done": None}
        # (layer-ordered backwards -- backward i entering each layer after backward i - 1 left it -- measured
        # bit-identical and step-neutral in round 5, and removed)
        for i in range(k + 1 if part == "all" else k):
            self._issue(i, k, model, n, acc, streams, inp, tgt, st)
        cur.wait_stream(streams[1])
        if part == "head":
            self._tail_state = st

    def _issue(self, i, k, model, n, acc, streams, inp, tgt, st):
        """Pipeline step i: the backward of micro-batch i - 1 (on its forward's stream, after backward i - 2), then
        the forward of micro-batch i (after forward i - 1)."""
        from . import ops
        losses = st["losses"]
        if i >= 1:
            s = streams[(i - 1) % 2]
            with torch.cuda.stream(s), ops.no_side_streams(), WP.micro_batch(i - 1, n):
                if st["bwd_done"] is not None:
                    s.wait_event(st["bwd_done"])
                loss, folded = losses[i - 1]
                loss.backward()
                if not folded:
                    acc += loss.detach()
                ev = torch.cuda.Event()
                ev.record(s)
                st["bwd_done"] = ev
            losses[i - 1] = None
        if i < k:
            s = streams[i % 2]
            with torch.cuda.stream(s), ops.no_side_streams(), WP.micro_batch(i, n):
                if st["fwd_done"] is not None:
                    s.wait_event(st["fwd_done"])
                losses[i] = _forward_loss(model, inp[i], tgt[i], n, acc)
                ev = torch.cuda.Event()
                ev.record(s)
                st["fwd_done"] = ev

    def _capture(self, batches, split=False):
        dev = batches[0][0].device
        if self.streams is None:
            self.streams = (None, torch.cuda.Stream(device=dev))  # slot 0: the caller's (capture) stream
        inp = torch.stack([b[0] for b in batches])
        tgt = torch.stack([b[1] for b in batches])
        if self.loss_acc is None:
            self.loss_acc = torch.zeros((), dtype=torch.float32, device=dev)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(1 if len(batches) > 1 else 2):  # eager warm-up: at least two micro-batches
                self._body(inp, tgt)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        if split:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._body(inp, tgt, "head")
            head_state = WP.pending_state()
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2, pool=g.pool()):
                self._body(inp, tgt, "tail")
            tail_state = WP.pending_state()
        else:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._body(inp, tgt)
        torch.cuda.synchronize()
        self.zero_grads()
        self.loss_acc.zero_()
        # a first half the graph's last micro-batch leaves deferred (wgrad_pair) for the eager one after it: the
        # replay runs no Python, so run() re-announces it after every replay
        if split:
            self.graphs[(len(batches), True)] = (g, inp, tgt, head_state, g2, tail_state)
        else:
            self.graphs[len(batches)] = (g, inp, tgt, WP.pending_state())
        self.pair_latched = WP.enabled()  # the pairing decisions are baked into the graph

    def run(self, batches, between=None):
        """Replay the graph of these micro-batches. between (callable, optional): issued on the caller's stream while
        the graph's last backward replays on a side stream (the split capture: head graph, then the tail beside
        `between`); its return value is returned. The tail's effects are complete on the caller's stream on return."""
        from . import ops
        ops.refresh_weight_transposes()  # dgrad W^T copies are graph inputs: bring them up to date
        if between is not None:
            key = (len(batches), True)
            if key not in self.graphs:
                self._capture(batches, split=True)
            if WP.enabled() != self.pair_latched:
                raise RuntimeError("PipelinedMicroBatchGraph: PICO_WGRAD_PAIR changed after the graph was captured (its "
                                   "wgrad pairing is fixed at capture); build a new graph")
            g, inp, tgt, head_state, g2, tail_state = self.graphs[key]
            for j, (x, y) in enumerate(batches):
                inp[j].copy_(x)
                tgt[j].copy_(y)
            g.replay()
            WP.restore_pending(head_state)
            cur = torch.cuda.current_stream()
            if self.tail_stream is None:
                self.tail_stream = torch.cuda.Stream(device=inp.device)
            self.tail_stream.wait_stream(cur)
            with torch.cuda.stream(self.tail_stream):
                g2.replay()
            out = between()
            cur.wait_stream(self.tail_stream)
            # the tail's group-state changes (deferrals of the last backward), on top of what `between` changed
            for b, v in tail_state.items():
                if head_state.get(b) != v:
                    b.pending = v
            for b in head_state:
                if b not in tail_state:
                    b.pending = None
            return out
        if len(batches) not in self.graphs:
            self._capture(batches)
        if WP.enabled() != self.pair_latched:
            raise RuntimeError("PipelinedMicroBatchGraph: PICO_WGRAD_PAIR changed after the graph was captured (its "
                               "wgrad pairing is fixed at capture); build a new graph")
        g, inp, tgt, pending = self.graphs[len(batches)]
        for j, (x, y) in enumerate(batches):
            inp[j].copy_(x)
            tgt[j].copy_(y)
        g.replay()
        WP.restore_pending(pending)

    def take_loss(self):
        if self.loss_acc is None:
            return None
        out = self.loss_acc.clone()
        self.loss_acc.zero_()
        return out


def tail_overlap_enabled():
    """PICO_DP_TAIL_OVERLAP (default 1): under a DP wrapper the syncing micro-batch's forward runs beside the
    pipelined graph's last backward (the graph captured as head + tail), only its backward eager after both."""
    return os.getenv("PICO_DP_TAIL_OVERLAP", "1") != "0"


def pipelined_enabled():
    """TrainingStep's graphs replay the step's micro-batches as one two-stream pipelined graph
    (PipelinedMicroBatchGraph; default) — PICO_MB_PIPELINE=0: one MicroBatchGraph replay per micro-batch.
    C2 step, same box, 2 x 2 alternating runs: 865.2 / 866.9 -> 848.8 / 850.0 ms (profiles/r04_ab_pipeline_actt.jsonl)."""
    return os.getenv("PICO_MB_PIPELINE", "1") != "0"


class TrainingStep:
    """One optimizer step of the reference loop (ref train.py:219-240) on this hot path, exactly as bench.py runs
    it: optimizer.zero_grad(), train_step over grad_acc micro-batches (the non-syncing ones replayed from a HIP
    graph when `graphs`; the syncing one eager, since its RCCL all-reduces launch from hooks), optimizer.step(),
    model.reset(). The phases are exposed separately (zero / micro_batches / optimizer_step / reset) so tests can
    inspect the gradients between them."""

    def __init__(self, model, optimizer, loader, device, graphs=True):
        self.model = model
        self.optimizer = optimizer
        self.loader = loader
        self.device = device
        cls = PipelinedMicroBatchGraph if pipelined_enabled() else MicroBatchGraph
        self.graphs = cls(model, loader.grad_acc_steps, self.zero_grads) if graphs else None

    def zero_grads(self):
        """Zero every gradient buffer in place (graph replays keep persistent buffers)."""
        for p in self.model.parameters():
            if p.grad is not None:
                p.grad.zero_()
        if hasattr(self.model, "bucket_manager"):
            self.model.bucket_manager.reset()

    def zero(self):
        # graphs: gradient buffers must persist (zeroed in place); eager: the reference's set_to_none
        self.optimizer.zero_grad(set_to_none=self.graphs is None)

    def micro_batches(self, sync_loss=True):
        return train_step(self.model, self.loader, self.device, graphs=self.graphs, sync_loss=sync_loss)

    def optimizer_step(self):
        self.optimizer.step()

    def reset(self):
        if hasattr(self.model, "reset"):
            self.model.reset()

    def __call__(self, sync_loss=True):
        self.zero()
        loss = self.micro_batches(sync_loss)
        self.optimizer_step()
        self.reset()
        return loss


def get_mfu(tokens_per_second_per_gpu, num_params, model_config, theoretical_flops=MI355X_BF16_PEAK):
    """ref picotron/utils.py:42-48 with the MI355X peak: 6N + 12*L*H*S FLOP per token."""
    flops_per_token = (6 * num_params + 12 * model_config.num_hidden_layers * model_config.hidden_size *
                       model_config.max_position_embeddings)
    return tokens_per_second_per_gpu * flops_per_token / theoretical_flops * 100


def get_num_params(model):
    """Parameter count (tp = 1, single pipeline stage; ref picotron/utils.py:50-79)."""
    return sum(p.numel() for p in model.parameters())
