"""Data-parallel wrappers — same API as the reference picotron/data_parallel/data_parallel.py:
DataParallelNaive (:10-60) and DataParallelBucket (:62-171).

DataParallelBucket keeps the reference's contract (attributes `.module`,
`.require_backward_grad_sync`, `.bucket_manager`; `forward`, `backward(input, output, output_grad)`
for pipeline parallelism, `no_sync()`, `reset()`; fp32 `param.main_grad` views; after a syncing
backward every param's `.grad` holds the bf16 average). Per-parameter post-accumulate hooks
(the reference hooks the AccumulateGrad node, ref :93-116; torch's
register_post_accumulate_grad_hook is the same event) run on the autograd device thread:
  * `main_grad += grad` on the pico_grad_accum kernel, fused with the 1/W pre-scale when syncing;
  * when a bucket's last param arrives, its RCCL all-reduce is launched asynchronously and its
    bf16 cast is queued behind it on a side stream (see bucket.py);
  * the post-backward callback makes the compute stream wait for every bucket and hands out the
    `.grad` views.
"""
import contextlib
import weakref

import torch
import torch.distributed as dist
from torch import nn
from torch.autograd import Variable

from .. import process_group_manager as pgm
from .bucket import BucketManager


class DataParallelNaive(nn.Module):
    """Per-gradient all-reduce (ref :10-60; kept for API completeness, unused by the trainer)."""

    def __init__(self, module):
        super().__init__()
        self.module = module
        self.require_backward_grad_sync = True
        self.register_backward_hook(self._allreduce_grads)

    def forward(self, *inputs, **kwargs):
        return self.module(*inputs, **kwargs)

    def register_backward_hook(self, hook):
        for p in self.module.parameters():
            if p.requires_grad is True:
                p.register_hook(hook)

    def _allreduce_grads(self, grad):
        if self.require_backward_grad_sync:
            dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=pgm.process_group_manager.cp_dp_group)
            grad /= pgm.process_group_manager.cp_dp_world_size
        return grad

    @contextlib.contextmanager
    def no_sync(self):
        self.require_backward_grad_sync = False
        yield
        self.require_backward_grad_sync = True


# DataParallelBucket wrappers with defer_grad_cast=True. A global optimizer step pre-hook runs their deferred
# fp32 -> bf16 .grad cast before any optimizer that does not read the fp32 main_grad itself (everything but
# picotron_amd.optim.AdamW) steps, so torch.optim optimizers see the same .grad as with the eager cast.
_DEFERRING = weakref.WeakSet()
_DEFER_HOOK = []


def _materialize_before_foreign_step(optimizer, args, kwargs):
    if getattr(optimizer, "reads_deferred_grads", False):
        return
    for dp in list(_DEFERRING):
        dp.materialize_grads()


class DataParallelBucket(nn.Module):

    def __init__(self, module, bucket_cap_mb=25, grad_type=torch.float32, defer_grad_cast=False):
        """ref :62-85. defer_grad_cast (an extension, off by default): after a syncing backward `.grad` is the
        bucket's bf16 view WITHOUT the fp32 -> bf16 cast of ref :165 having run; picotron_amd.optim.AdamW reads
        the averaged fp32 main_grad instead and rounds it to bf16 in register exactly as the cast would
        (bit-identical step, no bf16 .grad write + re-read: 4 B per parameter per step). Any other optimizer gets
        the cast run for it by a step pre-hook before it steps; code that reads `.grad` outside an optimizer step
        (clip_grad_norm_, grad-norm logging, checkpointing grads) must call materialize_grads() first."""
        super().__init__()
        self.module = module
        self.require_backward_grad_sync = True
        self.defer_grad_cast = bool(defer_grad_cast)
        if self.defer_grad_cast:
            _DEFERRING.add(self)
            if not _DEFER_HOOK:
                from torch.optim.optimizer import register_optimizer_step_pre_hook
                _DEFER_HOOK.append(register_optimizer_step_pre_hook(_materialize_before_foreign_step))
        grad_size = 2 if grad_type == torch.bfloat16 else 4
        bucket_size = bucket_cap_mb * 1024 * 1024 // grad_size
        self.bucket_manager = BucketManager(module.parameters(), pgm.process_group_manager.cp_dp_group, bucket_size,
                                            grad_type, defer_cast=self.defer_grad_cast)
        self._fused_pass = set()  # params a fused producer accumulated in the running backward pass
        self._pass_cb_set = False
        self.register_backward_hook()
        self._post_backward_callback_set = False
        self._comm_log = None
        self._anchor = None

    def comm_timing(self, on: bool) -> None:
        """Start (True) or stop (False) recording, per syncing backward pass, device events at the end of the
        backward's kernels, at each bucket's readiness and all-reduce completion, and after the post-backward
        wait — the communication the step does not hide (comm_report)."""
        if on and self.bucket_manager.device.type != "cuda":
            raise RuntimeError("DataParallelBucket.comm_timing: device events need the HIP device")
        self._comm_log = [] if on else None
        self.bucket_manager.set_timing(on)

    def comm_report(self):
        """Per recorded syncing backward (after a device synchronize): {"exposed_ms": end of backward -> end of
        the post-backward wait, "buckets": [(ready_ms, allreduce_done_ms, bytes)] relative to the end of the
        backward (negative: before it), in bucket order}.
        A pass recorded without an anchor (timing switched on partway through it) is skipped; a bucket that did not
        sync in a pass reports (None, None, bytes)."""
        out = []
        for a, t0, t1, bk in self._comm_log or []:
            if a is None or t0 is None or t1 is None:
                continue
            end = a.elapsed_time(t0)  # every time from the anchor (elapsed times are taken forward only)
            rows = [(a.elapsed_time(tm[0]) - end, a.elapsed_time(tm[1]) - end, nb) if tm is not None else
                    (None, None, nb) for tm, nb in bk]
            out.append({"exposed_ms": t0.elapsed_time(t1), "buckets": rows})
        return out

    def forward(self, *inputs, **kwargs):
        # per-pass state left by a backward that raised midway (its end-of-pass callbacks never ran) is dropped
        # here — unless this forward itself runs inside a backward pass (activation recompute, a
        # forward from a hook), whose state is live
        if torch._C._current_graph_task_id() == -1:
            self._end_pass()
            self._post_backward_callback_set = False
        return self.module(*inputs, **kwargs)

    def backward(self, input_tensor, output_tensor, output_tensor_grad):
        return self.module.backward(input_tensor, output_tensor, output_tensor_grad)

    def register_backward_hook(self):
        self.grad_accs = []
        for name, param in self.module.named_parameters():
            param._pico_name = name  # error messages only
            if param.requires_grad:
                self.grad_accs.append(param.register_post_accumulate_grad_hook(
                    self._make_param_hook(param, self.bucket_manager)))
                # fused path (ops.wgrad_accumulate): the wgrad GEMM accumulated into main_grad itself
                param._pico_wgrad_sync = self._wgrad_sync
                param._pico_wgrad_ready = self._make_ready_fn(param, self.bucket_manager)

    def _make_param_hook(self, param, bucket_manager):
        from .bucket import get_kernels
        world = bucket_manager.process_group_size

        def param_hook(*unused):
            # A producer that accumulated into main_grad itself (fused wgrad GEMM, RMSNorm dw, embedding
            # backward: ops.wgrad_accumulate / _norm_grad_target) hands autograd no gradient and records the
            # param in this backward pass's fused set (ready()); AccumulateGrad still calls post-accumulate
            # hooks for a None gradient, and with persistent .grad buffers (HIP-graph replay, set_to_none=
            # False) param.grad is not None then, so the set — not the .grad — says there is nothing to add.
            # The set is cleared at the end of every backward pass, so nothing carries over between
            # micro-batches: a param may switch between the fused and the hook path at any micro-batch
            # (PICO_WGRAD_FUSION toggled, a non-contiguous main_grad, TP layers swapped in).
            if param.grad is None or param in self._fused_pass:
                return
            if param.requires_grad:
                sync = self.require_backward_grad_sync
                # fold the bucket's 1/W pre-scale into this (final) accumulate when syncing
                get_kernels().accumulate(param.main_grad, param.grad, world if sync else 1)
                param.grad = None
                if sync:
                    self._queue_post_backward()
                    bucket_manager.mark_param_as_ready(param, prescaled=True)
        return param_hook

    def _end_pass(self):
        self._fused_pass.clear()
        self._pass_cb_set = False

    def _wgrad_sync(self):
        return self.require_backward_grad_sync, self.bucket_manager.process_group_size

    def _make_ready_fn(self, param, bucket_manager):
        def ready():
            # the GEMM already did main_grad = (main_grad + dW) / W on the syncing micro-batch
            self._fused_pass.add(param)
            if not self._pass_cb_set:
                Variable._execution_engine.queue_callback(self._end_pass)
                self._pass_cb_set = True
            if self.require_backward_grad_sync:
                self._queue_post_backward()
                bucket_manager.mark_param_as_ready(param, prescaled=True)
        return ready

    @contextlib.contextmanager
    def no_sync(self):
        self.require_backward_grad_sync = False
        yield
        self.require_backward_grad_sync = True

    def _queue_post_backward(self):
        if not self._post_backward_callback_set:
            Variable._execution_engine.queue_callback(self._post_backward)
            self._post_backward_callback_set = True
            if self._comm_log is not None:  # timing anchor: before the pass's first bucket can be ready
                self._anchor = torch.cuda.Event(enable_timing=True)
                self._anchor.record()

    def _post_backward(self):
        t0 = None
        if self._comm_log is not None:  # end of the backward's kernels on the compute stream
            t0 = torch.cuda.Event(enable_timing=True)
            t0.record()
        self.bucket_manager.wait()
        if t0 is not None:  # the compute stream has waited for every bucket's all-reduce (and cast)
            t1 = torch.cuda.Event(enable_timing=True)
            t1.record()
            bm = self.bucket_manager
            self._comm_log.append((self._anchor, t0, t1, [(b.timed, b.grad_data.numel() * b.grad_data.element_size())
                                                         for b in bm.buckets]))
        self._post_backward_callback_set = False
        for p in self.module.parameters():
            if p.requires_grad:
                p.grad = self.bucket_manager.grad_view(p)
                if self.defer_grad_cast:  # the optimizer reads main_grad (see __init__)
                    p._pico_grad_f32 = p.main_grad
                    p._pico_grad_deferred = True

    def materialize_grads(self):
        """Run the deferred bf16 cast (defer_grad_cast=True) so `.grad` holds the averaged gradient."""
        if any(getattr(p, "_pico_grad_deferred", False) for p in self.module.parameters()):
            self.bucket_manager.materialize()
            self._clear_deferred()

    def _clear_deferred(self):
        for p in self.module.parameters():
            if getattr(p, "_pico_grad_deferred", False):
                p._pico_grad_deferred = False

    def reset(self):
        self.bucket_manager.reset()
        self._clear_deferred()
        self._end_pass()
        self._post_backward_callback_set = False
