"""Gradient buckets for data parallelism — MI355X-native rebuild of the reference's
picotron/data_parallel/bucket.py (Bucket :6-57, BucketManager :59-156).

Bucket packing and indexing are identical to the reference (greedy, in module.parameters()
order; `params_to_bucket_location[param] = (start, end, bucket_idx)`; `param.main_grad` is a view
of the bucket's flat fp32 `grad_data`), so layouts are bit-exact.

What changes is the device work around the all-reduce:
  * accumulation `main_grad += grad` is the pico_grad_accum kernel; on the syncing micro-batch it
    also applies the 1/W pre-scale (`(m + g) / W` == the reference's add_ then `grad_data /= W`,
    bit for bit), so the bucket is not swept a second time;
  * the all-reduce is RCCL (torch.distributed "nccl" backend on ROCm) on its own stream, and the
    fp32 -> bf16 unflatten/cast into the params' `.grad` (ref data_parallel.py:165) runs as ONE
    pico_cast_f32_bf16 launch per bucket on a side stream right after that bucket's all-reduce, so
    it overlaps the rest of the backward instead of running after it;
  * `.grad` tensors are persistent views of one bf16 buffer per bucket (same values as the
    reference's fresh `main_grad.to(p.dtype)` allocations).

Device ops go through a small kernel table (`HipBucketKernels`); there is no CPU fallback. The
multi-process CPU tests (gloo) install the oracle's CPU table explicitly with `set_kernels()`.
"""
from typing import List

import torch
import torch.distributed as dist

from .. import _lib


class HipBucketKernels:
    """gfx950 kernels for the bucket's device work (pico_grad_accum / pico_scale_f32 / pico_cast_f32_bf16)."""

    @staticmethod
    def accumulate(main_grad, grad, divide_by):
        if grad.dtype != torch.bfloat16 or main_grad.dtype != torch.float32:
            raise TypeError(f"grad_accum: expected fp32 main_grad += bf16 grad, got {main_grad.dtype} += {grad.dtype}")
        if not grad.is_contiguous():
            grad = grad.contiguous()
        _lib.check(_lib.load().pico_grad_accum(_lib.ptr(main_grad), _lib.ptr(grad), main_grad.numel(),
                                               float(divide_by), _lib.stream_of(main_grad)), "pico_grad_accum")

    @staticmethod
    def scale(buf, divide_by):
        _lib.check(_lib.load().pico_scale_f32(_lib.ptr(buf), buf.numel(), float(divide_by), _lib.stream_of(buf)),
                   "pico_scale_f32")

    @staticmethod
    def cast(src, dst):
        if dst.dtype != torch.bfloat16:
            raise TypeError(f"bucket cast: params must be bf16 on the HIP path, got {dst.dtype}")
        _lib.check(_lib.load().pico_cast_f32_bf16(_lib.ptr(src), _lib.ptr(dst), src.numel(), _lib.stream_of(src)),
                   "pico_cast_f32_bf16")

    @staticmethod
    def zero(buf):
        buf.zero_()


_kernels = HipBucketKernels()


def set_kernels(k):
    """Install the device-op table (tests install the oracle's CPU table for gloo runs)."""
    global _kernels
    _kernels = k if k is not None else HipBucketKernels()


def get_kernels():
    return _kernels


class Bucket:
    def __init__(self, params: List[torch.nn.Parameter], grad_data: torch.Tensor, process_group,
                 grad_out: torch.Tensor = None, defer_cast: bool = False) -> None:
        self.params = set(params)
        self.defer_cast = defer_cast          # the bf16 cast is left to the optimizer (or materialize())
        self.params_with_grad_ready = set()
        self.grad_data = grad_data            # flat fp32 gradients of this bucket
        self.grad_out = grad_out              # flat param-dtype buffer whose views become p.grad
        self.process_group = process_group
        self.process_group_size = dist.get_world_size(group=self.process_group)
        self.handle = None
        self.n_prescaled = 0                  # params whose last accumulate already divided by W
        self.cast_done = None                 # event after the side-stream cast (HIP path)
        self.side_stream = None
        self.timing = False                   # record device events around the all-reduce (comm exposure)
        self.timed = None                     # (ready event, all-reduce done event) of the last sync
        self.reset()

    def sync_gradient(self) -> None:
        """Pre-scale (unless fused into the accumulates), launch the async all-reduce, and queue
        the fp32 -> bf16 cast behind it on the side stream."""
        assert self.handle is None
        if self.n_prescaled == 0:
            _kernels.scale(self.grad_data, self.process_group_size)
        elif self.n_prescaled != len(self.params):
            raise RuntimeError("bucket mixes pre-scaled and unscaled parameters")
        ready = None
        if self.timing and self.grad_data.is_cuda:  # on the compute stream: the bucket's last gradient is queued
            ready = torch.cuda.Event(enable_timing=True)
            ready.record()
        self.handle = dist.all_reduce(self.grad_data, group=self.process_group, async_op=True)
        if ready is not None:  # the all-reduce's completion, seen from a side stream (no effect on the compute one)
            if self.side_stream is None:
                self.side_stream = torch.cuda.Stream(device=self.grad_data.device)
            with torch.cuda.stream(self.side_stream):
                self.handle.wait()
                done = torch.cuda.Event(enable_timing=True)
                done.record(self.side_stream)
            self.timed = (ready, done)
        if self.grad_out is not None and self.grad_data.is_cuda and not self.defer_cast:
            if self.side_stream is None:
                self.side_stream = torch.cuda.Stream(device=self.grad_data.device)
            with torch.cuda.stream(self.side_stream):
                self.handle.wait()  # side stream waits for the RCCL stream (no host block)
                _kernels.cast(self.grad_data, self.grad_out)
                self.cast_done = torch.cuda.Event()
                self.cast_done.record(self.side_stream)

    def reset(self) -> None:
        self.handle = None
        self.cast_done = None
        self.timed = None
        self.n_prescaled = 0
        self.params_with_grad_ready.clear()
        _kernels.zero(self.grad_data)

    def wait(self) -> None:
        assert self.handle is not None, "You should launch an allreduce operation before waiting for it to finish"
        if self.cast_done is not None:
            torch.cuda.current_stream(self.grad_data.device).wait_event(self.cast_done)
        else:
            self.handle.wait()
            if self.grad_out is not None and not self.defer_cast:
                _kernels.cast(self.grad_data, self.grad_out)

    def materialize(self) -> None:
        """The deferred fp32 -> bf16 cast, on the current stream (after wait())."""
        if self.grad_out is not None:
            _kernels.cast(self.grad_data, self.grad_out)

    def mark_param_as_ready(self, param: torch.nn.Parameter, prescaled: bool = False) -> None:
        assert param in self.params and param not in self.params_with_grad_ready, \
            f"param {getattr(param, '_pico_name', '')}{tuple(param.shape)} marked ready twice (or foreign)"
        self.params_with_grad_ready.add(param)
        if prescaled:
            self.n_prescaled += 1
        if len(self.params_with_grad_ready) == len(self.params):
            self.sync_gradient()


class BucketManager:
    def __init__(self, params: List[torch.nn.Parameter], process_group, bucket_size: int,
                 grad_type: torch.dtype = torch.float32, defer_cast: bool = False) -> None:
        self.params = list(params)
        self.defer_cast = defer_cast
        self.device = self.params[0].device
        self.buckets = []
        self.process_group = process_group
        self.process_group_size = dist.get_world_size(group=self.process_group)
        self.params_to_bucket_location = {}
        self.bucket_size = bucket_size
        self.bucket_sizes = None
        self.grad_data_list = []
        self.grad_out_list = []
        self.grad_type = grad_type
        self._initialize_buckets()

    @staticmethod
    def compute_layout(numels, requires_grad, bucket_size):
        """Greedy packing of the reference (ref bucket.py:88-116): a parameter joins the current
        bucket if it fits (the first one always fits an empty bucket), else opens a new bucket.
        Returns ([(start, end, bucket_idx) or None per param], bucket_sizes)."""
        locs = []
        cur_size, cur_idx = 0, 0
        for n, rg in zip(numels, requires_grad):
            if not rg:
                locs.append(None)
                continue
            if cur_size == 0:
                locs.append((0, n, cur_idx))
                cur_size = n
            elif cur_size + n > bucket_size:
                cur_idx += 1
                locs.append((0, n, cur_idx))
                cur_size = n
            else:
                locs.append((cur_size, cur_size + n, cur_idx))
                cur_size += n
        nb = cur_idx + 1 if any(l is not None for l in locs) else 0
        sizes = [0] * nb
        for l in locs:
            if l is not None:
                sizes[l[2]] = max(sizes[l[2]], l[1])
        return locs, sizes

    def _initialize_buckets(self) -> None:
        locs, sizes = self.compute_layout([p.numel() for p in self.params], [p.requires_grad for p in self.params],
                                          self.bucket_size)
        buckets_to_params = [[] for _ in sizes]
        for p, loc in zip(self.params, locs):
            if loc is not None:
                self.params_to_bucket_location[p] = loc
                buckets_to_params[loc[2]].append(p)
        self.bucket_sizes = sizes
        for i, n in enumerate(sizes):
            gd = torch.zeros(n, dtype=self.grad_type, device=self.device)
            pdt = buckets_to_params[i][0].dtype
            go = torch.empty(n, dtype=pdt, device=self.device)
            self.grad_data_list.append(gd)
            self.grad_out_list.append(go)
            self.buckets.append(Bucket(buckets_to_params[i], gd, self.process_group, go, defer_cast=self.defer_cast))
        for param in self.params[::-1]:
            if not param.requires_grad:
                continue
            start, end, b = self.params_to_bucket_location[param]
            param.main_grad = self.grad_data_list[b][start:end].view(param.shape)

    def set_timing(self, on: bool) -> None:
        """Record device events per bucket: when its last gradient was queued (ready) and when its all-reduce
        completed (DataParallelBucket.comm_timing collects them per backward pass)."""
        for b in self.buckets:
            b.timing = bool(on)

    def grad_view(self, param):
        """bf16 view of the synchronised gradient of `param` (becomes param.grad)."""
        start, end, b = self.params_to_bucket_location[param]
        return self.grad_out_list[b][start:end].view(param.shape)

    def reset(self) -> None:
        for bucket in self.buckets:
            bucket.reset()

    def wait(self) -> None:
        for bucket in self.buckets:
            bucket.wait()

    def materialize(self) -> None:
        for bucket in self.buckets:
            bucket.materialize()

    def mark_param_as_ready(self, param: torch.nn.Parameter, prescaled: bool = False) -> None:
        bucket_idx = self.params_to_bucket_location[param][2]
        self.buckets[bucket_idx].mark_param_as_ready(param, prescaled)
