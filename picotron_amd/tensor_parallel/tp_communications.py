"""Tensor-parallel collectives (API of ref picotron/tensor_parallel/tp_communications.py:8-108): the
Megatron f / g regions and the column-parallel linear with the input-gradient all-reduce overlapped
with the weight-gradient GEMM.

MI355X-native: the collectives are RCCL over xGMI (torch.distributed "nccl" backend on ROCm) on the tp
group, in place on the activation dtype as the reference does (one bf16 rounding of the sum); the GEMMs
are picotron_amd.ops (hipBLASLt with the weight-gradient accumulation fused into the GEMM epilogue,
dgrad against the cached W^T). On a gloo group (the multi-rank tests that share one GPU, which RCCL
refuses) bf16 tensors are summed in fp32 and rounded once — the same value the reference's two-rank sum
has — because gloo has no bf16 reduction.
"""
from typing import Tuple

import torch
import torch.distributed as dist

from .. import ops
from .. import process_group_manager as pgm


def merge_first_two_dims(grad_output: torch.Tensor, input_: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """ref :8-10."""
    return grad_output.contiguous().view(-1, *grad_output.shape[2:]), input_.contiguous().view(-1, *input_.shape[2:])


def split_tensor_along_last_dim(tensor, num_partitions):
    """ref :12-17."""
    last_dim = tensor.dim() - 1
    assert tensor.size()[last_dim] % num_partitions == 0, f"{tensor.size()[last_dim]} is not divisible by {num_partitions}"
    return torch.split(tensor, tensor.size()[last_dim] // num_partitions, dim=last_dim)


def _gloo(group):
    return dist.get_backend(group) == "gloo"


def all_reduce_(t, group=None, async_op=False):
    """In-place SUM over the tp group; returns the work handle when async_op (RCCL)."""
    group = pgm.process_group_manager.tp_group if group is None else group
    if _gloo(group) and t.dtype in (torch.bfloat16, torch.float16):
        t32 = t.float()
        dist.all_reduce(t32, op=dist.ReduceOp.SUM, group=group)
        t.copy_(t32)
        return None
    return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=async_op)


def all_gather_last_dim(x, group=None):
    group = pgm.process_group_manager.tp_group if group is None else group
    m = pgm.process_group_manager
    x = x.contiguous()
    src = x.float() if _gloo(group) and x.dtype in (torch.bfloat16, torch.float16) else x
    parts = [torch.empty_like(src) for _ in range(m.tp_world_size)]
    dist.all_gather(parts, src, group=group)
    parts[m.tp_rank] = src
    return torch.cat(parts, dim=x.dim() - 1).to(x.dtype).contiguous()


class CopyToModelParallelRegion(torch.autograd.Function):
    """f: identity forward, all-reduce of the input gradient backward (ref :19-33)."""

    @staticmethod
    def forward(ctx, x):
        return x

    @staticmethod
    def backward(ctx, grad_output):
        if pgm.process_group_manager.tp_world_size == 1:
            return grad_output
        grad_output = grad_output.contiguous()
        all_reduce_(grad_output)
        return grad_output


class ReduceFromModelParallelRegion(torch.autograd.Function):
    """g: all-reduce forward (in place, as ref :35-48), identity backward."""

    @staticmethod
    def forward(ctx, x):
        if pgm.process_group_manager.tp_world_size == 1:
            return x
        all_reduce_(x)
        return x

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output


class GatherFromModelParallelRegion(torch.autograd.Function):
    """All-gather along the last dim forward, keep this rank's split backward (ref :50-72)."""

    @staticmethod
    def forward(ctx, x):
        if pgm.process_group_manager.tp_world_size == 1:
            return x
        return all_gather_last_dim(x)

    @staticmethod
    def backward(ctx, grad_output):
        m = pgm.process_group_manager
        if m.tp_world_size == 1:
            return grad_output
        return split_tensor_along_last_dim(grad_output, m.tp_world_size)[m.tp_rank].contiguous()


class LinearWithAsyncAllReduce(torch.autograd.Function):
    """Column-parallel y = x W^T (+ b) whose backward launches the input-gradient all-reduce
    asynchronously and runs the weight-gradient GEMM while it is in flight (ref :74-101). The wgrad GEMM
    accumulates into the parameter's gradient storage (ops.wgrad_accumulate) when it can."""

    @staticmethod
    def forward(ctx, input_, weight, bias):
        x2 = input_.reshape(-1, input_.shape[-1])
        ctx.save_for_backward(x2, weight)
        ctx.use_bias = bias is not None
        ctx.xshape = input_.shape
        out = torch.nn.functional.linear(input_, weight, bias)
        return out

    @staticmethod
    def backward(ctx, grad_output):
        x2, weight = ctx.saved_tensors
        dy2 = grad_output.reshape(-1, grad_output.shape[-1])
        grad_input = ops.dgrad(dy2, weight, (weight,)).view(ctx.xshape)
        handle = None
        if pgm.process_group_manager.tp_world_size > 1:
            handle = all_reduce_(grad_input, async_op=True)
        grad_weight = ops.wgrad_accumulate((weight,), dy2, x2)[0] if ctx.needs_input_grad[1] else None
        grad_bias = dy2.sum(0) if ctx.use_bias else None
        if handle is not None:
            handle.wait()
        return grad_input, grad_weight, grad_bias


def linear_with_all_reduce(x, weight, bias):
    """ref :103-106: f then x W_i^T (+ b_i)."""
    input_parallel = CopyToModelParallelRegion.apply(x)
    if bias is None and input_parallel.is_cuda:
        return ops.linear(input_parallel, weight)
    return torch.nn.functional.linear(input_parallel, weight, bias)


def linear_with_async_all_reduce(x, weight, bias):
    """ref :107-108."""
    return LinearWithAsyncAllReduce.apply(x, weight, bias)
