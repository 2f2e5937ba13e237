"""AdamW on the gfx950 pico_adamw_bf16 kernel: one launch updates every parameter.

Drop-in for the reference's optimizer, `torch.optim.AdamW(model.parameters(), lr=..., fused=...)`
(ref train.py:13,204-209; stepped at :235, zeroed at :221): same constructor arguments and defaults,
same `param_groups` / `state` layout (`step`, `exp_avg`, `exp_avg_sq` per parameter, states in the
parameter dtype), so checkpoints and LR schedules see a torch AdamW. The update has ATen's fused
AdamW expression order and types (decoupled weight decay; see csrc/adamw.hip). Parameters and
gradients must be bf16 HIP tensors (the training dtype of the hot path); anything else raises —
there is no CPU or eager fallback.
"""
import torch

from . import _lib


def _deferred_grad(p):
    """The fp32 main_grad the step reads instead of .grad when DataParallelBucket(defer_grad_cast=True) left
    the bf16 .grad cast to the optimizer (the kernel rounds it to bf16 in register, as the cast would)."""
    g32 = getattr(p, "_pico_grad_f32", None)
    if g32 is None or not getattr(p, "_pico_grad_deferred", False):
        return None
    if g32.dtype != torch.float32 or not g32.is_contiguous() or g32.shape != p.shape:
        raise ValueError("picotron_amd.optim.AdamW: deferred-cast gradient must be a contiguous fp32 main_grad")
    return g32


class AdamW(torch.optim.Optimizer):
    # reads DataParallelBucket(defer_grad_cast=True)'s fp32 main_grad itself: the bucket's step pre-hook leaves
    # the deferred cast to this optimizer (see data_parallel.py)
    reads_deferred_grads = True

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, amsgrad=False, *,
                 maximize=False, foreach=None, capturable=False, differentiable=False, fused=None):
        if amsgrad or maximize or capturable or differentiable:
            raise NotImplementedError("picotron_amd.optim.AdamW: amsgrad / maximize / capturable / differentiable")
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"invalid AdamW hyper-parameters lr={lr} betas={betas} eps={eps}")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False, maximize=False,
                        foreach=None, capturable=False, differentiable=False, fused=fused)
        super().__init__(params, defaults)
        # per (group, parameter set): device tables of sizes / 64 Ki-element chunks (fixed for the set) and of
        # the (param, grad, exp_avg, exp_avg_sq) pointers, re-uploaded only when a pointer changed (persistent
        # gradients: never after the first step); two pinned staging buffers used in turn
        self._tables = {}

    def _group_tables(self, gi, params):
        # keyed by pointer AND size: a parameter re-pointed at a different-sized tensor that the caching
        # allocator placed at the same address gets new size / chunk tables
        key = (gi, tuple((p.data_ptr(), p.numel()) for p in params))
        ent = self._tables.get(key)
        if ent is None:
            chunk = int(_lib.load().pico_adamw_chunk_elems())
            dev = params[0].device
            sizes = torch.tensor([p.numel() for p in params], dtype=torch.int64)
            chunks = torch.tensor([(i, c) for i, p in enumerate(params) for c in range(0, p.numel(), chunk)],
                                  dtype=torch.int64).reshape(-1, 2)
            ent = {"tens": torch.empty((len(params), 5), dtype=torch.int64, device=dev), "sizes": sizes.to(dev),
                   "chunks": chunks.to(dev), "n_chunks": chunks.shape[0], "ptrs": None, "turn": 0,
                   "host": [torch.empty((len(params), 5), dtype=torch.int64).pin_memory() for _ in range(2)],
                   "done": [None, None]}
            if len(self._tables) > 64:  # parameter sets keep changing (step counts diverging): keep the map small
                self._tables.clear()
            self._tables[key] = ent
        ptrs = []
        for p in params:
            g32 = _deferred_grad(p)
            ptrs.append((p.data_ptr(), (g32 if g32 is not None else p.grad).data_ptr(),
                         self.state[p]["exp_avg"].data_ptr(), self.state[p]["exp_avg_sq"].data_ptr(),
                         0 if g32 is None else 1))
        if ptrs != ent["ptrs"]:
            i = ent["turn"]
            if ent["done"][i] is not None:  # this staging buffer may still be feeding its previous copy
                ent["done"][i].synchronize()
            ent["host"][i].numpy()[:] = ptrs
            ent["tens"].copy_(ent["host"][i], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(params[0].device))
            ent["done"][i] = ev
            ent["turn"] = 1 - i
            ent["ptrs"] = ptrs
        return ent

    def zero_grad(self, set_to_none=True):
        """torch.optim.Optimizer.zero_grad; zeroing in place (set_to_none=False: persistent gradient buffers,
        as HIP-graph replay needs) runs as multi-tensor launches instead of one launch per parameter."""
        if set_to_none:
            return super().zero_grad(set_to_none=True)
        grads = []
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is not None:
                    if p.grad.grad_fn is not None:
                        p.grad.detach_()
                    else:
                        p.grad.requires_grad_(False)
                    grads.append(p.grad)
        if grads:
            torch._foreach_zero_(grads)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = _lib.load()
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            # validate everything before touching any state (a failed step leaves the state as it was)
            for p in params:
                if not (p.is_cuda and p.dtype == torch.bfloat16 and p.grad.dtype == torch.bfloat16):
                    raise TypeError("picotron_amd.optim.AdamW: parameters and gradients must be bf16 HIP tensors, "
                                    f"got {p.dtype} / {p.grad.dtype} on {p.device}")
                if p.grad.is_sparse or not p.grad.is_contiguous() or not p.is_contiguous():
                    raise ValueError("picotron_amd.optim.AdamW: dense contiguous parameters and gradients only")
            # per-parameter step counts, as torch.optim.AdamW keeps them: a parameter that had no gradient on
            # some steps (frozen for a while, an idle pipeline stage) advances only when it has one; one
            # launch per distinct step count. `step` stays a CPU scalar (a loaded state may carry it on the
            # device: moved back once, so reading it costs no host sync per step).
            by_step = {}
            for p in params:
                st = self.state[p]
                if not st:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                elif st["step"].device.type != "cpu":
                    st["step"] = st["step"].detach().to("cpu", torch.float32)
                st["step"] += 1
                by_step.setdefault(int(st["step"].item()), []).append(p)
            beta1, beta2 = group["betas"]
            for step, ps in sorted(by_step.items()):
                ent = self._group_tables(gi, ps)
                _lib.check(lib.pico_adamw_bf16(_lib.ptr(ent["tens"]), _lib.ptr(ent["sizes"]), _lib.ptr(ent["chunks"]),
                                               ent["n_chunks"], float(group["lr"]), float(beta1), float(beta2),
                                               float(group["eps"]), float(group["weight_decay"]), step,
                                               _lib.stream_of(ps[0])), "pico_adamw_bf16")
        return loss
