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


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, amsgrad=False, *,
                 maximize=False, foreach=None, capturable=False, differentiable=False, fused=None):
        if amsgrad or maximize or capturable or differentiable:
            raise NotImplementedError("picotron_amd.optim.AdamW: amsgrad / maximize / capturable / differentiable")
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"invalid AdamW hyper-parameters lr={lr} betas={betas} eps={eps}")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False, maximize=False,
                        foreach=None, capturable=False, differentiable=False, fused=fused)
        super().__init__(params, defaults)
        self._tables = {}  # group index -> (key, tensors_dev, sizes_dev, chunks_dev, n_chunks, pinned host table)
        self._copy_done = None  # event after the last host -> device table copy

    def _group_tables(self, gi, params):
        chunk = int(_lib.load().pico_adamw_chunk_elems())
        key = tuple((p.data_ptr(), p.numel()) for p in params)
        ent = self._tables.get(gi)
        if ent is None or ent[0] != key:
            sizes = torch.tensor([p.numel() for p in params], dtype=torch.int64)
            chunks = [(i, c) for i, p in enumerate(params) for c in range(0, p.numel(), chunk)]
            dev = params[0].device
            chunks_t = torch.tensor(chunks, dtype=torch.int64).reshape(-1, 2)
            host = torch.empty((len(params), 4), dtype=torch.int64).pin_memory()
            ent = (key, torch.empty((len(params), 4), dtype=torch.int64, device=dev), sizes.to(dev),
                   chunks_t.to(dev), len(chunks), host)
            self._tables[gi] = ent
        return ent

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
            steps = set()
            for p in params:
                if not (p.is_cuda and p.dtype == torch.bfloat16 and p.grad.dtype == torch.bfloat16):
                    raise TypeError("picotron_amd.optim.AdamW: parameters and gradients must be bf16 HIP tensors, "
                                    f"got {p.dtype} / {p.grad.dtype} on {p.device}")
                if p.grad.is_sparse or not p.grad.is_contiguous() or not p.is_contiguous():
                    raise ValueError("picotron_amd.optim.AdamW: dense contiguous parameters and gradients only")
                st = self.state[p]
                if not st:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                steps.add(int(st["step"].item()))
            if len(steps) != 1:
                raise RuntimeError("picotron_amd.optim.AdamW: parameters of one group at different step counts")
            key, tens, sizes, chunks, n_chunks, host = self._group_tables(gi, params)
            if self._copy_done is not None:  # the pinned table may still be feeding the previous copy
                self._copy_done.synchronize()
            host.numpy()[:] = [(p.data_ptr(), p.grad.data_ptr(), self.state[p]["exp_avg"].data_ptr(),
                                self.state[p]["exp_avg_sq"].data_ptr()) for p in params]
            tens.copy_(host, non_blocking=True)
            self._copy_done = torch.cuda.Event()
            self._copy_done.record(torch.cuda.current_stream(params[0].device))
            beta1, beta2 = group["betas"]
            _lib.check(lib.pico_adamw_bf16(_lib.ptr(tens), _lib.ptr(sizes), _lib.ptr(chunks), n_chunks,
                                           float(group["lr"]), float(beta1), float(beta2), float(group["eps"]),
                                           float(group["weight_decay"]), steps.pop(), _lib.stream_of(params[0])),
                       "pico_adamw_bf16")
        return loss
