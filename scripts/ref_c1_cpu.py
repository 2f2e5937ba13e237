"""Same-day C1 CPU cross-check: time the REFERENCE's own C1 step and the
port's (oracle/cpu_baseline.py c1_cpu_throughput) back to back in the build container, on equal cores.

C1 = SmolLM-1.7B geometry, 5 layers, dp 2 x tp 2 x pp 2, 1F1B, micro-batch 4 x seq 128, grad_acc 2, fp32 eager,
8 gloo ranks x 1 thread. The reference side runs its own modules end to end — Llama (ref picotron/model.py,
FLASH_ATTEN=0 eager path), apply_tensor_parallel (ref picotron/tensor_parallel/tensor_parallel.py:9-52),
PipelineParallel + train_step_pipeline_1f1b (ref picotron/pipeline_parallel/pipeline_parallel.py:8-145),
DataParallelBucket (ref picotron/data_parallel/data_parallel.py:62-171), torch AdamW — on synthetic tokens (the
reference's HF loader needs the network) with its random init (PipelineParallel.reset_parameters; the HF
safetensors load of checkpoint.py is skipped: timing only). Two shims, both needed on a GPU-less host and
both outside the timed arithmetic: flash-attn's three entry points are registered as raising stubs (never
called with FLASH_ATTEN=0) and torch.cuda.synchronize (called after every P2P, ref pp_communications.py:30,44)
is a no-op.

Build container only (the reference never travels to the GPU box). Writes one JSON line to stdout:
  python scripts/ref_c1_cpu.py [--steps 1] [--warmup 1] > profiles/r03_c1_cpu_crosscheck.json
"""
import argparse
import json
import os
import socket
import sys
import time
import types

import torch

REF = "/root/reference"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LAYERS, MBS, SEQ, GA = 5, 4, 128, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _import_reference():
    os.environ["FLASH_ATTEN"] = "0"
    os.environ["DEVICE"] = "cpu"
    os.environ["CONTEXT_PARALLEL"] = "0"
    if REF not in sys.path:
        sys.path.insert(0, REF)

    def _not_available(*a, **k):
        raise NotImplementedError("flash-attn is not installed; the eager path must not call it")

    for name in ["flash_attn", "flash_attn.flash_attn_interface", "flash_attn.layers", "flash_attn.layers.rotary",
                 "flash_attn.ops", "flash_attn.ops.triton", "flash_attn.ops.triton.layer_norm"]:
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["flash_attn.flash_attn_interface"].flash_attn_func = _not_available
    sys.modules["flash_attn.layers.rotary"].apply_rotary_emb = _not_available
    sys.modules["flash_attn.ops.triton.layer_norm"].layer_norm_fn = _not_available
    torch.cuda.synchronize = lambda *a, **k: None


class _Loader:
    """The reference loader's batch format (ref picotron/data.py:102-116) on synthetic tokens."""

    def __init__(self, dp_rank):
        self.grad_acc_steps = GA
        self.micro_batch_size = MBS
        self.seq_length_per_gpu = SEQ
        self.g = torch.Generator().manual_seed(1234 + dp_rank)

    def __next__(self):
        toks = torch.randint(0, 49152, (MBS, SEQ + 1), generator=self.g)
        return {"input_ids": toks[:, :-1], "target_ids": toks[:, 1:],
                "position_ids": torch.arange(SEQ).unsqueeze(0).expand(MBS, -1), "hidden_states": None}


def _ref_worker(rank, world, port, steps, warmup, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    _import_reference()
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import picotron.process_group_manager as pgm
    from picotron.data_parallel.data_parallel import DataParallelBucket
    from picotron.model import Llama
    from picotron.pipeline_parallel.pipeline_parallel import PipelineParallel, train_step_pipeline_1f1b
    from picotron.tensor_parallel.tensor_parallel import apply_tensor_parallel
    pgm.setup_process_group_manager(tp_size=2, cp_size=1, pp_size=2, dp_size=2)
    m = pgm.process_group_manager
    cfg = types.SimpleNamespace(hidden_size=2048, intermediate_size=8192, num_attention_heads=32,
                                num_key_value_heads=32, num_hidden_layers=LAYERS, vocab_size=49152,
                                max_position_embeddings=SEQ, rms_norm_eps=1e-5, rope_theta=10000.0)
    torch.manual_seed(42)
    model = Llama(config=cfg)
    model = apply_tensor_parallel(model)
    model = PipelineParallel(model, cfg)
    model = DataParallelBucket(model)
    opt = torch.optim.AdamW(model.parameters(), lr=3e-4)
    loader = _Loader(m.dp_rank)
    shapes = (MBS, SEQ, cfg.hidden_size)

    def step():
        opt.zero_grad()
        loss = train_step_pipeline_1f1b(model, loader, shapes, "cpu", torch.float32)
        opt.step()
        model.reset()
        return loss

    for _ in range(warmup):
        step()
    dist.barrier()
    t0 = time.perf_counter()
    loss = 0.0
    for _ in range(steps):
        loss = step()
    dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if m.pp_is_last_stage and m.tp_rank == 0 and m.dp_rank == 0:
        q.put((float(t.item()), float(loss)))
    dist.barrier()
    dist.destroy_process_group()


def reference_c1(steps, warmup):
    import torch.multiprocessing as mp
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ref_worker, args=(r, world, port, steps, warmup, q)) for r in range(world)]
    for p in procs:
        p.start()
    dt, loss = q.get(timeout=1800)
    for p in procs:
        p.join(timeout=120)
    tokens = 2 * MBS * SEQ * GA * steps
    return {"value": round(tokens / dt, 2), "unit": "tokens/s", "s_per_step": round(dt / steps, 2), "cores": world,
            "kind": "reference", "loss": round(loss, 4)}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    sys.path.insert(0, REPO)
    t0 = time.time()
    ref = reference_c1(args.steps, args.warmup)
    from oracle.cpu_baseline import c1_cpu_throughput
    port = c1_cpu_throughput(steps=args.steps, warmup=args.warmup)
    out = {"what": "C1 CPU cross-check, same container, same session, back to back (reference first)",
           "host_cpus": os.cpu_count(), "date": time.strftime("%Y-%m-%d %H:%M"),
           "reference": ref, "port": {k: port[k] for k in ("value", "unit", "cores", "kind", "loss")},
           "port_s_per_step": round(2 * MBS * SEQ * GA * args.steps / port["value"] / args.steps, 2),
           "ratio_port_over_reference_throughput": round(port["value"] / ref["value"], 3),
           "wall_s": round(time.time() - t0, 1)}
    print(json.dumps(out))
