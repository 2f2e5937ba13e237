"""ORACLE — TEST INFRASTRUCTURE ONLY. The reference's CPU/gloo training path timed on the host cores
(bench.py's `cpu_baseline` leg; BASELINE.md "CPU-baseline plan"): both configs of
the plan, dp2_cpu_throughput (DP = 2, 2 layers, seq 1024, 2 ranks x 4 threads) and c1_cpu_throughput
(C1: dp2 tp2 pp2 1F1B, 5 layers, seq 128, grad_acc 2, 8 ranks x 1 thread).

Config (the plan's second one, which the survey timed with the reference itself in the build container:
15.4 s/step, 531 tokens/s total on 8 cores): SmolLM-1.7B geometry with 2 layers, DP = 2 over gloo, micro-
batch 4, seq 1024, grad_acc 1, fp32, eager attention (the reference's FLASH_ATTEN=0 CPU path), 2 ranks x 4
threads. Each rank runs the reference's step (ref train.py:219-240): zero_grad, forward + mean CE, backward
with the DP bucket all-reduce (picotron_amd.data_parallel on the oracle's CPU device-op table: the
reference's bucket algorithm, ref picotron/data_parallel/*.py), AdamW step. The oracle model is
oracle/model.py (ref picotron/model.py eager path). Nothing here runs on, or is used by, the GPU product.
"""
import os
import socket
import time
from types import SimpleNamespace


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, threads, layers, seq, mbs, steps, warmup, q):
    import torch
    import torch.distributed as dist
    torch.set_num_threads(threads)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import hotpath as H
    from oracle import model as OM
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.data_parallel import bucket as B
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=1, dp_size=world)
    B.set_kernels(H.CpuBucketKernels())
    cfg = SimpleNamespace(hidden_size=2048, intermediate_size=8192, num_attention_heads=32, num_key_value_heads=32,
                          num_hidden_layers=layers, vocab_size=49152, max_position_embeddings=seq, rms_norm_eps=1e-5,
                          rope_theta=10000.0)
    torch.manual_seed(42)
    model = OM.build(cfg)
    ddp = DataParallelBucket(model)
    opt = torch.optim.AdamW(ddp.parameters(), lr=3e-4)
    gen = torch.Generator().manual_seed(1234 + rank)
    V = cfg.vocab_size

    def step():
        opt.zero_grad()
        toks = torch.randint(0, V, (mbs, seq + 1), generator=gen)
        ddp.require_backward_grad_sync = True  # grad_acc 1: the only micro-batch syncs
        logits = ddp(input_ids=toks[:, :-1])
        loss = torch.nn.functional.cross_entropy(logits.reshape(-1, V), toks[:, 1:].reshape(-1))
        loss.backward()
        opt.step()
        ddp.reset()
        return float(loss.detach())

    for _ in range(warmup):
        step()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    dist.barrier()
    dt = time.perf_counter() - t0
    if rank == 0:
        q.put((dt, loss))
    dist.destroy_process_group()


def dp2_cpu_throughput(layers=2, seq=1024, mbs=4, ranks=2, threads=4, steps=1, warmup=1):
    """Runs the plan's DP=2 CPU config in `ranks` fresh processes; returns the cpu_baseline dict."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ranks, port, threads, layers, seq, mbs, steps, warmup, q))
             for r in range(ranks)]
    for p in procs:
        p.start()
    dt, loss = q.get(timeout=900)
    for p in procs:
        p.join(timeout=120)
    tokens = ranks * mbs * seq * steps
    return {"value": round(tokens / dt, 2), "unit": "tokens/s", "cores": ranks * threads, "kind": "port",
            "sample": f"{steps} timed step(s) after {warmup} warm-up of SmolLM-1.7B geometry, {layers} layers, DP={ranks} "
                      f"over gloo ({ranks} ranks x {threads} threads), micro-batch {mbs} x seq {seq}, grad_acc 1, fp32 "
                      f"eager (oracle/model.py + the reference's bucket all-reduce) + AdamW: {dt / steps:.1f} s/step; "
                      "cross-check in the 8-core build container: the reference's own eager step (2 layers, 1 rank x 4 "
                      "threads) 20.7 s vs this port's 20.1 s (same container, same day); the survey's earlier reading of "
                      "this DP=2 config there was 531 tokens/s, the container has since run slower",
            "loss": round(loss, 4)}


def _c1_worker(rank, world, port, layers, seq, mbs, grad_acc, steps, warmup, q):
    import torch
    import torch.distributed as dist
    torch.set_num_threads(1)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import hotpath as H
    from oracle import model as OM
    from oracle.pipeline import Stage, train_step_1f1b
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.data_parallel import bucket as B
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    from picotron_amd.tensor_parallel.tensor_parallel import apply_tensor_parallel
    m = pgm.setup_process_group_manager(tp_size=2, cp_size=1, pp_size=2, dp_size=2)
    B.set_kernels(H.CpuBucketKernels())
    cfg = SimpleNamespace(hidden_size=2048, intermediate_size=8192, num_attention_heads=32, num_key_value_heads=32,
                          num_hidden_layers=layers, vocab_size=49152, max_position_embeddings=seq, rms_norm_eps=1e-5,
                          rope_theta=10000.0, tp_size=m.tp_world_size)
    torch.manual_seed(42)
    model = OM.build(cfg)
    apply_tensor_parallel(model, shard_weights=True)  # the product's TP layers (CPU fallbacks), this rank's shards
    stage = Stage(model, layers, m)
    del model
    ddp = DataParallelBucket(stage)
    opt = torch.optim.AdamW(ddp.parameters(), lr=3e-4)
    gen = torch.Generator().manual_seed(1234 + m.dp_rank)  # same data on every tp / pp rank of a dp replica
    V, Hd = cfg.vocab_size, cfg.hidden_size

    def step():
        opt.zero_grad()
        toks = [torch.randint(0, V, (mbs, seq + 1), generator=gen) for _ in range(grad_acc)]
        loss = train_step_1f1b(ddp, [(t[:, :-1], t[:, 1:]) for t in toks], (mbs, seq, Hd), m)
        opt.step()
        ddp.reset()
        return loss

    for _ in range(warmup):
        step()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    dist.barrier()
    dt = time.perf_counter() - t0
    if m.pp_is_last_stage and m.dp_rank == 0 and m.tp_rank == 0:
        q.put((dt, loss))
    dist.barrier()
    dist.destroy_process_group()


def c1_cpu_throughput(layers=5, seq=128, mbs=4, grad_acc=2, steps=1, warmup=1):
    """BASELINE.md's C1 CPU config: SmolLM-1.7B geometry, 5 layers, dp2 tp2 pp2, 1F1B, micro-batch 4 x seq 128,
    grad_acc 2, fp32 eager, 8 gloo ranks x 1 thread; returns a cpu_baseline-style dict."""
    import torch.multiprocessing as mp
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c1_worker, args=(r, world, port, layers, seq, mbs, grad_acc, steps, warmup, q))
             for r in range(world)]
    for p in procs:
        p.start()
    dt, loss = q.get(timeout=900)
    for p in procs:
        p.join(timeout=120)
    tokens = 2 * mbs * seq * grad_acc * steps  # dp 2 replicas
    return {"value": round(tokens / dt, 2), "unit": "tokens/s", "cores": world, "kind": "port",
            "sample": f"{steps} timed step(s) after {warmup} warm-up of C1: SmolLM-1.7B geometry, {layers} layers, dp2 tp2 "
                      f"pp2 1F1B (8 gloo ranks x 1 thread), micro-batch {mbs} x seq {seq}, grad_acc {grad_acc}, fp32 eager "
                      f"(oracle/model.py + oracle/pipeline.py + the product's TP layers and DP bucket on CPU) + AdamW: "
                      f"{dt / steps:.1f} s/step; the reference's own run of this config in the build container: 14.9 s/step, "
                      "137 tokens/s",
            "loss": round(loss, 4)}
