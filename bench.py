"""Throughput benchmark of the picotron training step on MI355X (BASELINE.json metric:
tokens/sec/GPU + MFU, SmolLM-1.7B seq1024 at DP=1/2/4/8).

A step is the reference's training step (ref train.py:219-240): optimizer.zero_grad(), grad_acc
micro-batches of forward + backward (DP bucket all-reduce on the last), optimizer.step(), model.reset().
Workload: SmolLM-1.7B geometry, 15 layers, seq 1024, micro-batch 4, grad_acc 32 per GPU (the
reference README / config 3 per-GPU workload; weak scaling over DP), bf16, random init with the
reference's init procedure, synthetic uniform tokens already resident on the GPU.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--grad-acc G] [--no-cpu-baseline]
For N > 1 the driver launches one process per GPU with torch.distributed.run (`python bench.py --gpus N`
without that launcher starts it itself, before touching the GPU); DP gradients are all-reduced over RCCL
(xGMI) by DataParallelBucket.

Rank 0 prints ONE JSON line with `value` = whole-job tokens/s, a `roofline` object for the
dominant kernel (timed live with HIP events on its own launch stream) and a `cpu_baseline` object
(the oracle's CPU restatement of the same step on a bounded sample, rank 0 at N=1 only).
"""
import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SEQ, MBS, LAYERS = 1024, 4, 15
HBM_PEAK_GBS = 8000.0
BF16_PEAK_TFLOPS = 256 * 4096 * 2.4e9 / 1e12  # 2516.6 dense


def pmc_traffic(kernel_name):
    """HBM bytes per launch of `kernel_name` from the newest committed PMC summary
    (profiles/r*_pmc_attn_c2.json: scripts/pmc_attn.sh + scripts/pmc_summary.py --json on the attention
    micro-bench at this bench's shapes; 2 x FETCH_SIZE (gfx950 half-count correction) + WRITE_SIZE,
    MI355X_MICROARCH.md §HBM). (None, None) when no summary covers the kernel."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_attn_c2.json")))
    if not files:
        return None, None
    with open(files[-1]) as fh:
        recs = json.load(fh)
    # the device kernels behind a launch id, newest form first (attn_bwd_kv: the 64-row kernel for D = 64)
    forms = {"attn_bwd_kv": ("attn_bwd_kvp_kernel<", "attn_bwd_kv_kernel<")}.get(kernel_name, (kernel_name + "_kernel<",))
    for form in forms:
        for k, rec in recs.items():
            if k.startswith(form) and "traffic_bytes" in rec:
                return round(rec["traffic_bytes"]), os.path.relpath(files[-1], ROOT) + ": " + k
    return None, None


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def kernel_work(kid, cfg, mbs, seq):
    """Algorithmic work of ONE launch of kernel `kid` at this workload: (amount, unit, bound).
    Bytes: every input read once + every output written once."""
    from picotron_amd import _lib as L
    T = mbs * seq
    Hd, I, H = cfg.hidden_size, cfg.intermediate_size, cfg.num_attention_heads
    Hkv = cfg.num_key_value_heads
    D = Hd // H
    attn_fwd = 4.0 * mbs * H * seq * seq * D / 2  # causal
    table = {
        L.K_ATTN_FWD: (attn_fwd, "flop", "mfma"),
        # the backward as one operation (5 products): the roofline prices the dQ + dK/dV pair on it
        L.K_ATTN_BWD: (2.5 * attn_fwd, "flop", "mfma"),
        # split backward (head_dim 64, csrc/attn_bwd_split.hip): EXECUTED products per kernel — the dQ kernel
        # recomputes S and dP (3 products), the dK/dV kernel 4; the roofline entry for the backward prices
        # the pair on the ALGORITHMIC 5 products (2.5 x forward) over the sum of the two launch times
        L.K_ATTN_BWD_Q: (1.5 * attn_fwd, "flop", "mfma"),
        L.K_ATTN_BWD_KV: (2.0 * attn_fwd, "flop", "mfma"),
        # residual-fused form (29 of 31 launches): fwd reads x, residual, writes y, residual_out and y^T
        # (the next projection's wgrad input); bwd reads dy, d(residual_out), x, writes dx (+4 B/row
        # rstd, small dw partials)
        L.K_RMSNORM_FWD: (5 * T * Hd * 2 + 4 * T, "byte", "hbm"),
        L.K_RMSNORM_BWD: (4 * T * Hd * 2 + 4 * T, "byte", "hbm"),
        # k heads (q is rotated inside the attention forward), read + write; q|k with PICO_FUSE_ROPE_Q=0
        L.K_ROPE: (2 * T * (Hkv + (H if os.getenv("PICO_FUSE_ROPE_Q", "1") == "0" else 0)) * D * 2, "byte", "hbm"),
        L.K_SWIGLU_FWD: (4 * T * I * 2, "byte", "hbm"),  # g, u read; h and h^T written
        L.K_SWIGLU_BWD: (5 * T * I * 2, "byte", "hbm"),
    }
    return table.get(kid)


def _spawn_workers(n):
    """`--gpus N` without a launcher: run this script under torch.distributed.run with N ranks (one per GPU) as a
    child process and return its exit code. Called before this process touches the GPU; rank 0 of the child job
    writes the JSON line to the stdout this process inherited."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n), "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    log(f"[launcher] --gpus {n} without WORLD_SIZE: " + " ".join(cmd))
    return subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))


def setup(layers, grad_acc, world, device, optimizer="pico", fused_adam=True, post_build=None, dp_bucket=False):
    """The benchmark's model, optimizer and data (also used by tests/test_dp_hip_gpu.py's C3 check, so both run
    the same step): SmolLM-1.7B geometry with `layers` layers at seq 1024, the reference's random init with seed 42
    on every rank (identical replicas, ref train.py:103), DataParallelBucket when world > 1 (the bf16 .grad cast
    fused into the pico AdamW step), AdamW lr 3e-4 (ref train.py:204-209), synthetic uniform tokens resident on the
    device. post_build(model) runs before the DP wrapper (tests: a non-zero LM head)."""
    from picotron_amd.data import SyntheticDataLoader
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    from picotron_amd.model import build_llama, smollm_1_7b
    cfg = smollm_1_7b(num_hidden_layers=layers, seq_length=SEQ)
    torch.manual_seed(42)  # ref train.py:103 (same seed on every rank: identical replicas)
    model = build_llama(cfg, device=device, dtype=torch.bfloat16)
    if post_build is not None:
        post_build(model)
    num_params = sum(p.numel() for p in model.parameters())
    if world > 1 or dp_bucket:
        # the bf16 .grad cast (ref data_parallel.py:165) fused into the pico AdamW step (bit-identical)
        model = DataParallelBucket(model, defer_grad_cast=optimizer == "pico")
    # ref train.py:204-209: AdamW(lr), fused when the config's use_fused_adam is set (template default true)
    if optimizer == "pico":
        from picotron_amd.optim import AdamW
        opt = AdamW(model.parameters(), lr=3e-4)
    else:
        opt = torch.optim.AdamW(model.parameters(), lr=3e-4, **({"fused": True} if fused_adam else {}))
    loader = SyntheticDataLoader(MBS, SEQ, grad_acc, cfg.vocab_size, seed=1234, kind="uniform",
                                 num_batches=grad_acc, device=device)
    return cfg, model, opt, loader, num_params


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--grad-acc", type=int, default=32)
    ap.add_argument("--layers", type=int, default=LAYERS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="nccl",
                    help="process-group backend: nccl (= RCCL over xGMI, the product) or gloo (tests: several "
                         "ranks sharing one GPU, which RCCL refuses)")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--sync-steps", action="store_true",
                    help="read the loss on the host after every step (one device sync per step, as a per-step "
                         "log line would) instead of once after the timed region")
    ap.add_argument("--fused-adam", type=int, default=1,
                    help="AdamW(fused=True): the reference's use_fused_adam config (ref template/base_config.json:18, "
                         "train.py:204-207)")
    ap.add_argument("--optimizer", default="pico", choices=["pico", "torch"],
                    help="pico: picotron_amd.optim.AdamW (pico_adamw_bf16, one launch); torch: "
                         "torch.optim.AdamW (fused per --fused-adam), the reference's optimizer")
    ap.add_argument("--dp-bucket", action="store_true",
                    help="wrap the model in DataParallelBucket even at one rank (rehearses the N > 1 step: the "
                         "syncing micro-batch's bucket all-reduces and their exposure, on RCCL at W = 1)")
    ap.add_argument("--graphs", type=int, default=1,
                    help="replay non-syncing micro-batches as a HIP graph (1) or run them eagerly (0)")
    ap.add_argument("--comm-steps", type=int, default=1,
                    help="DataParallelBucket runs: untimed steps after the timed region that record the exposed "
                         "all-reduce time (RCCL only; 0 = skip)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(_spawn_workers(args.gpus))
    # Keep stdout for the ONE JSON line: native libraries (RCCL prints a banner at communicator
    # creation) write to fd 1, so point fd 1 at stderr and write the result to the saved fd.
    json_fd = os.dup(1)
    os.dup2(2, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # CPU baseline first, before this process touches the GPU (its gloo ranks are fresh processes):
    # BASELINE.md's CPU plan, DP = 2 x 4 threads, SmolLM-1.7B geometry 2 layers, seq 1024 (oracle/cpu_baseline.py)
    cpu_baseline = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle.cpu_baseline import c1_cpu_throughput, dp2_cpu_throughput
        t0 = time.time()
        cpu_baseline = dp2_cpu_throughput()
        log(f"[rank 0] cpu baseline DP=2 {cpu_baseline['value']} tok/s ({time.time() - t0:.0f}s)")
        t0 = time.time()
        # the plan's other config, C1 (dp2 tp2 pp2 1F1B, 8 ranks x 1 thread), reported beside it
        cpu_baseline["c1"] = c1_cpu_throughput()
        log(f"[rank 0] cpu baseline C1 {cpu_baseline['c1']['value']} tok/s ({time.time() - t0:.0f}s)")
    # one GPU per rank; ranks beyond the visible GPUs share them round-robin (gloo rehearsal only)
    device = torch.device("cuda", local_rank % torch.cuda.device_count())
    torch.cuda.set_device(device)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    os.environ.setdefault("RANK", str(rank))
    os.environ.setdefault("WORLD_SIZE", str(world))
    if args.backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)
    else:
        dist.init_process_group(args.backend, rank=rank, world_size=world)

    from picotron_amd import _lib as L
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.train import TrainingStep, get_mfu, pipelined_enabled, train_step

    L.load()
    pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=1, dp_size=world)
    t0 = time.time()
    cfg, model, opt, loader, num_params = setup(args.layers, args.grad_acc, world, device, args.optimizer,
                                                bool(args.fused_adam), dp_bucket=args.dp_bucket)
    log(f"[rank {rank}] model {num_params / 1e9:.3f}B params built in {time.time() - t0:.1f}s")
    step = TrainingStep(model, opt, loader, device, graphs=bool(args.graphs))

    for i in range(args.warmup):
        ts = time.time()
        loss = step()
        log(f"[rank {rank}] warmup {i}: loss {loss:.4f} ({time.time() - ts:.2f}s)")

    kernel_ids = [L.K_ATTN_FWD, L.K_ATTN_BWD_Q, L.K_ATTN_BWD_KV, L.K_ATTN_BWD_DKV, L.K_RMSNORM_FWD, L.K_RMSNORM_BWD,
                  L.K_RMSNORM_DW, L.K_ROPE, L.K_SWIGLU_FWD, L.K_SWIGLU_BWD, L.K_GRAD_ACCUM, L.K_CAST]
    # Per-launch HIP events cannot ride inside a graph replay, so with graphs the kernels are timed
    # over one extra eagerly launched step right after the timed region (same shapes, same stream).
    kernel_timing_live = not args.graphs
    if not args.no_kernel_timing and kernel_timing_live:
        cap = args.steps * args.grad_acc * (args.layers * 4 + 8) + 16
        for k in kernel_ids:
            L.prof_enable(k, cap)

    dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    losses = []
    for i in range(args.steps):
        # the loss stays on the device until the timed region ends: no host sync inside it (the host queues
        # step i + 1 while the device runs step i; --sync-steps restores one .item() per step)
        losses.append(step(sync_loss=args.sync_steps))
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - t_start
    losses = [float(l) for l in losses]
    from picotron_amd import ops as _ops
    from picotron_amd import wgrad_pair as _WP
    _ops.check_lm_head_grad_scale()  # the chunked CE's unit-upstream contract held over the timed steps
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    kernels = {}
    if not args.no_kernel_timing and not kernel_timing_live:
        cap = args.grad_acc * (args.layers * 4 + 8) + 16
        for k in kernel_ids:
            L.prof_enable(k, cap)
        opt.zero_grad(set_to_none=False)
        train_step(model, loader, device, graphs=None)
        torch.cuda.synchronize()
        if hasattr(model, "reset"):  # as TrainingStep.reset: the syncing micro-batch left every bucket marked ready
            model.reset()
    if not args.no_kernel_timing:
        for k in kernel_ids:
            tot, n = L.prof_collect(k)
            if n:
                kernels[L.KERNEL_NAMES[k]] = {"total_ms": tot, "launches": n, "avg_us": 1e3 * tot / n}
        L.load().pico_prof_enable(0, 0)

    # Exposed all-reduce time: device events around the syncing micro-batch's bucket all-reduces, over untimed steps
    # AFTER the throughput region (the per-bucket events and waits stay out of the timed steps). Only on
    # RCCL: gloo's Work.wait() blocks the host inside the backward, so its timings would describe the harness.
    # The steps run on every backend (the gloo tests exercise the same sequence as the RCCL run: kernel-timing step,
    # then these); only RCCL's timings are reported.
    exposure = None
    if hasattr(model, "comm_timing") and args.comm_steps > 0:
        model.comm_timing(True)
        for _ in range(args.comm_steps):
            step(sync_loss=True)
        torch.cuda.synchronize()
        report = model.comm_report()
        model.comm_timing(False)
        if dist.get_backend() == "nccl":
            exposure = comm_exposure(report, world, device)
        else:
            exposure = {"exposed_ms": None, "exposed_over": f"not measured: {dist.get_backend()} backend"}
    allreduce = measure_allreduce(model, world, device) if world > 1 else None
    if exposure is not None:
        allreduce = dict(allreduce or {"buckets": len(model.bucket_manager.buckets)}, **exposure)

    tokens = world * MBS * SEQ * args.grad_acc * args.steps
    value = tokens / elapsed
    tps_gpu = value / world
    mfu = get_mfu(tps_gpu, num_params, cfg)
    ms_per_step = 1e3 * elapsed / args.steps
    log(f"[rank {rank}] Step time {ms_per_step:.1f} ms | Loss: {losses[-1]:6.4f} | Tokens/s: {value:,.0f} | "
        f"Tokens/s/GPU: {tps_gpu:,.0f} | MFU: {mfu:5.2f}%")

    roofline = None
    if kernels:
        for name, v in kernels.items():
            kk = [k for k in kernel_ids if L.KERNEL_NAMES[k] == name][0]
            w = kernel_work(kk, cfg, MBS, SEQ)
            if w:
                a = w[0] / (v["avg_us"] * 1e-6)
                v["achieved"] = round(a / 1e12, 2) if w[1] == "flop" else round(a / 1e9, 1)
                v["unit"] = "TFLOP/s" if w[1] == "flop" else "GB/s"
                v["frac"] = round(v["achieved"] / (BF16_PEAK_TFLOPS if w[1] == "flop" else HBM_PEAK_GBS), 4)
        # candidates: (total ms, name, algorithmic work per launch, unit, bound, avg launch us, kernels)
        cand = []
        for name, v in kernels.items():
            kk = [k for k in kernel_ids if L.KERNEL_NAMES[k] == name][0]
            w = kernel_work(kk, cfg, MBS, SEQ)
            if w and kk not in (L.K_ATTN_BWD_Q, L.K_ATTN_BWD_KV):
                cand.append((v["total_ms"], name, w[0], w[1], w[2], v["avg_us"], [name]))
        if "attn_bwd_q" in kernels and "attn_bwd_kv" in kernels:
            # the split backward as ONE operation: 2.5 x forward FLOPs over the two kernels' mean launch times
            q, kv = kernels["attn_bwd_q"], kernels["attn_bwd_kv"]
            parts = ["attn_bwd_q", "attn_bwd_kv"] + (["attn_bwd_dkv"] if "attn_bwd_dkv" in kernels else [])
            avg = sum(kernels[n]["avg_us"] * kernels[n]["launches"] / q["launches"] for n in parts)
            cand.append((sum(kernels[n]["total_ms"] for n in parts), "attn_bwd_q+attn_bwd_kv",
                         kernel_work(L.K_ATTN_BWD, cfg, MBS, SEQ)[0], "flop", "mfma", avg, parts))
        _, dom, amount, unit, bound, avg_us, parts = max(cand)
        avg_s = avg_us * 1e-6
        if unit == "flop":
            achieved, peak, u = amount / avg_s / 1e12, BF16_PEAK_TFLOPS, "TFLOP/s"
        else:
            achieved, peak, u = amount / avg_s / 1e9, HBM_PEAK_GBS, "GB/s"
        traffic, srcs = 0, []
        for n in parts:
            t, src = pmc_traffic(n)
            if t is None:
                traffic = None
                break
            traffic += t
            srcs.append(src)
        roofline = {"kernel": dom, "bound": bound, "achieved": round(achieved, 2), "peak": round(peak, 1), "unit": u,
                    "frac": round(achieved / peak, 4), "traffic": traffic,
                    "traffic_source": "; ".join(srcs) if traffic is not None else None,
                    "work_per_launch": amount, "avg_launch_us": round(avg_us, 2),
                    "timed_over": ("the timed region" if kernel_timing_live else
                                   "one eager step right after the timed region (graph replays carry no per-launch events)")}
        if len(parts) > 1:
            roofline["note"] = ("algorithmic backward FLOPs (5 products, 2.5 x forward) over the summed mean launch "
                                "times of " + " + ".join(parts) + "; the kernels execute 7 products (S and dP "
                                "recomputed in the dQ kernel)")
        if "attn_fwd" in kernels and roofline["kernel"].startswith("attn_bwd"):
            # north_star's attention target is fwd + bwd together: 3.5 x forward FLOPs over the forward's
            # and the backward kernels' mean launch times
            fwd_us = kernels["attn_fwd"]["avg_us"]
            tf = 3.5 * kernel_work(L.K_ATTN_FWD, cfg, MBS, SEQ)[0] / ((fwd_us + avg_us) * 1e-6) / 1e12
            roofline["attention_fwd_bwd"] = {"us": round(fwd_us + avg_us, 2), "achieved": round(tf, 2),
                                             "frac": round(tf / BF16_PEAK_TFLOPS, 4)}
        for v in kernels.values():
            v["total_ms"] = round(v["total_ms"], 3)
            v["avg_us"] = round(v["avg_us"], 2)

    if rank == 0:
        out = {
            "metric": "tokens/sec/GPU + MFU, SmolLM-1.7B seq1024",
            "value": round(value, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (uniform token ids, reference random init)",
            "config": {"workload": "SmolLM-1.7B 15 layers, seq 1024, micro-batch 4, grad_acc %d per GPU, "
                                   "full training step (fwd+bwd+AdamW%s)" % (
                                       args.grad_acc, " pico_adamw_bf16" if args.optimizer == "pico" else
                                       (" torch fused" if args.fused_adam else " torch")),
                       "model": "SmolLM-1.7B-%dL" % args.layers, "global_batch": MBS * args.grad_acc * world,
                       "seq_len": SEQ, "micro_batch": MBS, "grad_acc": args.grad_acc, "parallelism": f"dp{world}",
                       "schedule": ("eager" if not args.graphs else
                                    "pipelined graph (forward i beside backward i-1)" if pipelined_enabled() else
                                    "graph per micro-batch"),
                       "wgrad": ("grouped micro-batches (one GEMM per projection per %d micro-batches)" % _WP.group_size(
                           getattr(model, "module", model).final_proj.weight)
                                 if _WP.enabled() and (not args.graphs or pipelined_enabled()) else "per micro-batch"),
                       "wgrad_group_buffers_gb": round(_WP.footprint_bytes() / 1e9, 2),
                       "peak_memory_gb": round(torch.cuda.max_memory_allocated(device) / 1e9, 1)},
            "tokens_per_sec_per_gpu": round(tps_gpu, 1),
            "mfu_pct": round(mfu, 2),
            "mfu_peak_tflops": round(BF16_PEAK_TFLOPS, 1),
            "num_params": num_params,
            "loss_last": round(losses[-1], 4),
            "roofline": roofline,
            "kernels": kernels,
            "cpu_baseline": cpu_baseline,
            "allreduce": allreduce,
        }
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    dist.barrier()
    dist.destroy_process_group()


XGMI_LINK_GBS, XGMI_LINKS = 153.0, 7  # MI355X xGMI: 7 point-to-point links per GPU, ~153 GB/s each


def exposure_model(buckets, world, busbw_gbs):
    """Exposed communication of one syncing backward if its bucket all-reduces ran at `busbw_gbs` bus bandwidth
    on `world` ranks: each bucket's all-reduce (2(W-1)/W * bytes of wire per GPU, ring) starts when it is ready
    and the previous one is done (RCCL serialises them on one stream); exposed = last completion - end of the
    backward (0 = the backward's own kernels). buckets: [(ready_ms rel. to the end of the backward, bytes)]."""
    t = None
    for ready, nbytes in sorted(buckets):
        dur = 2.0 * (world - 1) / world * nbytes / (busbw_gbs * 1e9) * 1e3
        t = max(ready, t if t is not None else ready) + dur
    return max(0.0, t) if t is not None else 0.0


def comm_exposure(report, world, device):
    """From DataParallelBucket.comm_report() over the timed steps: the measured exposed all-reduce time per step
    (end of the syncing backward -> end of the post-backward wait; max over ranks), the buckets' readiness times
    relative to the end of the backward (the mean over steps, rank 0), and what the same readiness would expose
    at W = 8 (or this world) at 300 / 600 / 1071 GB/s busbw (exposure_model)."""
    if not report:
        return None
    exp = sum(r["exposed_ms"] for r in report) / len(report)
    # buckets that did not sync in some recorded pass (None timings) are left out of the means
    nb0 = len(report[0]["buckets"])
    keep = [i for i in range(nb0) if all(r["buckets"][i][0] is not None for r in report)]
    report = [dict(r, buckets=[r["buckets"][i] for i in keep]) for r in report]
    t = torch.tensor([exp], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    nb = len(report[0]["buckets"])
    ready = [sum(r["buckets"][i][0] for r in report) / len(report) for i in range(nb)]
    done = [sum(r["buckets"][i][1] for r in report) / len(report) for i in range(nb)]
    sizes = [report[0]["buckets"][i][2] for i in range(nb)]
    w = world if world > 1 else 8
    order = sorted(range(nb), key=lambda i: ready[i])
    return {"exposed_ms": round(float(t.item()), 3), "exposed_over": f"{len(report)} timed steps (mean), max over ranks",
            "first_ready_ms": round(ready[order[0]], 3), "last_ready_ms": round(ready[order[-1]], 3),
            "last_ready_bytes": sizes[order[-1]], "last_done_ms": round(max(done), 3),
            "model_world": w,
            "model_exposed_ms": {str(g): round(exposure_model(list(zip(ready, sizes)), w, g), 3)
                                 for g in (300.0, 600.0, XGMI_LINK_GBS * XGMI_LINKS)},
            "bucket_ready_ms": [round(ready[i], 3) for i in order],
            "bucket_bytes": [sizes[i] for i in order]}


def measure_allreduce(model, world, device, reps=3):
    """Bus bandwidth of the DP gradient all-reduce (north_star: "all-reduce bus bandwidth against
    xGMI peak"): the step's own fp32 bucket buffers (reference layout, ref bucket.py:84-129),
    all-reduced back to back in readiness order (last bucket first, ref data_parallel.py:93-144),
    timed after the throughput region with barrier + synchronize, max over ranks.
    busbw = 2(W-1)/W * bytes / time (the ring algorithm's per-GPU wire bytes)."""
    bufs = [b.grad_data for b in reversed(model.bucket_manager.buckets)]
    nbytes = sum(b.numel() * b.element_size() for b in bufs)
    for b in bufs:  # warm-up (communicator channels for every size class)
        dist.all_reduce(b)
    times = []
    for _ in range(reps):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for b in bufs:
            dist.all_reduce(b)
        torch.cuda.synchronize()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        times.append(float(t.item()))
    t = min(times)
    busbw = 2.0 * (world - 1) / world * nbytes / t / 1e9
    peak = XGMI_LINK_GBS * XGMI_LINKS
    return {"buckets": len(bufs), "bytes": nbytes, "ms": round(1e3 * t, 3), "algbw_GBps": round(nbytes / t / 1e9, 1),
            "busbw_GBps": round(busbw, 1), "peak_GBps": peak, "frac": round(busbw / peak, 4),
            "single_link_GBps": XGMI_LINK_GBS, "timed_over": f"best of {reps} passes over all buckets, after the timed region"}


if __name__ == "__main__":
    main()
