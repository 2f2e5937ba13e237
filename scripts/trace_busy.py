"""Device occupancy of a training step from a rocprofv3 --kernel-trace CSV (bench.py run): over the last
`--steps` optimizer steps (delimited by the AdamW launches), the wall time, the time with no kernel running
(idle), with one, and with two or more kernels in flight (the pipelined micro-batches' overlap), the biggest idle
gaps with the kernels around them, and the busy time per kernel class.

  python scripts/trace_busy.py <kernel_trace.csv> [--steps 2] [--json out.json]
"""
import argparse
import csv
import json
import re


def klass(n):
    if "Cijk" in n:
        return "gemm"
    for key in ("attn_fwd", "attn_bwd_q", "attn_bwd_kv", "rmsnorm", "rope", "swiglu_fwd", "swiglu_bwd", "ce_", "adamw",
                "transpose", "embedding", "sort_ids"):
        if key in n:
            return key.rstrip("_")
    return "other"


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "").replace("at::native::", "")
    if "Cijk" in n:
        m = re.search(r"MT(\d+x\d+x\d+)", n)
        return "GEMM " + (m.group(1) if m else "?")
    return re.sub(r"[(<].*", "", n)[:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.csv)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    adam = [e for e in ev if "adamw" in e[2]]
    if len(adam) < args.steps + 1:
        raise SystemExit(f"need {args.steps + 1} AdamW launches, found {len(adam)}")
    t0, t1 = adam[-args.steps - 1][1], adam[-1][1]  # from the end of one optimizer step to the end of the last
    win = [e for e in ev if e[1] > t0 and e[0] < t1]
    # sweep: time with 0 / 1 / >= 2 kernels in flight
    pts = []
    for s, e, _ in win:
        pts.append((max(s, t0), 1))
        pts.append((min(e, t1), -1))
    pts.sort()
    depth, last, acc = 0, t0, {0: 0, 1: 0, 2: 0}
    for t, d in pts:
        acc[min(depth, 2)] += t - last
        depth += d
        last = t
    acc[min(depth, 2)] += t1 - last
    gaps = []
    end_max = t0
    prev = None
    for j, (s, e, n) in enumerate(win):
        if s > end_max and prev is not None:
            ctx = [f"{(win[q][0] - t0) / 1e3:.1f}+{(win[q][1] - win[q][0]) / 1e3:.1f}us {short(win[q][2])}"
                   for q in range(max(0, j - 4), min(len(win), j + 3))]
            gaps.append((s - end_max, short(prev), short(n), round((end_max - t0) / 1e3, 1), ctx))
        if e > end_max:
            end_max, prev = e, n
    gaps.sort(reverse=True)
    per = {}
    for s, e, n in win:
        per[klass(n)] = per.get(klass(n), 0) + (min(e, t1) - max(s, t0))
    wall = t1 - t0
    out = {"steps": args.steps, "wall_ms_per_step": round(wall / 1e6 / args.steps, 2),
           "idle_ms_per_step": round(acc[0] / 1e6 / args.steps, 2),
           "one_kernel_ms_per_step": round(acc[1] / 1e6 / args.steps, 2),
           "two_plus_kernels_ms_per_step": round(acc[2] / 1e6 / args.steps, 2),
           "kernel_ms_per_step_by_class": {k: round(v / 1e6 / args.steps, 2) for k, v in
                                           sorted(per.items(), key=lambda x: -x[1])},
           "largest_gaps_us": [(round(g / 1e3, 1), a, b, at) for g, a, b, at, _ in gaps[:12]],
           "largest_gaps_context": [ctx for *_, ctx in gaps[:4]]}
    print(json.dumps(out, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
