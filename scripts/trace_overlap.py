"""Where a training step's wall time goes, from a rocprofv3 kernel trace (run_kernel_trace.csv):

  python scripts/trace_overlap.py gpurun_out/final_prof/run_kernel_trace.csv

The last step is the interval between the ends of the last two AdamW launches. Every instant of it is classed by
what runs: a hipBLASLt GEMM (alone or beside other kernels), only non-GEMM kernels, or nothing; and by how many
hardware queues (the pipelined graph's two streams) have a kernel in flight. Prints those totals and the non-GEMM
kernels that fill the GEMM-free time (each instant split evenly over the kernels running then).
"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows)
    ad = [e for e in ev if "adamw" in e[2]]
    if len(ad) < 2:
        raise SystemExit("need two AdamW launches in the trace")
    a, b = ad[-2][1], ad[-1][1]
    win = [e for e in ev if e[0] >= a and e[1] <= b]
    pts = []
    for s, e, n, q in win:
        pts.append((s, 1, n, q))
        pts.append((e, -1, n, q))
    pts.sort(key=lambda x: (x[0], x[1]))
    active = collections.Counter()  # kernel name -> in flight
    queues = collections.Counter()
    cls = collections.Counter()
    fill = collections.Counter()
    last = a
    for t, d, n, q in pts:
        dt = (t - last) / 1e6
        gem = sum(v for k, v in active.items() if "Cijk" in k)
        oth = sum(v for k, v in active.items() if "Cijk" not in k)
        nq = sum(1 for v in queues.values() if v > 0)
        kind = "gemm" if gem else ("non-gemm only" if oth else "idle")
        cls[(kind, "2+ queues" if nq > 1 else ("1 queue" if nq == 1 else "-"))] += dt
        if kind == "non-gemm only":
            for k, v in active.items():
                if v > 0:
                    fill[k[:70]] += dt * v / oth
        last = t
        active[n] += d
        queues[q] += d
    print(f"step {(b - a) / 1e6:.1f} ms")
    for k in sorted(cls):
        print(f"  {k[0]:14s} {k[1]:10s} {cls[k]:8.1f} ms")
    print("GEMM-free time by kernel:")
    for k, v in fill.most_common(15):
        print(f"  {v:7.2f} ms  {k}")


if __name__ == "__main__":
    main()
