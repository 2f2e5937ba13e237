"""Print one decoder layer's kernel sequence (forward and backward) from a rocprofv3 --kernel-trace CSV
of an eager bench step (bench.py --graphs 0), with per-kernel durations; GEMMs are labelled by tile.
usage: python scripts/trace_layer.py <kernel_trace.csv> [layer_from_end]"""
import csv
import re
import sys


def short(n):
    if "Cijk" in n:
        m = re.search(r"MT(\d+x\d+x\d+)", n)
        lay = re.search(r"Cijk_(A\w{3})_(B\w{3})", n)
        return "GEMM %s %s%s" % (m.group(1) if m else "?", lay.group(1) + "_" + lay.group(2) if lay else "",
                                 " SK" if re.search(r"_SK\d", n) else "")
    n = n.replace("void ", "").replace("(anonymous namespace)::", "").replace("at::native::", "")
    return re.sub(r"\(.*", "", n)[:70]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    fwd = [i for i, r in enumerate(rows) if "attn_fwd_kernel" in r["Kernel_Name"]]
    bwd = [i for i, r in enumerate(rows) if "attn_bwd_kernel" in r["Kernel_Name"]]
    for title, idx, lo, hi in (("forward", fwd, 8, 8), ("backward", bwd, 12, 10)):
        i = idx[-k]
        print(f"--- {title} (attention launch {len(idx) - k} of {len(idx)})")
        for r in rows[i - lo:i + hi]:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            print(f"{d:8.1f} us  {short(r['Kernel_Name'])}  grid={r['Grid_Size_X']}")


if __name__ == "__main__":
    main()
