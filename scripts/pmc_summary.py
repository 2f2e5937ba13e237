"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*/run_counter_collection.csv): mean counter value
per dispatch for every kernel whose name matches --match, plus derived ratios.

  python scripts/pmc_summary.py [--dir gpurun_out/pmc] [--match attn_,rmsnorm,swiglu,rope] [--json OUT]

--json writes per kernel: mean counters per dispatch, median duration, and HBM traffic per launch =
2 x FETCH_SIZE (gfx950 reports half of wide streaming reads, MI355X_MICROARCH.md §HBM) + WRITE_SIZE,
in bytes (rocprofv3 reports both in KB).
"""
import json
import argparse
import collections
import csv
import glob
import os
import re


def short(name):
    m = re.search(r"(\w+_kernel)(<[^(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="gpurun_out/pmc")
    ap.add_argument("--match", default="attn_")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    out = {}
    pats = args.match.split(",")
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(args.dir, "p*", "run_counter_collection.csv"))):
        per_dispatch = collections.defaultdict(dict)
        meta = {}
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if not any(p in row["Kernel_Name"] for p in pats):
                    continue
                k = short(row["Kernel_Name"])
                per_dispatch[(k, row["Dispatch_Id"])][row["Counter_Name"]] = float(row["Counter_Value"])
                meta[(k, row["Dispatch_Id"])] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"]),
                                                 row["VGPR_Count"], row["Accum_VGPR_Count"], row["LDS_Block_Size"])
        for (k, d), cs in per_dispatch.items():
            for c, v in cs.items():
                acc[k][c].append(v)
            dur[k].append(meta[(k, d)])
    for k in sorted(acc):
        cs = {c: sum(v) / len(v) for c, v in acc[k].items()}
        ds = dur[k]
        ns = sorted(x[0] for x in ds)[len(ds) // 2]
        print(f"== {k}  (dispatches/pass ~{len(ds) // max(1, len(glob.glob(os.path.join(args.dir, 'p*'))))}, "
              f"median dur {ns / 1e3:.1f} us, vgpr {ds[0][1]} agpr {ds[0][2]} lds {ds[0][3]})")
        for c in sorted(cs):
            print(f"   {c:28s} {cs[c]:16.1f}")
        w = cs.get("SQ_WAVE_CYCLES")
        if w:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_MFMA", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
                if c in cs:
                    print(f"   {c + '/WAVE_CYCLES':40s} {cs[c] / w:8.3f}")
        if "GRBM_GUI_ACTIVE" in cs:
            print(f"   effective clock GHz (GRBM/8/dur)        {cs['GRBM_GUI_ACTIVE'] / 8 / ns:8.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in cs and "GRBM_GUI_ACTIVE" in cs:
            # MFMA busy cycles summed over SIMDs vs available SIMD-cycles (1024 SIMDs x GUI cycles / 8 XCD sum)
            simd_cycles = 1024 * cs["GRBM_GUI_ACTIVE"] / 8
            print(f"   MFMA busy fraction                      {cs['SQ_VALU_MFMA_BUSY_CYCLES'] / simd_cycles:8.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in cs:
            # the same over the kernel's median duration at the 2.4 GHz MFMA clock (GRBM_GUI_ACTIVE can span more than
            # the dispatch for short kernels: the effective clock above then reads high and the fraction low)
            print(f"   MFMA busy fraction (median dur, 2.4 GHz) {cs['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * ns * 2.4):8.3f}")
        if "SQ_LDS_BANK_CONFLICT" in cs and "SQ_LDS_IDX_ACTIVE" in cs:
            print(f"   LDS bank-conflict share                 {cs['SQ_LDS_BANK_CONFLICT'] / max(1, cs['SQ_LDS_IDX_ACTIVE']):8.3f}")
        if "FETCH_SIZE" in cs:
            print(f"   FETCH bytes (x2 gfx950 corr, KB->MB)    {2 * cs['FETCH_SIZE'] / 1e3:8.2f} MB")
        if "WRITE_SIZE" in cs:
            print(f"   WRITE bytes                             {cs['WRITE_SIZE'] / 1e3:8.2f} MB")
        rec = {"median_dur_us": ns / 1e3, "counters_per_dispatch": cs}
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            rec["fetch_bytes_corrected"] = 2 * cs["FETCH_SIZE"] * 1e3
            rec["write_bytes"] = cs["WRITE_SIZE"] * 1e3
            rec["traffic_bytes"] = rec["fetch_bytes_corrected"] + rec["write_bytes"]
        out[k] = rec
    if args.json:
        with open(args.json, "w") as fh:
            json.dump(out, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
