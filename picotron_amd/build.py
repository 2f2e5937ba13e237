"""Build the gfx950 C-ABI library `picotron_amd/lib/libpicotron_hip.so` in-tree with hipcc.

The library has no torch types in its interface (see include/picotron_hip.h); it is loaded with
ctypes by picotron_amd/_lib.py after torch, so it binds to the HIP runtime torch already loaded
(both export the soname libamdhip64.so.7).

Usage: python -m picotron_amd.build [--verbose] [--resource-usage]
"""
import argparse
import concurrent.futures as cf
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "lib", "obj")
LIB = os.path.join(HERE, "lib", "libpicotron_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
          "-munsafe-fp-atomics"]


# per-source flags: the split attention backward keeps MFMA results in VGPRs (its softmax reads them every
# tile; AGPR accumulators cost one v_accvgpr_read per score) and no SLP-packed f32 VALU beside the MFMAs
# (cdna_hip_programming.md / MI355X_MICROARCH.md: packed f32 ops are an anti-lever there)
FILE_FLAGS = {
    "attn_bwd_split.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form"],
    "attn_fwd.hip": ["-fno-slp-vectorize", "-fno-honor-nans"],
    "attn_fwdp.hip": ["-fno-slp-vectorize", "-fno-honor-nans", "-mllvm", "-amdgpu-mfma-vgpr-form"],
    "attn_bwd_split_d128.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form"],
}


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def deps(src):
    """Files whose change rebuilds `src`: itself, every csrc header, the C-ABI header, this file (per-file
    flags) and any .hip source it #includes (attn_bwd_split_d128.hip includes attn_bwd_split.hip)."""
    out = [src] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    with open(src) as f:
        out += [os.path.join(CSRC, m.group(1)) for m in re.finditer(r'#include "([^"]+\.hip)"', f.read())]
    out.append(os.path.join(HERE, "..", "include", "picotron_hip.h"))
    out.append(os.path.abspath(__file__))
    return out


def _compile(src, extra, verbose):
    obj = os.path.join(OBJ, os.path.basename(src)[:-4] + ".o")
    if os.path.exists(obj) and not extra and all(os.path.getmtime(obj) >= os.path.getmtime(d) for d in deps(src)):
        return obj, ""
    cmd = [HIPCC, *CFLAGS, *FILE_FLAGS.get(os.path.basename(src), []), *extra, "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj, r.stderr


def build(verbose=False, resource_usage=False, jobs=8):
    os.makedirs(OBJ, exist_ok=True)
    extra = ["-Rpass-analysis=kernel-resource-usage"] if resource_usage else []
    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=min(jobs, len(srcs))) as ex:
        results = list(ex.map(lambda s: _compile(s, extra, verbose), srcs))
    objs = [o for o, _ in results]
    if resource_usage:
        for (o, log), s in zip(results, srcs):
            if log:
                print(f"== {os.path.basename(s)}\n{log}")
    need_link = not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs)
    if need_link:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--resource-usage", action="store_true")
    args = ap.parse_args()
    print(build(verbose=args.verbose, resource_usage=args.resource_usage))
    sys.exit(0)
