"""Debug: does graph capture survive allocations on a stream forked from the capture stream?

  python scripts/dbg_fork_capture.py [--mode none|alloc|alloc_nodel|prealloc]

Prints the capture status / id HIP reports for the capture stream and for the forked stream, then runs
x -> 6x + 3 inside the capture: on the capture stream (none), on the forked stream with fresh tensors freed
inside the capture (alloc), without the free (alloc_nodel), or into buffers allocated on the capture stream
before the fork (prealloc); ends the capture, replays, and checks the result.
"""
import argparse
import ctypes
import json

import torch


def capture_info(lib, stream):
    status = ctypes.c_int(-1)
    cid = ctypes.c_ulonglong(0)
    rc = lib.hipStreamGetCaptureInfo(ctypes.c_void_p(stream.cuda_stream), ctypes.byref(status), ctypes.byref(cid))
    return {"rc": rc, "status": status.value, "id": cid.value}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="none")
    args = ap.parse_args()
    lib = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    x = torch.randn(1 << 20, device="cuda")
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    info = {}
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream()
        info["capture_stream"] = capture_info(lib, cur)
        bufs = [torch.empty_like(x) for _ in range(3)] if args.mode == "prealloc" else None
        s.wait_stream(cur)
        info["forked_stream"] = capture_info(lib, s)
        out = None
        with torch.cuda.stream(s):
            if args.mode == "alloc":
                y = x * 2
                z = y + 1
                del y
                out = z * 3
            elif args.mode == "alloc_nodel":
                y = x * 2
                z = y + 1
                out = z * 3
            elif args.mode == "prealloc":
                torch.mul(x, 2, out=bufs[0])
                torch.add(bufs[0], 1, out=bufs[1])
                torch.mul(bufs[1], 3, out=bufs[2])
                out = bufs[2]
        cur.wait_stream(s)
        if out is None:
            out = x * 6 + 3
    print(json.dumps({"phase": "captured", **info}), flush=True)
    g.replay()
    torch.cuda.synchronize()
    ref = x * 6 + 3
    ok = bool(torch.allclose(out, ref))
    print(json.dumps({"phase": "replayed", "ok": ok, "mode": args.mode,
                      "max_err": float((out - ref).abs().max()), "out_head": out[:4].tolist(),
                      "ref_head": ref[:4].tolist()}), flush=True)


if __name__ == "__main__":
    main()
