#!/bin/bash
# Round 5, box g: kvp lifetime anatomy (stamps: loop / prologue / epilogue shares), the HBM kernels in eager
# micro-batches (base vs RMSNorm-backward R = 2), and the DP-bucket step vs the plain step on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=picotron_amd/lib/variants
for g in 1 0; do
  PICO_LIB_PATH=$V/kvpstamp.so PICO_ATTN_KVP=1 PICO_ATTN_GROUPS=$g timeout -k 10 120 python -u scripts/kvp_stamps.py > gpurun_out/r05_g_kvpstamps_g$g.json 2> gpurun_out/r05_g_kvpstamps.log || { tail -20 gpurun_out/r05_g_kvpstamps.log; exit 1; }
  cat gpurun_out/r05_g_kvpstamps_g$g.json
done
rm -f gpurun_out/r05_g_hbm.jsonl
for r in 1 2; do
  for v in base rms_r2; do
    LIB=""; [ "$v" != base ] && LIB=$V/$v.so
    PICO_LIB_PATH=$LIB timeout -k 10 240 python -u scripts/hbm_instep.py --layers 4 --mb 4 >> gpurun_out/r05_g_hbm.jsonl 2>> gpurun_out/r05_g_hbm.log || { tail -20 gpurun_out/r05_g_hbm.log; exit 1; }
  done
done
cat gpurun_out/r05_g_hbm.jsonl
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > gpurun_out/r05_g_bench_plain_$r.json 2> gpurun_out/r05_g_bench.log || { tail -20 gpurun_out/r05_g_bench.log; exit 1; }
  timeout -k 10 400 python -u bench.py --dp-bucket --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > gpurun_out/r05_g_bench_dp_$r.json 2>> gpurun_out/r05_g_bench.log || { tail -20 gpurun_out/r05_g_bench.log; exit 1; }
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r05_g_bench_*.json")):
    d = json.loads(open(f).read())
    ar = d.get("allreduce") or {}
    print(f, d["value"], d["ms_per_step"], d["mfu_pct"], ar.get("exposed_ms"), ar.get("model_exposed_ms"))
PY
