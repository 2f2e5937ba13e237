#!/bin/bash
# Round 5, box c: the AccumulateGrad stream probe; the loss-overlay curves (PICO_LOSS_OUT); C4 attention at the
# reference's micro-batch 4 (micro-bench, rocprof stats, PMC); the DP exposure rehearsal (bench --dp-bucket on
# RCCL at W = 1, 15 layers).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/dbg_accgrad_stream.py > gpurun_out/r05_c_accgrad.log 2>&1 || { tail -20 gpurun_out/r05_c_accgrad.log; exit 1; }
tail -30 gpurun_out/r05_c_accgrad.log
PICO_LOSS_OUT=gpurun_out/r05_loss.json timeout -k 10 600 python -u -m pytest -q -s --timeout 300 --timeout-method thread \
  "tests/test_model_gpu.py::test_loss_curve_shipped_path_overlays_reference" "tests/test_model_gpu.py::test_loss_curve_overlays_reference" \
  > gpurun_out/r05_c_overlay.log 2>&1
rc=$?; grep loss-overlay gpurun_out/r05_c_overlay.log; tail -2 gpurun_out/r05_c_overlay.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 1000 bash scripts/gpu_c4_measure.sh || exit $?
timeout -k 10 400 python -u bench.py --dp-bucket --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05_c_bench_dp1.json 2> gpurun_out/r05_c_bench_dp1.log || { tail -20 gpurun_out/r05_c_bench_dp1.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r05_c_bench_dp1.json').read()); print(d['value'], d['ms_per_step'], json.dumps(d['allreduce'])[:1500])"
