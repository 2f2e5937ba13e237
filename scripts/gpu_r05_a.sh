#!/bin/bash
# Round 5, first box: the C4 micro-batch-4 parity tests, the composition at seq 1024 / mbs 4, the wgrad-pair
# and loss-overlay tests (with -s: the overlay statistics), then the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s -rw --timeout 600 --timeout-method thread \
  tests/test_configs_gpu.py tests/test_composition_gpu.py \
  "tests/test_model_gpu.py::test_wgrad_pairs_match_unpaired" "tests/test_model_gpu.py::test_loss_curve_overlays_reference" \
  "tests/test_model_gpu.py::test_loss_curve_shipped_path_overlays_reference" > gpurun_out/r05_a_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r05_a_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r05_a_bench.json 2> gpurun_out/r05_a_bench.log || exit $?
cat gpurun_out/r05_a_bench.json
