set -u
mkdir -p gpurun_out
for v in fold512 fold768; do
  PICO_LIB_PATH=picotron_amd/lib/variants/$v.so timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -q -k "cross_entropy" --timeout 120 --timeout-method thread > gpurun_out/t_$v.log 2>&1 || exit $?
done
for r in 1 2 3; do for v in ce256 fold256 fold512 fold768; do
  PICO_LIB_PATH=picotron_amd/lib/variants/$v.so timeout -k 10 120 python scripts/kernel_bench.py 2>/dev/null | grep cross_entropy | sed "s/^{/{\"variant\": \"$v\", /" >> gpurun_out/ce_ab.jsonl || exit $?
done; done
