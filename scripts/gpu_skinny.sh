# Skinny decode GEMM: numerics, small-batch bench A/B (tuned table vs library only), headline.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "skinny or tuned_linear" > gpurun_out/skinny_test.log 2>&1 && tail -3 gpurun_out/skinny_test.log &&
for b in ${BATCHES:-1 4 16}; do
  timeout -k 10 200 python -u bench.py --batch $b --steps 3 --warmup 1 > gpurun_out/b${b}_skinny.log 2>&1 && tail -1 gpurun_out/b${b}_skinny.log | cut -c1-420 &&
  DRTC_SKINNY_MAX_M=0 timeout -k 10 200 python -u bench.py --batch $b --steps 3 --warmup 1 > gpurun_out/b${b}_lt.log 2>&1 && tail -1 gpurun_out/b${b}_lt.log | cut -c1-420 || exit 1
done
