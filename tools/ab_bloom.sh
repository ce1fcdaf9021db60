set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bloom.py > gpurun_out/tb.txt 2>&1 || { tail -30 gpurun_out/tb.txt; exit 1; }
tail -1 gpurun_out/tb.txt
for rep in 1 2; do for p in 1 2; do
  timeout -k 10 120 python tools/bench_bloom.py --path $p --verify 2>/dev/null | tail -1 | cut -c1-300 || exit 1
done; done
