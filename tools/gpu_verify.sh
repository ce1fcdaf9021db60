# fused verify+tree: its GPU tests, then records vs records_verify benches on one box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_verify.py tests/test_gpu_crc.py tests/test_abi.py > gpurun_out/verify_tests.txt 2>&1 || { tail -40 gpurun_out/verify_tests.txt; exit 1; }
tail -1 gpurun_out/verify_tests.txt
for cfg in "--config records" "--config records_verify"; do
  timeout -k 10 200 python bench.py $cfg --no-cpu-baseline --verify 2>gpurun_out/bench_err.txt | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[$cfg]', d['value'], d['kernel_ms'], d['roofline']['achieved'], d.get('verified_vs_oracle'))" || { tail -20 gpurun_out/bench_err.txt; exit 1; }
done
timeout -k 10 100 python tools/bench_crc.py 2>&1 | tail -2
