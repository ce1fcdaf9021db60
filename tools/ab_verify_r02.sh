# verify path (records_verify) parity + bench on one box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_verify.py tests/test_gpu_crc.py tests/test_gpu_api.py > gpurun_out/gpu_tests_verify.txt 2>&1 || { tail -30 gpurun_out/gpu_tests_verify.txt; exit 1; }
tail -1 gpurun_out/gpu_tests_verify.txt
for i in 1 2; do
for cfg in "--config records_verify" "--config records" ""; do
  timeout -k 10 120 python bench.py $cfg --no-cpu-baseline --steps 100 --verify 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[$cfg]', d['value'], d['ms_per_step'], d['kernel_ms'], d.get('verified_vs_oracle'))" || exit 1
done
done
