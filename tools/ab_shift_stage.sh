# LOAD 11 (register stage, uniform misalignment) parity, then records A/B vs LOAD 10
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "line_pair or shift_stage" > gpurun_out/shift_tests.txt 2>&1 || { tail -30 gpurun_out/shift_tests.txt; exit 1; }
tail -2 gpurun_out/shift_tests.txt
for i in 1 2; do
for cfg in "--config records --leaf-load 10" "--config records --leaf-load 11" "--config records --leaf-load 11 --bucket 0" ""; do
  timeout -k 10 120 python bench.py $cfg --no-cpu-baseline --steps 100 --verify 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[$cfg]', d['value'], d['ms_per_step'], d['kernel_ms'], d.get('verified_vs_oracle'))" || exit 1
done
done
