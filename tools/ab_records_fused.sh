# records form: fused k_leaf_records vs separate locate + k_leaf (same box)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_api.py tests/test_gpu_verify.py tests/test_gpu_round2.py > gpurun_out/gpu_tests_rec.txt 2>&1 || { tail -30 gpurun_out/gpu_tests_rec.txt; exit 1; }
tail -1 gpurun_out/gpu_tests_rec.txt
for i in 1 2 3; do
for cfg in "--config records --records-fused 1" "--config records --records-fused 0" ""; do
  timeout -k 10 120 python bench.py $cfg --no-cpu-baseline --steps 100 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[$cfg]', d['value'], d['ms_per_step'], d['kernel_ms'])" || exit 1
done
done
