# GPU suite, then the records config under rocprofv3 (k_locate's mean duration) and plain
set -o pipefail
mkdir -p gpurun_out/prof
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/gpu_tests.txt
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o records -- python3 bench.py --config records --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/prof/records.json 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --config records --no-cpu-baseline --verify 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('records', d['value'], d['kernel_ms'], d.get('verified_vs_oracle'))" || exit 1
done
