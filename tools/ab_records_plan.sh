set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
for cfg in "" "--config records" "--config records --bucket 0" "--config records --key-bytes 34"; do
  timeout -k 10 120 python bench.py $cfg --no-cpu-baseline --steps 100 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[$cfg]', d['value'], d['ms_per_step'], d['kernel_ms'])" || exit 1
done
done
