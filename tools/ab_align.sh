set -o pipefail
for args in "--key-bytes 16" "--key-bytes 34" "--key-bytes 16 --bucket 0" "--key-bytes 34 --bucket 0"; do
  timeout -k 10 150 python bench.py --config records $args --no-cpu-baseline --verify 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('records $args', d['value'], d['kernel_ms'], d.get('verified_vs_oracle'))" || exit 1
done
timeout -k 10 150 python bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('cfg2', d['value'], d['kernel_ms'])"
