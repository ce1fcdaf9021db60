# usage: tools/ab_bench.sh "<label>|<bench args>" ... -- several bench.py variants on one box, one line each
set -o pipefail
for spec in "$@"; do
  label="${spec%%|*}"; args="${spec#*|}"
  timeout -k 10 150 python bench.py $args --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$label', d['value'], d['kernel_ms'], d.get('verified_vs_oracle'))" || exit 1
done
