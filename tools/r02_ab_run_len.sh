# cfg2: 128-byte (LOAD 4, default) vs 256-byte (LOAD 5) register runs, four alternating rounds, same box
set -o pipefail
for i in 1 2 3 4; do
  for l in 4 5; do
    timeout -k 10 120 python bench.py --leaf-load $l --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[load $l]', d['value'], d['ms_per_step'], d['kernel_ms']['leaf'])" || exit 1
  done
done
