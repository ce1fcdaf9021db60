# same-box step ratio records / cfg2 (and mixed, records_verify) with the final library, alternating, no profiler
set -o pipefail
for i in 1 2 3; do
  for cfg in "" "--config records" "--config records_verify" "--config mixed"; do
    timeout -k 10 200 python bench.py $cfg --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[$cfg]', d['value'], d['ms_per_step'], d['kernel_ms']['leaf'], d['roofline']['frac'], d['roofline']['traffic'])" || exit 1
  done
done
