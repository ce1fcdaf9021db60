set -o pipefail
for v in 0 1 2 3 4; do
  timeout -k 10 120 python tools/bench_crc.py --crc-load $v 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['load'], d['value'], d['ms_per_launch'])" || exit 1
done
