# usage: tools/sweep_queue.sh "<waves list>" "<split list>"
set -o pipefail
for w in $1; do for sp in $2; do
  echo "waves=$w split=$sp"
  timeout -k 10 120 python bench.py --config mixed --deep 3 --queue-waves $w --queue-split $sp --no-cpu-baseline --steps 50 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['kernel_ms'])" || exit 1
done; done
