# usage: tools/sweep_ring.sh <config> "<ring:waves list>" -- bench per work-queue ring depth / waves per SIMD
set -o pipefail
for rw in $2; do
  r="${rw%%:*}"; w="${rw#*:}"
  echo "config=$1 ring=$r waves=$w"
  timeout -k 10 120 python bench.py --config $1 --queue-ring $r --queue-waves $w --no-cpu-baseline --steps 50 --verify 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['kernel_ms'], d.get('verified_vs_oracle'))" || exit 1
done
