# A/B: product library vs an experiment library (tools/libnkvmerkle_<tag>.so) on given configs
#   bash tools/ab_lib.sh <tag> "<cfg1>" "<cfg2>" ...
set -o pipefail
tag=$1; shift
for i in 1 2; do
for lib in nakevaleng_amd/libnkvmerkle.so tools/libnkvmerkle_$tag.so; do
for cfg in "$@"; do
  NKV_LIB=$lib timeout -k 10 120 python bench.py $cfg --no-cpu-baseline --steps 100 --verify 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[$lib $cfg]', d['value'], d['ms_per_step'], d['kernel_ms'], d.get('verified_vs_oracle'))" || exit 1
done
done
done
