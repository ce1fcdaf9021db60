# A/B over several experiment libraries (tools/libnkvmerkle_<tag>.so) and the product, same box
#   bash tools/ab_tags.sh "<cfg>" tag1 tag2 ...
set -o pipefail
cfg=$1; shift
for i in 1 2; do
for lib in nakevaleng_amd/libnkvmerkle.so "$@"; do
  [ -f "$lib" ] || lib=tools/libnkvmerkle_$lib.so
  NKV_LIB=$lib timeout -k 10 120 python bench.py $cfg --no-cpu-baseline --steps 100 --verify 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[$lib $cfg]', d['value'], d['ms_per_step'], d['kernel_ms'], d.get('verified_vs_oracle'))" || exit 1
done
done
