# usage: bash tools/ab_libs.sh "<bench args>" lib1 lib2 ... -- the same bench.py
# line against several builds of the library (nakevaleng_amd/libnkv_<name>.so,
# "default" = libnkvmerkle.so) on one box, round-robin twice, one line each.
set -o pipefail
args="$1"; shift
for rep in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = default ]; then unset NKV_LIB; else export NKV_LIB=$PWD/nakevaleng_amd/libnkv_$lib.so; fi
    timeout -k 10 150 python bench.py $args --no-cpu-baseline --verify 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$lib [$args]', d['value'], d['kernel_ms'], d.get('verified_vs_oracle'))" || exit 1
  done
done
