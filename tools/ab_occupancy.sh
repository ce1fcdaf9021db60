# cfg2 / records leaf kernel at 8 (product), 7 and 6 waves per SIMD (LDS-padded experiment builds)
set -o pipefail
for i in 1 2; do
for lib in nakevaleng_amd/libnkvmerkle.so tools/libnkvmerkle_w7.so tools/libnkvmerkle_w6.so; do
for cfg in "" "--config records"; do
  NKV_LIB=$lib timeout -k 10 120 python bench.py $cfg --no-cpu-baseline --steps 100 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[$lib $cfg]', d['value'], d['ms_per_step'], d['kernel_ms'])" || exit 1
done
done
done
