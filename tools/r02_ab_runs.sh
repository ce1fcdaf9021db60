# cfg2: LDS-DMA stage (load 1, product default) vs 128-byte runs into VGPRs
# (load 4) at 4 / 5 / 6 waves per SIMD, with and without one run of
# register lookahead (experiment libraries tools/libnkvmerkle_{w5,w6,pf,pf5}.so), same box
set -o pipefail
run() {  # lib load tag
  NKV_LIB=$1 timeout -k 10 120 python bench.py --leaf-load $2 --no-cpu-baseline --verify 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[$3]', d['value'], d['ms_per_step'], d['kernel_ms'], d.get('verified_vs_oracle'))" || exit 1
}
P=nakevaleng_amd/libnkvmerkle.so
for i in 1 2; do
  run $P 1 "load1 (stage, 8 w)" || exit 1
  run $P 4 "load4 (runs, 4 w)" || exit 1
  run tools/libnkvmerkle_w5.so 4 "load4 5 w" || exit 1
  run tools/libnkvmerkle_w6.so 4 "load4 6 w" || exit 1
  run tools/libnkvmerkle_pf.so 4 "load4 pf 4 w" || exit 1
  run tools/libnkvmerkle_pf5.so 4 "load4 pf 5 w" || exit 1
  run $P 5 "load5 (256-B runs, 4 w)" || exit 1
done
