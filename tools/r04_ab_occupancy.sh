# Round 4: occupancy of the three register-run leaf kernels, each one step up
# (launch bounds; the compiler spills a few registers to get there):
#   k_leaf<0, 4>   7 -> 8 waves/SIMD (66 -> 64 VGPRs)   libnkv_w8.so  (cfg2)
#   k_leaf_records 5 -> 6 (86 -> 80)                   libnkv_r6.so  (--config records)
#   k_leaf_verify  4 -> 5 (105 -> 96)                  libnkv_v5.so  (--config records_verify)
# Same box, round-robin x3, every root verified against the committed roots.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
one() {  # lib, bench args
  local lib=$1; shift
  if [ "$lib" = default ]; then unset NKV_LIB; else export NKV_LIB=$PWD/nakevaleng_amd/libnkv_$lib.so; fi
  timeout -k 10 200 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-capi "$@" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$lib', '$*', d['value'], d['kernel_ms']['leaf'], d['sclk_mhz'], d['roofline']['valu_frac'], d.get('verified_vs_oracle'))"
}
for rep in 1 2 3; do
  one default || exit 1; one w8 || exit 1
  one default --config records || exit 1; one r6 --config records || exit 1
  one default --config records_verify || exit 1; one v5 --config records_verify || exit 1
done
