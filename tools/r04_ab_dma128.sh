# Round 4 experiment: 128-byte runs per value through an 8 KiB LDS-DMA stage
# (every DMA instruction fetching 8 whole lines), default cache policy (dma0)
# and non-temporal (dma2), against the product's register runs; libraries
# built by tools/build_exp.sh dma<aux> -DNKV_EXP_DMA128=<aux> with tools/exp/r04_dma128.patch
# applied (git apply; the experiment is not in the product sources).  Same box,
# round-robin x3, every root verified against the committed roots.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
one() {  # lib, bench args
  local lib=$1; shift
  if [ "$lib" = product ]; then unset NKV_LIB; else export NKV_LIB=$PWD/tools/libnkvmerkle_$lib.so; fi
  timeout -k 10 200 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-capi "$@" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$lib', '$*', d['value'], d['ms_per_step'], d['kernel_ms'], d['sclk_mhz'], d['roofline']['valu_frac'], d.get('verified_vs_oracle'))"
}
for rep in 1 2 3; do
  one product || exit 1; one dma0 || exit 1; one dma2 || exit 1
done
unset NKV_LIB
