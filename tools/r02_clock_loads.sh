# in-kernel shader clock of the cfg2 leaf kernel: LDS-DMA stage (LOAD 1) vs
# 128-byte register runs (LOAD 4), stamp build (never the product)
set -o pipefail
mkdir -p gpurun_out/clk
timeout -k 10 300 python nakevaleng_amd/build.py --diag > /dev/null || exit 1
i=0
for l in 1 4 1 4; do
  i=$((i+1))
  NKV_LEAF_LOAD=$l timeout -k 10 120 python tools/diag_timeline.py > gpurun_out/clk/load${l}_$i.txt 2>/dev/null || exit 1
  echo "== LOAD $l"; head -3 gpurun_out/clk/load${l}_$i.txt
done
