# cfg2 leaf load paths on the final kernel, same box, three rounds:
# 1 = LDS-DMA stage (default), 2 = direct global_load_dwordx4 into VGPRs, 4 = 128-byte runs
set -o pipefail
for i in 1 2 3; do
  for l in 1 2 4; do
    timeout -k 10 120 python bench.py --leaf-load $l --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[load $l]', d['value'], d['ms_per_step'], d['kernel_ms'])" || exit 1
  done
done
