#!/bin/bash
# Round 6: the work queue's blocks compressed by every lane (product) against
# only the live lanes (tools/libnkvmerkle_partialring.so: build_exp.sh
# partialring -DNKV_EXP_PARTIAL_RING=1), configs[2] (--config mixed) without
# sub-records, alternating x4 on one box; roots verified each run.  Reproduces
# only on commit d4a64e5 (the switch was removed with the change: no gain).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2 3 4; do
  for lib in default partialring; do
    if [ "$lib" = default ]; then unset NKV_LIB; else export NKV_LIB=$PWD/tools/libnkvmerkle_partialring.so; fi
    timeout -k 10 200 python3 bench.py --config mixed --steps 20 --warmup 5 --no-capi --no-subconfigs \
      --no-cpu-baseline 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$lib', d['value'], d['kernel_ms'], d['sclk_mhz'], d.get('verified_vs_oracle'))" \
      || exit 1
  done
done
