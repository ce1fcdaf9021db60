#!/bin/bash
# Round 6: the tree levels with every lane of a working wave active (product)
# against only the live lanes (tools/libnkvmerkle_partial.so, built by
# build_exp.sh partial -DNKV_EXP_PARTIAL_REDUCE=1), the default line without
# sub-records, alternating x4 on one box; roots verified each run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2 3 4; do
  for lib in default partial; do
    if [ "$lib" = default ]; then unset NKV_LIB; else export NKV_LIB=$PWD/tools/libnkvmerkle_partial.so; fi
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --no-capi --no-subconfigs --no-cpu-baseline 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$lib', d['value'], d['kernel_ms'], d['sclk_mhz'], d.get('verified_vs_oracle'))" \
      || exit 1
  done
done
