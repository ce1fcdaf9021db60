#!/bin/bash
# Round 6, third GPU call: the resident small-tree service after the
# wave-uniform control-flow fix (probe, then its parity tests and small_flush
# with every mode), then tools/r06_second.sh (records experiments, PMC).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r06c
mkdir -p $O
timeout -k 5 90 python3 -u tools/svc_debug.py --limit 75 > $O/svc_debug.txt 2>&1
rc=$?; echo "svc_debug rc=$rc"; cat $O/svc_debug.txt
if [ $rc -eq 0 ]; then
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_small.py -x -v --timeout 120 --timeout-method thread \
      > $O/small_tests.txt 2>&1 || { tail -40 $O/small_tests.txt; exit 1; }
  tail -3 $O/small_tests.txt
  timeout -k 10 300 python3 bench.py --config small_flush > $O/small_flush.json 2> $O/small_flush.err \
      || { tail -5 $O/small_flush.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('small_flush', d['value'], 'cross', d['crossover_payload_bytes'], d['verified_vs_oracle'])
for r in d['shapes']:
    print(r['shape'], r['payload_bytes'], {k: r[k]['mirror_us'] for k in ('small_pinned','small_resident','small_hbm','grid') if k in r},
          {k: r[k]['abi_us'] for k in ('small_pinned','small_resident') if k in r}, r['cpu'])
" $O/small_flush.json
fi
bash tools/r06_second.sh
