#!/bin/bash
# Round 6, thirteenth GPU call: the one-launch small path's packed input in
# BAR-mapped device memory (NKV_OPT_SERVICE_MAILBOX 0): small-path parity,
# latency of modes 1 and 3 (svc_debug), small_flush with 1, 3, 3h (3h: host
# memory for both the service and, in that process, the one-launch input).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${OUT:-r06q}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_small.py tests/test_cpp_api.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for mb in 0 1; do
  timeout -k 5 120 python3 -u tools/svc_debug.py --limit 110 --modes 1,3 --mailbox $mb > $O/svc_mb$mb.txt 2>&1 \
      || { cat $O/svc_mb$mb.txt; exit 1; }
  echo "mailbox $mb"; grep -E "x300|ok=False" $O/svc_mb$mb.txt | cut -c1-120
done
timeout -k 10 300 python3 bench.py --config small_flush --small-modes 1,3,3h > $O/small_flush.json 2> $O/small_flush.err \
    || { tail -5 $O/small_flush.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('small_flush', d['value'], 'cross', d['crossover_payload_bytes'], d['verified_vs_oracle'])
K=('small_pinned','small_resident','small_resident_host_mailbox')
for r in d['shapes']:
    print(r['shape'], r['payload_bytes'], {k: r[k]['mirror_us'] for k in K if k in r},
          {k: r[k]['abi_us'] for k in K if k in r}, r['cpu']['openssl_1core_us'])
" $O/small_flush.json
echo all done
