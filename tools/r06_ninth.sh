#!/bin/bash
# Round 6, ninth GPU call: the resident service with its requests (doorbell,
# request line, packed input) in fine-grained device memory the host stores to
# through the large BAR (NKV_OPT_SERVICE_MAILBOX 0) against host memory (1):
# probe, small-path parity, phase stamps of both forms, small_flush with both.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${OUT:-r06k}
mkdir -p $O
timeout -k 5 90 python3 -u tools/svc_debug.py --limit 75 --sizes 1,2,3,10,100,256,257,1000 > $O/svc_probe.txt 2>&1 \
    || { cat $O/svc_probe.txt; exit 1; }
grep -E "rc=|close|mailbox" $O/svc_probe.txt
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_small.py -x -q --timeout 120 --timeout-method thread \
    > $O/small_tests.txt 2>&1 || { tail -40 $O/small_tests.txt; exit 1; }
tail -1 $O/small_tests.txt
for mb in 0 1 0 1; do
    timeout -k 5 150 python3 -u tools/svc_debug.py --limit 140 --modes 3 --trace --mailbox $mb > $O/svc_trace_mb$mb.txt 2>&1 \
        || { cat $O/svc_trace_mb$mb.txt; exit 1; }
    echo "mailbox $mb"; grep -E "x300|trace|ok=False" $O/svc_trace_mb$mb.txt | cut -c1-400
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
          {k: r[k]['abi_us'] for k in K if k in r}, r['cpu'])
" $O/small_flush.json
echo all done
