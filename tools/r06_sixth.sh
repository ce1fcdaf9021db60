#!/bin/bash
# Round 6, sixth GPU call: the resident service with its request read as one
# line and one 256-thread workgroup (n <= 256): parity (every small-path mode),
# phase stamps and small_flush.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${OUT:-r06f}
mkdir -p $O
timeout -k 5 90 python3 -u tools/svc_debug.py --limit 75 --sizes 1,2,3,10,100,256,257,1000 > $O/svc_probe.txt 2>&1 \
    || { cat $O/svc_probe.txt; exit 1; }
grep -E "rc=|close" $O/svc_probe.txt
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_small.py -x -q --timeout 120 --timeout-method thread \
    > $O/small_tests.txt 2>&1 || { tail -40 $O/small_tests.txt; exit 1; }
tail -1 $O/small_tests.txt
timeout -k 5 150 python3 -u tools/svc_debug.py --limit 140 --modes 1,3 --trace > $O/svc_trace.txt 2>&1 \
    || { cat $O/svc_trace.txt; exit 1; }
grep -E "x300|trace|close|ok=False" $O/svc_trace.txt
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
echo all done
