#!/bin/bash
# Round 6, eighth GPU call: the small path without a device image when the
# caller asks for none (the mirrors' New): parity (every mode), the C++ mirror
# tests, small_flush with every mode, the service's phase stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_small.py tests/test_cpp_api.py -x -q -m gpu --timeout 120 \
    --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python3 bench.py --config small_flush > $O/small_flush.json 2> $O/small_flush.err \
    || { tail -5 $O/small_flush.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('small_flush', d['value'], 'cross', d['crossover_payload_bytes'], d['verified_vs_oracle'])
for r in d['shapes']:
    print(r['shape'], r['payload_bytes'], {k: r[k]['mirror_us'] for k in ('small_pinned','small_resident','small_hbm','grid') if k in r},
          {k: r[k]['abi_us'] for k in ('small_pinned','small_resident') if k in r}, r['cpu'], r['gpu_over_cpu_time'])
" $O/small_flush.json
timeout -k 5 150 python3 -u tools/svc_debug.py --limit 140 --sizes 1,10 --modes 1,3 --trace > $O/svc_trace.txt 2>&1 \
    || { cat $O/svc_trace.txt; exit 1; }
grep -E "x300|trace|close" $O/svc_trace.txt
echo all done
