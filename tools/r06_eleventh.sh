#!/bin/bash
# Round 6, eleventh GPU call: the small-tree kernels with every lane of a
# working wave active (sha1_value_all_lanes, the levels likewise): parity of the
# small path, the interleaved mailbox A/B with each launch's phases and CU
# (the per-CU spread should be gone), small_flush with modes 1, 3 and 3h.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${OUT:-r06n}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_small.py tests/test_gpu_parity.py -x -q --timeout 120 \
    --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 5 170 python3 -u tools/svc_ab.py --rounds 12 --calls 300 --limit 160 > $O/svc_ab.txt 2>&1 \
    || { cat $O/svc_ab.txt; exit 1; }
grep -v "n=40" $O/svc_ab.txt | cut -c1-260
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
