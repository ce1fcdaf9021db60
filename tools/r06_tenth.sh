#!/bin/bash
# Round 6, tenth GPU call: why the resident service's compute phases depend on
# the CU it lands on (tools/svc_ab.py: leaves 5.5-7.3 us by CU at one clock) --
# instruction-cache counters of the service per dispatch, one pass each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${OUT:-r06l}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ -d $O/p1 -o run \
    --output-format csv -- python3 -u tools/svc_pmc.py --calls 40 --limit 80 > $O/p1.txt 2>&1 || { tail -20 $O/p1.txt; exit 1; }
tail -2 $O/p1.txt
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -d $O/p2 -o run \
    --output-format csv -- python3 -u tools/svc_pmc.py --calls 40 --limit 80 > $O/p2.txt 2>&1 || { tail -20 $O/p2.txt; exit 1; }
tail -2 $O/p2.txt
find $O -name "*counter_collection.csv" | head
echo all done
