#!/bin/bash
# Round 6, fifth GPU call: the whole GPU suite and smoke() on this build, then
# where a small flush's time goes -- the resident service's phase stamps
# (tools/svc_debug.py --trace) and the one-launch kernel's (tools/small_diag.py,
# the NKV_DIAG stamp build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r06e
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_suite.txt 2>&1 \
    || { tail -40 $O/gpu_suite.txt; exit 1; }
tail -3 $O/gpu_suite.txt
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 5 150 python3 -u tools/svc_debug.py --limit 140 --modes 1,3 --trace > $O/svc_trace.txt 2>&1 \
    || { cat $O/svc_trace.txt; exit 1; }
grep -E "x300|trace|close|ok=False" $O/svc_trace.txt
for shape in "10 1 200" "40 1 200" "256 1 200"; do
  timeout -k 10 120 python3 tools/small_diag.py $shape 200 50 >> $O/small_diag.jsonl 2>> $O/small_diag.err || { tail -5 $O/small_diag.err; exit 1; }
done
cat $O/small_diag.jsonl
echo all done
