#!/bin/bash
# Round 5, fourth GPU call: the arena coherence A/B and the default line's
# rocprof summary (tools/r05_arena_ab.sh), then the over-fetch PMC passes
# (tools/r05_pmc_overfetch.sh), the small tree's phase stamps, and the
# gated kernel on the side stream against the same stream (configs[2]).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=r05d bash tools/r05_arena_ab.sh || exit $?
OUT=r05e bash tools/r05_pmc_overfetch.sh || exit $?
for shape in "10 1 200" "40 1 200" "256 1 200" "1024 1 200" "1024 1024 1024"; do
  timeout -k 10 120 python3 tools/small_diag.py $shape 200 50 >> gpurun_out/r05e/small_diag.jsonl 2>> gpurun_out/r05e/small_diag.err || exit $?
done
cat gpurun_out/r05e/small_diag.jsonl
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "side_gate or bucket_modes" -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/r05e/side_gate_tests.txt 2>&1 || { tail -20 gpurun_out/r05e/side_gate_tests.txt; exit 1; }
tail -2 gpurun_out/r05e/side_gate_tests.txt
for rep in 1 2; do
  for sg in 1 0; do
    timeout -k 10 180 python3 bench.py --config mixed --steps 40 --warmup 5 --no-capi --no-subconfigs --no-cpu-baseline \
        --side-gate $sg > gpurun_out/r05e/mixed_sg${sg}_${rep}.log 2>&1 || { tail -5 gpurun_out/r05e/mixed_sg${sg}_${rep}.log; exit 1; }
    echo "side_gate=$sg rep=$rep $(grep '^{' gpurun_out/r05e/mixed_sg${sg}_${rep}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
echo all done
