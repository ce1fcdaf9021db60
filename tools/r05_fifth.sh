#!/bin/bash
# Round 5, fifth GPU call: the side-stream gate and the work queue's pair mode
# (parity first), the lone-wave split probe, configs[2] with and without pairs,
# the small tree's phase stamps, then the arena A/B + default rocprof
# (tools/r05_arena_ab.sh) and the over-fetch PMC passes (tools/r05_pmc_overfetch.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05f
mkdir -p $O
NKV_TEST_QUEUE_PAIR=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -k "side_gate or queue_pair or bucket_modes" -x -q \
    --timeout 120 --timeout-method thread > $O/pair_tests.txt 2>&1 || { tail -30 $O/pair_tests.txt; exit 1; }
tail -2 $O/pair_tests.txt
NKV_LONE_SPLIT=1 timeout -k 10 120 ./tools/lone_wave.bin > $O/lone_split.txt 2>&1 || { cat $O/lone_split.txt; exit 1; }
cat $O/lone_split.txt
for rep in 1 2; do
  for qp in 0 50 80; do
    timeout -k 10 180 python3 bench.py --config mixed --steps 40 --warmup 5 --no-capi --no-subconfigs --no-cpu-baseline \
        --queue-pair $qp > $O/mixed_qp${qp}_${rep}.log 2>&1 || { tail -5 $O/mixed_qp${qp}_${rep}.log; exit 1; }
    echo "queue_pair=$qp rep=$rep $(grep '^{' $O/mixed_qp${qp}_${rep}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('kernel_ms'))")"
  done
done
timeout -k 10 180 python3 bench.py --config mixed --steps 40 --warmup 5 --no-capi --no-subconfigs --no-cpu-baseline \
    --side-gate 0 > $O/mixed_sg0.log 2>&1 || { tail -5 $O/mixed_sg0.log; exit 1; }
echo "side_gate=0 $(grep '^{' $O/mixed_sg0.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
for shape in "10 1 200" "40 1 200" "256 1 200" "1024 1 200" "1024 1024 1024"; do
  timeout -k 10 120 python3 tools/small_diag.py $shape 200 50 >> $O/small_diag.jsonl 2>> $O/small_diag.err || exit $?
done
cat $O/small_diag.jsonl
OUT=r05f bash tools/r05_arena_ab.sh || exit $?
OUT=r05f bash tools/r05_pmc_overfetch.sh || exit $?
echo all done
