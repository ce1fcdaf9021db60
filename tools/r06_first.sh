#!/bin/bash
# Round 6, first GPU call:
#   1. pair mode's gated parity tests (NKV_TEST_QUEUE_PAIR=1), bounded spins;
#   1b. the small path's parity tests (modes 1-3: mode 3 = the resident service) and small_flush;
#   2. the lone-wave split-schedule probe;
#   3. configs[2] with pairs at 0 / 50 / 80 %, alternating x3, every root verified;
#   4. rocprofv3 --kernel-trace --stats of the default line and of each
#      sub-config's command (mixed, records, records_verify);
#   5. the mixed leaf phase's PMC traffic passes (tools/pmc_config.sh mixed).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r06a
mkdir -p $O
NKV_TEST_QUEUE_PAIR=1 timeout -k 10 420 python3 -u -m pytest tests/test_gpu_parity.py -k "side_gate or queue_pair or bucket_modes" \
    -x -v --timeout 120 --timeout-method thread > $O/pair_tests.txt 2>&1 || { tail -40 $O/pair_tests.txt; exit 1; }
tail -3 $O/pair_tests.txt
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
    print(r['shape'], r['payload_bytes'], {k: r[k]['mirror_us'] for k in ('small_pinned','small_resident','small_hbm','grid')},
          {k: r[k]['abi_us'] for k in ('small_pinned','small_resident')}, r['cpu'])
" $O/small_flush.json
NKV_LONE_SPLIT=1 timeout -k 10 120 ./tools/lone_wave.bin > $O/lone_split.txt 2>&1 || { cat $O/lone_split.txt; exit 1; }
cat $O/lone_split.txt
for rep in 1 2 3; do
  for qp in 0 50 80; do
    timeout -k 10 180 python3 bench.py --config mixed --steps 40 --warmup 5 --no-capi --no-subconfigs --no-cpu-baseline \
        --queue-pair $qp > $O/mixed_qp${qp}_${rep}.json 2> $O/mixed_qp${qp}_${rep}.err || { tail -5 $O/mixed_qp${qp}_${rep}.err; exit 1; }
    echo "queue_pair=$qp rep=$rep $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['sclk_mhz'], d['kernel_ms'], d['verified_vs_oracle'])" $O/mixed_qp${qp}_${rep}.json)"
  done
done
for cfg in sstable4k mixed records records_verify; do
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$GRAFT_REPO_ROOT/$O/prof_$cfg" -o $cfg -- python3 "$GRAFT_REPO_ROOT/bench.py" --config $cfg --steps 20 --warmup 5 \
      --no-capi --no-subconfigs --no-cpu-baseline ) > "$O/prof_$cfg.json" 2> "$O/prof_$cfg.err" \
      || { tail -5 "$O/prof_$cfg.err"; exit 1; }
  echo "rocprof $cfg: $(grep '^{' $O/prof_$cfg.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'], d['verified_vs_oracle'])")"
done
bash tools/pmc_config.sh mixed --config mixed || { echo "pmc mixed failed"; exit 1; }
echo all done
