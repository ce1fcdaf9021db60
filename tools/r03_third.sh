#!/bin/bash
# Round 3, third pass: the CRC kernel after the scratch fix, mixed (configs[2])
# with two tables per step against one after another, records / records_verify
# after the pruning, api_flush with the non-temporal arena copy, then tools/r03_pmc.sh (kernel summaries and PMC passes).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 200 python -u tools/bench_crc.py --verify > $O/crc_lanes.json 2> $O/crc_lanes.err || exit $?
timeout -k 10 200 python -u tools/bench_crc.py --crc-load 8 > $O/crc_group.json 2> $O/crc_group.err || exit $?
cat $O/crc_lanes.json $O/crc_group.json
N="--no-cpu-baseline"
timeout -k 10 300 python -u bench.py --config mixed $N --verify > $O/mixed.json 2> $O/mixed.err || exit $?
timeout -k 10 300 python -u bench.py --config mixed --tables 2 $N --verify > $O/mixed2.json 2> $O/mixed2.err || exit $?
timeout -k 10 300 python -u bench.py --config mixed --tables 2 --table-lanes 1 $N > $O/mixed2_serial.json 2> $O/mixed2_serial.err || exit $?
timeout -k 10 300 python -u bench.py --config mixed $N > $O/mixed_b.json 2> $O/mixed_b.err || exit $?
timeout -k 10 300 python -u bench.py --config mixed --tables 2 $N > $O/mixed2_b.json 2> $O/mixed2_b.err || exit $?
timeout -k 10 300 python -u bench.py --config mixed --tables 2 --table-lanes 1 $N > $O/mixed2_serial_b.json 2> $O/mixed2_serial_b.err || exit $?
timeout -k 10 300 python -u bench.py --config records $N --verify > $O/records.json 2> $O/records.err || exit $?
timeout -k 10 300 python -u bench.py --config records_verify $N --verify > $O/records_verify.json 2> $O/records_verify.err || exit $?
for f in mixed mixed2 mixed2_serial mixed_b mixed2_b mixed2_serial_b records records_verify; do python -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d.get('sclk_mhz'), d['kernel_ms'], d.get('verified_vs_oracle'))"; done
timeout -k 10 600 python -u bench.py --config api_flush --verify > $O/api_flush.json 2> $O/api_flush.err || exit $?
cat $O/api_flush.json
bash tools/r03_pmc.sh
