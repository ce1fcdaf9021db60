#!/bin/bash
# Round 3, first GPU pass: the new entries' tests, the GPU suite, the default
# bench line (clock probe), runs4 (4 tables per step) against the same tables
# one after another, and the capi group backend (one process, RCCL) at N = 1.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }  # 1 = test failures (no crash): keep going
true
true
timeout -k 10 300 python -u bench.py --verify > $O/bench_default.json 2> $O/bench_default.err || exit $?
echo default; cat $O/bench_default.json
timeout -k 10 300 python -u bench.py --config runs4 --no-cpu-baseline --verify > $O/runs4.json 2> $O/runs4.err || exit $?
timeout -k 10 300 python -u bench.py --config runs4 --table-lanes 1 --no-cpu-baseline > $O/runs4_serial.json 2> $O/runs4_serial.err || exit $?
timeout -k 10 300 python -u bench.py --config runs4 --no-cpu-baseline > $O/runs4_b.json 2> $O/runs4_b.err || exit $?
timeout -k 10 300 python -u bench.py --config runs4 --table-lanes 1 --no-cpu-baseline > $O/runs4_serial_b.json 2> $O/runs4_serial_b.err || exit $?
for f in runs4 runs4_serial runs4_b runs4_serial_b; do python -c "import json,sys; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d.get('sclk_mhz'), d.get('verified_vs_oracle'))"; done
timeout -k 10 300 python -u bench.py --backend capi --no-cpu-baseline --verify > $O/capi.json 2> $O/capi.err || exit $?
echo capi; cat $O/capi.json
timeout -k 10 300 python -u bench.py --backend capi --config one_tree --verify > $O/capi_one_tree.json 2> $O/capi_one_tree.err || exit $?
echo capi_one_tree; cat $O/capi_one_tree.json
timeout -k 10 400 python -u bench.py --config api_flush --verify > $O/api_flush.json 2> $O/api_flush.err || exit $?
echo api_flush; python -c "import json; d=json.load(open('$O/api_flush.json')); d.pop('cycles'); print(json.dumps(d))"
timeout -k 10 200 python -u tools/bench_crc.py --verify > $O/crc_lanes.json 2> $O/crc_lanes.err || exit $?
timeout -k 10 200 python -u tools/bench_crc.py --crc-load 8 > $O/crc_group.json 2> $O/crc_group.err || exit $?
echo crc; cat $O/crc_lanes.json $O/crc_group.json
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -q --timeout 120 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -3 $O/pytest_gpu.log
exit $rc
