#!/bin/bash
# Round 3 check pass after the CRC / flush-path changes: smoke, the whole GPU
# suite, the default bench line (verified), the flush path, the CRC kernel, and
# the rocprofv3 summary of the default bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03y
mkdir -p $O
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 900 python -u -m pytest tests -q --timeout 120 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --verify > $O/bench_default.json 2> $O/bench_default.err || exit $?
cat $O/bench_default.json
timeout -k 10 200 python -u tools/bench_crc.py --verify > $O/crc.json 2> $O/crc.err || exit $?
cat $O/crc.json
timeout -k 10 400 python -u bench.py --config api_flush --verify > $O/api_flush.json 2> $O/api_flush.err || exit $?
python -c "import json; d=json.load(open('$O/api_flush.json')); d.pop('cycles'); print(json.dumps(d))"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/cfg2 -o cfg2 --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/cfg2_prof.json 2>&1 || exit $?
echo done
exit $rc
