#!/bin/bash
# Round 3: the C++ mirror after the inline-digest Data type and the reserved
# node pool: its GPU test, then the flush path end to end twice; rocprofv3
# kernel summaries of records, records_verify and mixed.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_cpp_api.py -x -q --timeout 200 --timeout-method thread > $O/test_cpp.txt 2>&1 || { tail -30 $O/test_cpp.txt; exit 1; }
tail -1 $O/test_cpp.txt
for r in a b; do
  timeout -k 10 400 python -u bench.py --config api_flush --verify > $O/api_flush_$r.json 2> $O/api_flush_$r.err || exit $?
  python -c "import json; d=json.load(open('$O/api_flush_$r.json')); d.pop('cycles'); print(json.dumps(d))"
done
B="--steps 20 --warmup 5 --preroll-s 0.2 --no-cpu-baseline --no-kernel-timing --no-clock"
for c in records records_verify mixed; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/$c -o $c --output-format csv -- python3 bench.py --config $c $B > $O/${c}_prof.json 2>&1 || exit $?
done
echo done
