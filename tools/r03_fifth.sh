#!/bin/bash
# Round 3, fifth pass: CRC lanes kernel, past-span lanes on a cache-resident
# dummy line, header + head word + first line issued together (CRC_LOAD 0), and the span-group form (8).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_crc.py -x -q --timeout 120 --timeout-method thread > $O/test_crc.txt 2>&1 || { tail -30 $O/test_crc.txt; exit 1; }
tail -2 $O/test_crc.txt
for r in a b; do
  for v in 0 1; do
    timeout -k 10 200 python -u tools/bench_crc.py --verify --crc-load $v > $O/crc_v${v}_$r.json 2> $O/crc_v${v}_$r.err || exit $?
    python -c "import json; d=json.load(open('$O/crc_v${v}_$r.json')); print('v$v $r', d['value'], d['ms_per_launch'], d.get('verified_vs_oracle'))"
  done
done
for v in 0 1; do
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_req_v$v -o req -- python3 tools/bench_crc.py --steps 3 --warmup 1 --crc-load $v > $O/pmc_req_v$v.json 2>&1 || exit $?
done
echo done
