#!/bin/bash
# Round 3, fourth pass: the CRC lanes kernel with unconditional ping-pong line
# loads (parity tests, rate, PMC traffic and LDS), and the flush tool with the
# arena copy non-temporal vs memcpy, streaming on and off.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_crc.py -x -q --timeout 120 --timeout-method thread > $O/test_crc.txt 2>&1 || { tail -30 $O/test_crc.txt; exit 1; }
tail -2 $O/test_crc.txt
timeout -k 10 200 python -u tools/bench_crc.py --verify > $O/crc_lanes.json 2> $O/crc_lanes.err || exit $?
timeout -k 10 200 python -u tools/bench_crc.py > $O/crc_lanes_b.json 2> $O/crc_lanes_b.err || exit $?
cat $O/crc_lanes.json $O/crc_lanes_b.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/crc -o crc --output-format csv -- python3 tools/bench_crc.py --steps 20 --warmup 5 > $O/crc_prof.json 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_crc_lds -o lds -- python3 tools/bench_crc.py --steps 3 --warmup 1 > $O/pmc_crc_lds.json 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM --output-format csv -d $O/pmc_crc_req -o req -- python3 tools/bench_crc.py --steps 3 --warmup 1 > $O/pmc_crc_req.json 2>&1 || exit $?
python -c "from nakevaleng_amd import build as b; b.build_api_flush()" || exit $?
mkdir -p /tmp/af
k=0
for m in "1 1" "1 0" "0 1" "0 0" "1 1" "1 0"; do
  set -- $m
  k=$((k+1))
  timeout -k 10 120 build/api_flush 1048576 4096 4 /tmp/af $1 0x6e616b65 $2 > $O/af$k.jsonl 2> $O/af$k.err || exit $?
  tail -3 $O/af$k.jsonl | cut -c1-330
done
echo done
