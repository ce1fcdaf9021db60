#!/bin/bash
# Round 6, fourth GPU call:
#   1. the small path's completion with one release per workgroup (this build)
#      against the per-wave fences (tools/oldfence/libnkvmerkle.so), modes 1 and 3,
#      alternating x2 (tools/svc_debug.py --modes);
#   2. the small path's parity tests (every mode) and small_flush (every mode);
#   3. where the compaction read's extra line fetches come from: memory-side read
#      requests of k_leaf_records / k_leaf_verify with the product library, with
#      no tail-window load (-DNKV_EXP_NOTAIL) and with no header-size load
#      (-DNKV_EXP_FIXEDHDR); traffic only, the experiment digests are wrong.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r06d
mkdir -p $O
for rep in 1 2; do
  for lib in product oldfence; do
    if [ $lib = product ]; then unset NKV_LIB; else export NKV_LIB=$PWD/tools/oldfence/libnkvmerkle.so; fi
    timeout -k 5 120 python3 -u tools/svc_debug.py --limit 100 --modes 1,3 > $O/svc_${lib}_$rep.txt 2>&1 \
        || { cat $O/svc_${lib}_$rep.txt; exit 1; }
    echo "$lib rep=$rep"; grep -E "x300|close|ok=False" $O/svc_${lib}_$rep.txt
  done
done
unset NKV_LIB
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_small.py -x -v --timeout 120 --timeout-method thread \
    > $O/small_tests.txt 2>&1 || { tail -40 $O/small_tests.txt; exit 1; }
tail -2 $O/small_tests.txt
timeout -k 10 300 python3 bench.py --config small_flush > $O/small_flush.json 2> $O/small_flush.err \
    || { tail -5 $O/small_flush.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('small_flush', d['value'], 'cross', d['crossover_payload_bytes'], d['verified_vs_oracle'])
for r in d['shapes']:
    print(r['shape'], r['payload_bytes'], {k: r[k]['mirror_us'] for k in ('small_pinned','small_resident','small_hbm','grid') if k in r},
          {k: r[k]['abi_us'] for k in ('small_pinned','small_resident') if k in r}, r['cpu'])
" $O/small_flush.json
export TMPDIR=/tmp
for lib in product notail fixedhdr; do
  for cfg in records records_verify; do
    if [ $lib = product ]; then unset NKV_LIB; else export NKV_LIB=$PWD/tools/libnkvmerkle_$lib.so; fi
    timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM --output-format csv -d "$O/pmc_${lib}_${cfg}" \
        -o req -- python3 bench.py --config $cfg --steps 3 --warmup 1 --preroll-s 0 --no-cpu-baseline \
        --no-kernel-timing --no-capi --no-subconfigs > "$O/pmc_${lib}_${cfg}.log" 2>&1 \
        || { tail -5 "$O/pmc_${lib}_${cfg}.log"; exit 1; }
    echo "pmc $lib $cfg done"
  done
done
unset NKV_LIB
echo all done
