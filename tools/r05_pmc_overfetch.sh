#!/bin/bash
# Round 5, VERDICT r04 item 6: where the compaction read's extra line fetches
# come from.  Memory-side read requests (TCC_EA0_RDREQ) of k_leaf_records and
# k_leaf_verify on 1 Mi x 4 KiB records, with the product library and with an
# experiment build whose value-tail window loads are replaced by zeros
# (tools/libnkvmerkle_notail.so, built from a patched copy of the sources:
# wrong digests, traffic only).  If the tail re-reads the record's last line
# after the L2 turned over, the experiment reads ~1 line per record less.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/${OUT:-r05e}
mkdir -p "$OUT"
for lib in product notail; do
  for cfg in records records_verify; do
    if [ $lib = notail ]; then export NKV_LIB=$PWD/tools/libnkvmerkle_notail.so; else unset NKV_LIB; fi
    timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM --output-format csv -d "$OUT/pmc_${lib}_${cfg}" \
        -o req -- python3 bench.py --config $cfg --steps 3 --warmup 1 --preroll-s 0 --no-cpu-baseline \
        --no-kernel-timing --no-capi --no-subconfigs > "$OUT/pmc_${lib}_${cfg}.log" 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/pmc_${lib}_${cfg}.log"; exit $rc; }
    echo "$lib $cfg done"
  done
done
unset NKV_LIB
echo done
