#!/bin/bash
# Round 6, second GPU call:
#   1. the counters this box offers (rocprofv3 -L);
#   2. k_leaf_records' issue gap: the product against two prefetch experiments
#      (tools/build_exp.sh rec1 -DNKV_EXP_REC=1: four segment sets, each line one
#      block ahead, 4 waves/SIMD; rec2 -DNKV_EXP_REC=2: three sets, each 64-B
#      segment one block ahead, 5 waves/SIMD), alternating x3, roots verified;
#   3. SQ counters of k_leaf<0,4> (cfg2) and k_leaf_records: VALU issue, waits;
#   4. PMC traffic of records and records_verify on this build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || { tail -5 $O/counters.txt; exit 1; }
B="--steps 40 --warmup 5 --no-capi --no-subconfigs --no-cpu-baseline"
for rep in 1 2 3; do
  for lib in product rec1 rec2; do
    if [ $lib = product ]; then unset NKV_LIB; else export NKV_LIB=$PWD/tools/libnkvmerkle_$lib.so; fi
    timeout -k 10 180 python3 bench.py --config records $B > $O/rec_${lib}_$rep.json 2> $O/rec_${lib}_$rep.err \
        || { tail -5 $O/rec_${lib}_$rep.err; exit 1; }
    echo "records $lib rep=$rep $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['sclk_mhz'], d['kernel_ms']['leaf'], d['roofline']['valu_frac'], d['verified_vs_oracle'])" $O/rec_${lib}_$rep.json)"
  done
done
for lib in product rec1 rec2; do
  if [ $lib = product ]; then unset NKV_LIB; else export NKV_LIB=$PWD/tools/libnkvmerkle_$lib.so; fi
  timeout -k 10 180 python3 bench.py --config records_verify $B > $O/ver_${lib}.json 2> $O/ver_${lib}.err \
      || { tail -5 $O/ver_${lib}.err; exit 1; }
  echo "records_verify $lib $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['sclk_mhz'], d['kernel_ms']['leaf'], d['roofline']['valu_frac'], d['verified_vs_oracle'], d.get('crc_checked'))" $O/ver_${lib}.json)"
done
unset NKV_LIB
P="--steps 3 --warmup 1 --preroll-s 0 --no-cpu-baseline --no-kernel-timing --no-clock --no-capi --no-subconfigs"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
for c in SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD; do
  grep -qw "$c" $O/counters.txt && echo "$c listed"
done
for cfg in sstable4k records; do
  timeout -s KILL 90 rocprofv3 --pmc $SQ --output-format csv -d $O/pmc_sq_$cfg -o sq -- python3 bench.py --config $cfg $P \
      > $O/pmc_sq_$cfg.log 2>&1 || { tail -5 $O/pmc_sq_$cfg.log; exit 1; }
  W=""
  for c in SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY; do grep -qw "$c" $O/counters.txt && W="$W $c"; done
  if [ -n "$W" ]; then
    timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES $W --output-format csv -d $O/pmc_wait_$cfg -o wait -- \
        python3 bench.py --config $cfg $P > $O/pmc_wait_$cfg.log 2>&1 || { tail -5 $O/pmc_wait_$cfg.log; exit 1; }
  fi
  echo "pmc $cfg done"
done
bash tools/pmc_config.sh records --config records || { echo "pmc records failed"; exit 1; }
bash tools/pmc_config.sh records_verify --config records_verify || { echo "pmc records_verify failed"; exit 1; }
echo all done
