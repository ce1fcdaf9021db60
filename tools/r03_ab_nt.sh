#!/bin/bash
# Round 3: cfg2 with the leaf kernel's line loads non-temporal (global_load
# ... nt: tools/libnkvmerkle_nt.so, built by tools/build_exp.sh nt -DNKV_EXP_NT
# from a one-line change to sha1_blocks_runs) against the product, same box.
# Question: does a streaming cache policy lower the data path's power enough
# to raise the shader clock?
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03s
mkdir -p $O
for r in a b c; do
  for lib in nakevaleng_amd/libnkvmerkle.so tools/libnkvmerkle_nt.so; do
    NKV_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --verify > $O/cfg2_$(basename $lib .so)_$r.json 2> $O/cfg2_$(basename $lib .so)_$r.err || exit $?
    python -c "import json; d=json.load(open('$O/cfg2_$(basename $lib .so)_$r.json')); print('$lib $r', d['value'], d['ms_per_step'], d.get('sclk_mhz'), d['kernel_ms'], d['roofline']['valu_frac'], d.get('verified_vs_oracle'))"
  done
done
NKV_LIB=tools/libnkvmerkle_nt.so timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_nt -o req -- python3 bench.py --steps 3 --warmup 1 --preroll-s 0 --no-cpu-baseline --no-kernel-timing --no-clock > $O/pmc_nt.json 2>&1 || exit $?
echo done
