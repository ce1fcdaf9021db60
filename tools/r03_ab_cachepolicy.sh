#!/bin/bash
# Round 3: cfg2 with the leaf kernel's line loads issued by inline asm with
# cache-policy bits (tools/build_exp.sh <tag> -DNKV_EXP_CP=...): "" (the same
# asm and explicit wait, no bits: the control), sc0, sc1 -- against the
# product, same box.  Question: does a different L1/L2 policy for the
# streamed lines lower the data path's power and raise the clock?
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03u
mkdir -p $O
for r in a b; do
  for lib in nakevaleng_amd/libnkvmerkle.so tools/libnkvmerkle_asm.so tools/libnkvmerkle_sc0.so tools/libnkvmerkle_sc1.so; do
    tag=$(basename $lib .so)
    NKV_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --verify > $O/cfg2_${tag}_$r.json 2> $O/cfg2_${tag}_$r.err || exit $?
    python -c "import json; d=json.load(open('$O/cfg2_${tag}_$r.json')); print('$tag $r', d['value'], d['ms_per_step'], d.get('sclk_mhz'), d['kernel_ms']['leaf'], d['roofline']['valu_frac'], d.get('verified_vs_oracle'))"
  done
done
echo done
