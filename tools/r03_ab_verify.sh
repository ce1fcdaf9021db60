#!/bin/bash
# Round 3: records_verify with the verify kernel in 1024-thread workgroups and a 16-copy
# copies (product) against one copy (tools/libnkvmerkle_base.so), same box,
# after the verify parity tests.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_fuzz.py tests/test_gpu_round2.py tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in a b c; do
  for lib in nakevaleng_amd/libnkvmerkle.so tools/libnkvmerkle_base.so; do
    NKV_LIB=$lib timeout -k 10 200 python -u bench.py --config records_verify --no-cpu-baseline --verify > $O/rv_$(basename $lib .so)_$r.json 2> $O/rv_$(basename $lib .so)_$r.err || exit $?
    python -c "import json; d=json.load(open('$O/rv_$(basename $lib .so)_$r.json')); print('$lib $r', d['value'], d['ms_per_step'], d.get('sclk_mhz'), d['kernel_ms'], d.get('verified_vs_oracle'))"
  done
done
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_lds -o lds -- python3 bench.py --config records_verify --steps 3 --warmup 1 --preroll-s 0 --no-cpu-baseline --no-kernel-timing --no-clock > $O/pmc_lds.json 2>&1 || exit $?
echo done
