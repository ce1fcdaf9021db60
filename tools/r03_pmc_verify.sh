#!/bin/bash
# Round 3: PMC passes on the compaction-read kernels (records_verify's
# k_leaf_verify, records' k_leaf_records): VALU issue and LDS bank conflicts.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03l
mkdir -p $O
P="--steps 3 --warmup 1 --preroll-s 0 --no-cpu-baseline --no-kernel-timing --no-clock"
for c in records_verify records; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_valu_$c -o valu -- python3 bench.py --config $c $P > $O/pmc_valu_$c.json 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_lds_$c -o lds -- python3 bench.py --config $c $P > $O/pmc_lds_$c.json 2>&1 || exit $?
done
echo done
