#!/bin/bash
# Round 3 profiles: rocprofv3 kernel-trace summaries of the default bench,
# runs4 and the CRC kernel; PMC passes (each its own run) for the leaf kernel's
# VALU issue (-> the VALU ceiling in bench.py) and the CRC kernel's LDS bank
# conflicts and HBM traffic.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
B="--steps 20 --warmup 5 --preroll-s 0.2 --no-cpu-baseline --no-kernel-timing --no-clock"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/cfg2 -o cfg2 --output-format csv -- python3 bench.py $B > $O/cfg2.json 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/runs4 -o runs4 --output-format csv -- python3 bench.py --config runs4 $B > $O/runs4.json 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/crc -o crc --output-format csv -- python3 tools/bench_crc.py --steps 20 --warmup 5 > $O/crc.json 2>&1 || exit $?
P="--steps 3 --warmup 1 --preroll-s 0 --no-cpu-baseline --no-kernel-timing --no-clock"
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_valu -o valu -- python3 bench.py $P > $O/pmc_valu.json 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_crc_lds -o lds -- python3 tools/bench_crc.py --steps 3 --warmup 1 > $O/pmc_crc_lds.json 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM --output-format csv -d $O/pmc_crc_req -o req -- python3 tools/bench_crc.py --steps 3 --warmup 1 > $O/pmc_crc_req.json 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B --output-format csv -d $O/pmc_crc_sizes -o sizes -- python3 tools/bench_crc.py --steps 3 --warmup 1 > $O/pmc_crc_sizes.json 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_crc_write -o write -- python3 tools/bench_crc.py --steps 3 --warmup 1 > $O/pmc_crc_write.json 2>&1 || exit $?
echo done
