# GPU suite + smoke, then records PMC (default path) and a records/cfg2 bench pair
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc3
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_tests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for v in "mem:TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" "sq:SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM"; do
  tag=${v%%:*}; ctr=${v#*:}
  timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc3 -o "rec_$tag" -- \
    python3 bench.py --config records --steps 3 --warmup 1 --preroll-s 0 --no-cpu-baseline --no-kernel-timing \
    > "gpurun_out/pmc3/rec_$tag.json" 2>&1 || exit 1
done
python3 tools/pmc_summary.py gpurun_out/pmc3 | grep -v queue
for cfg in "--config records" ""; do
  timeout -k 10 120 python bench.py $cfg --no-cpu-baseline --steps 100 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[$cfg]', d['value'], d['ms_per_step'], d['kernel_ms'])" || exit 1
done
