# L1->L2 read requests and memory-side reads of the records leaf kernel, value at +46 (window stage)
# against +64 (64-B aligned values, LOAD 1): does the slower form issue more line requests?
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcr
for kb in 16 34; do
  timeout -s KILL 90 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_EA0_RDREQ GRBM_GUI_ACTIVE \
    --output-format csv -d gpurun_out/pmcr -o "kb$kb" -- \
    python3 bench.py --config records --key-bytes $kb --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing \
    > "gpurun_out/pmcr/kb$kb.json" 2>&1 || exit 1
done
