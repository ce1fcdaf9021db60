# Records leaf kernel, round 2: memory-side reads and issue counters for the
# 80-byte window stage (LOAD 10), the register segment stage (LOAD 11), 64-B
# aligned values (--key-bytes 34) and cfg2.  One --pmc pass per counter group.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc2
run() {  # tag, counters, bench args...
  local tag=$1 ctr=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc2 -o "$tag" -- \
    python3 bench.py "$@" --steps 3 --warmup 1 --preroll-s 0 --no-cpu-baseline --no-kernel-timing \
    > "gpurun_out/pmc2/$tag.json" 2>&1
}
MEM="TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM"
for v in "l10:--config records --leaf-load 10" "l11:--config records --leaf-load 11" "kb34:--config records --key-bytes 34" "cfg2:"; do
  tag=${v%%:*}; args=${v#*:}
  run "${tag}_mem" "$MEM" $args || exit 1
  run "${tag}_sq" "$SQ" $args || exit 1
done
python3 tools/pmc_summary.py gpurun_out/pmc2
