# read-request sizes at the L2's memory side (TCC_EA0_RDREQ_{32B,64B,128B}) for
# the cfg2 leaf kernel and for tools/fetch_calib.hip (reads exactly 4 GiB with
# the same LDS-DMA pattern): bytes = 32 x n32 + 64 x n64 + 128 x n128
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o /tmp/fetch_calib &&
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B \
  --output-format csv -d gpurun_out/pmc -o sizes -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline \
  --no-kernel-timing > gpurun_out/pmc/sizes.json &&
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B \
  --output-format csv -d gpurun_out/pmc -o calib -- /tmp/fetch_calib > gpurun_out/pmc/calib.txt
