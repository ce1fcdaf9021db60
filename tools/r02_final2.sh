# Final state after the register line loads: GPU suite + smoke, the default
# bench line (verified), RCCL world-1 line, rocprofv3 kernel summaries of every
# config, and the PMC traffic of the records / records_verify leaf kernels
set -o pipefail
export TMPDIR=/tmp
bash tools/r02_final.sh || exit 1
bash tools/pmc_config.sh records_lines --config records || exit 1
bash tools/pmc_config.sh records_verify_lines --config records_verify || exit 1
