# records: segment stage through LDS-DMA (product) vs whole 128-byte lines
# straight into registers (experiment libraries: NKV_SHIFT_LINES=1 at 5 / 6
# waves per SIMD), same box, verified against the oracle
set -o pipefail
bash tools/ab_tags.sh "--config records" lines5 lines6 || exit 1
