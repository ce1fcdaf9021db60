# records_verify: k_leaf_verify through the LDS-DMA segment stage (product) vs
# whole 128-byte lines into registers (NKV_VERIFY_LINES=1 at 5 / 4 waves per SIMD), same box, verified
set -o pipefail
bash tools/ab_tags.sh "--config records_verify" v5 v4 || exit 1
