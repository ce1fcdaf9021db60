# Round 4: cfg2's leaf-kernel HBM traffic on the round's build (four --pmc
# passes, tools/pmc_config.sh), summarised by tools/pmc_traffic_cfg.py into
# profiles/pmc_traffic_cfg2_r04.json (the bench line's roofline.traffic).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/pmc_config.sh cfg2_r04 || exit 1
python tools/pmc_traffic_cfg.py cfg2_r04 "void nkv::k_leaf<0, 4>" 4294967296 1048576 || exit 1
cp profiles/pmc_traffic_cfg2_r04.json gpurun_out/ 2>/dev/null || true
