# rocprofv3 kernel stats: records (fused and separate locate), aligned records, cfg2
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof5
for v in "fused:--config records --records-fused 1" "sep:--config records --records-fused 0" "cfg2:"; do
  tag=${v%%:*}; args=${v#*:}
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5 -o $tag -- python3 bench.py $args --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/prof5/$tag.json || exit 1
done
python3 - <<'PY'
import csv
for t in ["fused", "sep", "cfg2"]:
    print(t)
    for r in list(csv.DictReader(open(f"gpurun_out/prof5/{t}_kernel_stats.csv")))[:6]:
        print("  %-50s calls=%s avg_us=%.1f" % (r["Name"][:50], r["Calls"], float(r["AverageNs"])/1e3))
PY
