# A/B of the binned engine's env knobs on C2 (same box, 20 steps each)
set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in "KB_BIN_FILL_PCT=60" "KB_BIN_FILL_PCT=50" "KB_BIN_FILL_PCT=55" "KB_BIN_BIG_DIV=1" "KB_BIN_BIG_DIV=4" "KB_BIN_FILL_PCT=60"; do
  env $cfg timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/knob.json 2>/dev/null || exit 1
  echo "$cfg $(python -c "import json;d=json.load(open('gpurun_out/knob.json'));print(d['ms_per_step'],d['roofline']['kernel_ms'],d['phases_ms'])")" >> gpurun_out/knobs.txt
done
echo rc=$?
