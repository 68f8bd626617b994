set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3i; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 20 --warmup 5"
for cfg in "base" "KB_BIN_LDSBAR=0" "KB_BIN_TS_ADAPT=0" "KB_BIN_SUB=0" "KB_BIN_SUB=2" "KB_BIN_SUB_FILL_PCT=80" "KB_BIN_FILL_LIGHT_PCT=60"; do
  tag=$(echo $cfg | tr '=' '_')
  if [ "$cfg" = base ]; then envs=""; else envs="$cfg"; fi
  env $envs timeout -k 10 120 python -u bench.py $NOX > $O/ab_$tag.json 2> $O/ab_$tag.err || exit 1
done
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 120 python -u bench.py --cpu-sample 0 --no-capacity --no-host-input --steps 3 --warmup 2 > $O/c2_prof.json 2> $O/c2_prof.err
echo rc=$?
