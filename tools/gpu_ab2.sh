# A/B of an env knob on the binned bench: $1 = NAME, then values
set -o pipefail
cd $GRAFT_REPO_ROOT
name=$1; shift
for v in "$@"; do
  env $name=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/ab_$v.log 2>&1 || exit 1
done
echo rc=$?
