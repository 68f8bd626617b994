# parity of the binned engine first, then an A/B of an env knob on the C2 bench
# (and optionally a second workload): $1 = NAME, then values
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "binned" > gpurun_out/t_par.log 2>&1 || exit 1
name=$1; shift
for v in "$@"; do
  env $name=$v timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/ab_$v.log 2>&1 || exit 1
  env $name=$v timeout -k 10 200 python bench.py --steps 5 --warmup 2 --workload c2 --K 63 --read-len 250 --err-ppm 10000 --cpu-sample 0 > gpurun_out/ab63_$v.log 2>&1 || exit 1
done
echo rc=$?
