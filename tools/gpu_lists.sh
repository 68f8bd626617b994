# lists kernel (windowed staging): full GPU suite, then C2 and the N-rank emulation with a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > gpurun_out/t_all.log 2>&1 || exit 1
for w in "1000000 1" "2000000 2" "8000000 8"; do
  set -- $w
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ls_$2 -o kt -- python3 bench.py --reads $1 --parts $2 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/ls_$2.log 2>&1 || exit 1
done
echo rc=$?
