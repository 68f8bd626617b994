# C2 and the N-rank receiver emulation (bench JSON lines only)
set -o pipefail
cd $GRAFT_REPO_ROOT
for w in "1000000 1 10" "2000000 2 3" "8000000 8 2"; do
  set -- $w
  timeout -k 10 300 python bench.py --reads $1 --parts $2 --steps $3 --warmup 1 --cpu-sample 0 > gpurun_out/e_$2.log 2>&1 || exit 1
done
echo rc=$?
