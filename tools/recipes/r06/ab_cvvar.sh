# r06 A/B: the received-record conversion's trip shape (KB_CONVERT_VAR):
# 0 = 8 records x 256 lanes (138 VGPRs, 3 waves/SIMD), 1 = 4 x 512 (70, 7),
# 2 = 4 x 256 (72, 7), 3 = 8 x 512 (124, 4); C3 digest-checked and the
# routed one-rank C2 line, alternating on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab_cvvar; mkdir -p $O
for i in 1 2; do
  for v in 0 1 2 3; do
    KB_CONVERT_VAR=$v timeout -k 10 400 python -u bench.py --workload c3 --steps 3 --warmup 1 --cpu-sample 0 --digest > $O/c3_v${v}_$i.json 2>> $O/err.txt || exit 1
  done
  for v in 0 1 2 3; do
    KB_CONVERT_VAR=$v timeout -k 10 300 python -u bench.py --routed --steps 20 --warmup 3 --cpu-sample 0 --no-host-input --no-capacity > $O/rt_v${v}_$i.json 2>> $O/err.txt || exit 1
  done
done
echo done
