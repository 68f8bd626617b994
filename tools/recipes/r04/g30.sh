# r04 g30: light-bin table fill 60 % (default 50) at C2 (alternating), C3,
# and 70 % at the C4 share
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g30; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $NOX --steps 30 --warmup 5 > $O/c2_fl50_$i.json 2> $O/c2_fl50_$i.err || exit 1
  KB_BIN_FILL_LIGHT_PCT=60 timeout -k 10 200 python -u bench.py $NOX --steps 30 --warmup 5 --digest > $O/c2_fl60_$i.json 2> $O/c2_fl60_$i.err || exit 1
done
KB_BIN_FILL_LIGHT_PCT=60 timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 2 --digest > $O/c3_fl60.json 2> $O/c3_fl60.err || exit 1
timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 2 > $O/c3_fl50.json 2> $O/c3_fl50.err || exit 1
KB_BIN_FILL_LIGHT_PCT=70 timeout -k 10 400 python -u bench.py $NOX --workload c4 --steps 2 --warmup 1 --digest > $O/c4_fl70.json 2> $O/c4_fl70.err || exit 1
echo rc=$?
