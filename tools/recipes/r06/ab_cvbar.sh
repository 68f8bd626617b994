# r06 A/B: the received-record conversion's trip barriers LDS-only (no wait
# for the trip's record stores) against the round's tree: C3 (digest) and the
# routed one-rank C2 line, alternating on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab_cvbar; mkdir -p $O
L=genome-assembly_amd/lib
for i in 1 2; do
  KB_LIB_PATH=$L/base/libkbin.so timeout -k 10 400 python -u bench.py --workload c3 --steps 3 --warmup 1 --cpu-sample 0 --digest > $O/c3_base$i.json 2>> $O/err.txt || exit 1
  timeout -k 10 400 python -u bench.py --workload c3 --steps 3 --warmup 1 --cpu-sample 0 --digest > $O/c3_new$i.json 2>> $O/err.txt || exit 1
  KB_LIB_PATH=$L/base/libkbin.so timeout -k 10 300 python -u bench.py --routed --steps 20 --warmup 3 --cpu-sample 0 --no-host-input --no-capacity > $O/rt_base$i.json 2>> $O/err.txt || exit 1
  timeout -k 10 300 python -u bench.py --routed --steps 20 --warmup 3 --cpu-sample 0 --no-host-input --no-capacity > $O/rt_new$i.json 2>> $O/err.txt || exit 1
done
echo done
