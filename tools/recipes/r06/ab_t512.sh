# r06 A/B: bin_kernel with 512-thread workgroups and 4096-slot tables (two
# workgroups per CU: one's barrier waits covered by the other's work) against
# the default 1024 threads / 8192 slots, C2 bench alternating on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab_t512; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 20 --warmup 3"
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py $NOX > $O/a$i.json 2>> $O/err.txt || exit 1
  KB_LIB_PATH=genome-assembly_amd/lib/t512/libkbin.so KB_BIN_TS_LOG2=12 timeout -k 10 300 python -u bench.py $NOX > $O/b$i.json 2>> $O/err.txt || exit 1
done
echo done
