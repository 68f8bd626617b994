# r04 g25: C3 with smaller context sub-bins (more of them ranked): sub-bin
# fill 40 % / 25 % of a table, extra-bin budget raised
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g25; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 2 --digest > $O/c3_base.json 2> $O/c3_base.err && \
KB_BIN_SUB_FILL_PCT=40 KB_BIN_SUB_EXTRA=240 timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 2 --digest > $O/c3_f40.json 2> $O/c3_f40.err && \
KB_BIN_SUB_FILL_PCT=25 KB_BIN_SUB_EXTRA=240 timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 2 --digest > $O/c3_f25.json 2> $O/c3_f25.err && \
KB_BIN_SUB_EXTRA=240 timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 2 --digest > $O/c3_x240.json 2> $O/c3_x240.err
echo rc=$?
