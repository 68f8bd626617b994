# r04 g29: capacity knob sweep at the final build -- C5 share: flat depth 4
# (default 3), extra-bin budget 240; C4 share: light-bin table fill 40 / 60 %
# (default 50)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g29; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 400 python -u bench.py $NOX --workload c5 --steps 2 --warmup 2 > $O/c5_base.json 2> $O/c5_base.err && \
KB_BIN_FLAT_L=4 timeout -k 10 400 python -u bench.py $NOX --workload c5 --steps 2 --warmup 2 --digest > $O/c5_flat4.json 2> $O/c5_flat4.err && \
KB_BIN_SUB_EXTRA=240 timeout -k 10 400 python -u bench.py $NOX --workload c5 --steps 2 --warmup 2 --digest > $O/c5_x240.json 2> $O/c5_x240.err && \
timeout -k 10 400 python -u bench.py $NOX --workload c4 --steps 2 --warmup 1 > $O/c4_base.json 2> $O/c4_base.err && \
KB_BIN_FILL_LIGHT_PCT=40 timeout -k 10 400 python -u bench.py $NOX --workload c4 --steps 2 --warmup 1 --digest > $O/c4_fl40.json 2> $O/c4_fl40.err && \
KB_BIN_FILL_LIGHT_PCT=60 timeout -k 10 400 python -u bench.py $NOX --workload c4 --steps 2 --warmup 1 --digest > $O/c4_fl60.json 2> $O/c4_fl60.err
echo rc=$?
