# round-3 evidence, part 2: the capacity configurations (C3 = the bench's
# capacity leg, C4 and C5 per-GPU shares): kernel trace, FETCH/WRITE passes
set -o pipefail
cd $GRAFT_REPO_ROOT
NOX="--no-capacity --no-host-input --steps 1 --warmup 1"
bash tools/gpu.sh ktrace r3_c3 $NOX --workload c3 && \
bash tools/gpu.sh pmc r3_c3 $NOX --workload c3 && \
bash tools/gpu.sh ktrace r3_c4 $NOX --workload c4 && \
bash tools/gpu.sh pmc r3_c4 $NOX --workload c4 && \
bash tools/gpu.sh ktrace r3_c5 $NOX --workload c5 && \
bash tools/gpu.sh pmc r3_c5 $NOX --workload c5
echo rc=$?
