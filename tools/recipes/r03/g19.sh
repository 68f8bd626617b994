# round-3 evidence, part 1: C2 and the N-receiver emulations (kernel trace,
# FETCH/WRITE passes, one SQ pass each)
set -o pipefail
cd $GRAFT_REPO_ROOT
NOX="--no-capacity --no-host-input"
ZS2="--reads 2000000 --genome 10000000 --parts 2"
ZS8="--reads 8000000 --genome 40000000 --parts 8"
bash tools/gpu.sh ktrace r3_c2 $NOX --steps 20 --warmup 3 && \
bash tools/gpu.sh pmc r3_c2 $NOX --steps 5 --warmup 2 && \
bash tools/gpu.sh sq r3_c2 $NOX --steps 5 --warmup 2 && \
bash tools/gpu.sh ktrace r3_zs2 $NOX $ZS2 --steps 5 --warmup 2 && \
bash tools/gpu.sh pmc r3_zs2 $NOX $ZS2 --steps 3 --warmup 2 && \
bash tools/gpu.sh sq r3_zs2 $NOX $ZS2 --steps 3 --warmup 2 && \
bash tools/gpu.sh ktrace r3_zs8 $NOX $ZS8 --steps 3 --warmup 2 && \
bash tools/gpu.sh pmc r3_zs8 $NOX $ZS8 --steps 3 --warmup 2 && \
bash tools/gpu.sh sq r3_zs8 $NOX $ZS8 --steps 3 --warmup 2
echo rc=$?
