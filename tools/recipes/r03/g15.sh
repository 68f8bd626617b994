set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3n; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 2 --warmup 1 --workload c5"
for ex in 48 120; do for P in 4 8; do
  KB_BIN_SUB_EXTRA=$ex timeout -k 10 200 python -u bench.py $NOX --parts $P > $O/c5_e${ex}_p$P.json 2> $O/c5_e${ex}_p$P.err || exit 1
done; done

timeout -k 10 100 python -u tools/cold.py --workload c2 --steps 3 > $O/cold_c2.txt 2>&1 || exit 1
timeout -k 10 100 python -u tools/cold.py --workload c2 --steps 3 --prewarm 2000 > $O/cold_c2_pw.txt 2>&1 || exit 1
KB_DEBUG=1 timeout -k 10 100 python -u tools/cold.py --workload c2 --steps 2 --prewarm 2000 > $O/cold_c2_pw_dbg.txt 2>&1 || exit 1
echo rc=$?
