# r06: the routed C4 leg at 1/1, 1/2, 1/4 of a rank's reads (KB_DEBUG:
# records per received pass, the largest bucket) -- where the receiver's
# bucket blows up.  A Python exception (rc 1) goes on; a crash, abort or
# time limit ends the script
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/legs4; mkdir -p $O
for s in 1 2 4; do
  KB_DEBUG=1 KB_CAPACITY_SCALE=$s timeout -k 10 300 python -u bench.py --routed --multi-legs --steps 1 --warmup 0 --cpu-sample 0 --no-host-input > $O/legs_s$s.json 2> $O/legs_s$s.err
  rc=$?; echo "scale $s rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
echo done
