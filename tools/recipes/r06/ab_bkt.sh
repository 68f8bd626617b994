# r06 A/B: bucket_kernel workgroup size 512 (default) against 1024 and 256, C2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab_bkt; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 20 --warmup 3"
L=genome-assembly_amd/lib
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $NOX > $O/t512_$i.json 2>> $O/err.txt || exit 1
  for t in 1024 256; do
    KB_LIB_PATH=$L/bkt$t/libkbin.so timeout -k 10 300 python -u bench.py $NOX > $O/t${t}_$i.json 2>> $O/err.txt || exit 1
  done
done
echo done
