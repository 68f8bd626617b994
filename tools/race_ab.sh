#!/bin/bash
# Evidence build for VERDICT r04 item 1: the diagnostic library (KB_BIN_ABL,
# with the KB_DIAG_SKEW late wave) with bin_body's partition-stack depth back in
# ONE word (round 4's code), into genome-assembly_amd/lib/race_old/.  Under
# KB_DIAG_SKEW it must fail (tests/test_gpu_race.py against this build), while
# lib/abl (the fix: one word per partition parity) stays bit-exact.
set -euo pipefail
REPO=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
trap 'rm -rf "$T"' EXIT
mkdir -p "$T/genome-assembly_amd" "$T/include"
cp -r "$REPO/genome-assembly_amd/csrc" "$T/genome-assembly_amd/"
cp "$REPO"/include/*.h "$T/include/"
sed -i 's/const uint32_t pq = p0 & 1u;/const uint32_t pq = 0u;  \/\/ (race_ab.sh: round 4 single word)/' \
    "$T/genome-assembly_amd/csrc/kbin_bins.hip"
grep -q "pq = 0u;  // (race_ab.sh" "$T/genome-assembly_amd/csrc/kbin_bins.hip"
make -s -j8 -C "$T/genome-assembly_amd/csrc" OUT="$REPO/genome-assembly_amd/lib/race_old" \
    HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -DKB_BIN_ABL" 2>&1 |
    grep -v "warning: loop not unrolled\|^ *[0-9]* |\|^ *|\|warnings generated" || true
ls -la "$REPO/genome-assembly_amd/lib/race_old/libkbin.so"
