#!/usr/bin/env bash
# build_ref.sh -- TEST INFRASTRUCTURE ONLY.
#
# Compiles the reference hot path (binning.c + zhash.c + llist.c, straight from
# /root/reference) together with our own ref_harness.c into
#   oracle/_ref/ref_k<K>_m<M>_c<C>
# The reference hard-codes KMER_SIZE/MMER_SIZE/ABUNDANCE_CUTOFF with plain
# #defines (binning.c:10-12), so a guarded copy of binning.c is produced in a
# private temp dir (deleted on exit) -- no reference source is ever written
# into the repository tree.  Only the binary lands in oracle/_ref/ (git-ignored).
#
# Usage: oracle/build_ref.sh K M [CUTOFF]      (no-op when /root/reference is absent)
set -euo pipefail
K=${1:?K}; M=${2:?M}; C=${3:-1}
REF=${KB_REFERENCE_DIR:-/root/reference}
HERE="$(cd "$(dirname "$0")" && pwd)"
OUT="$HERE/_ref"
BIN="$OUT/ref_k${K}_m${M}_c${C}"
if [ ! -f "$REF/binning.c" ]; then
  echo "reference not present at $REF; skipping" >&2
  exit 0
fi
mkdir -p "$OUT"
if [ -x "$BIN" ]; then exit 0; fi
TMP="$(mktemp -d)"
trap 'rm -rf "$TMP"' EXIT
sed -e 's/^#define MMER_SIZE \(.*\)$/#ifndef MMER_SIZE\n#define MMER_SIZE \1\n#endif/' \
    -e 's/^#define KMER_SIZE \(.*\)$/#ifndef KMER_SIZE\n#define KMER_SIZE \1\n#endif/' \
    -e 's/^#define ABUNDANCE_CUTOFF \(.*\)$/#ifndef ABUNDANCE_CUTOFF\n#define ABUNDANCE_CUTOFF \1\n#endif/' \
    "$REF/binning.c" > "$TMP/binning_guarded.c"
gcc -O2 -w -I"$REF" -DKMER_SIZE="$K" -DMMER_SIZE="$M" -DABUNDANCE_CUTOFF="$C" \
    -Dmain=binning_main -c "$TMP/binning_guarded.c" -o "$TMP/binning.o"
gcc -O2 -w -I"$REF" -c "$REF/zhash.c" -o "$TMP/zhash.o"
gcc -O2 -w -I"$REF" -c "$REF/llist.c" -o "$TMP/llist.o"
gcc -O2 -w -I"$REF" -c "$HERE/ref_harness.c" -o "$TMP/harness.o"
gcc -O2 "$TMP/binning.o" "$TMP/zhash.o" "$TMP/llist.o" "$TMP/harness.o" -o "$BIN"
echo "built $BIN"
