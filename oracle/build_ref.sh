#!/usr/bin/env bash
# build_ref.sh -- TEST INFRASTRUCTURE ONLY.
#
# Compiles the reference (binning.c + zhash.c + llist.c, straight from
# /root/reference) into oracle/_ref/ (git-ignored).  The reference hard-codes
# KMER_SIZE/MMER_SIZE/ABUNDANCE_CUTOFF with plain #defines (binning.c:10-12),
# so a guarded copy of binning.c is produced in a private temp dir that is
# deleted on exit -- no reference source is ever written into the repository.
#
#   build_ref.sh K M [C]          ref_k<K>_m<M>_c<C>: reference hot path + our
#                                 ref_harness.c main -> canonical post-prune dump
#   build_ref.sh g K M [C]        refg_k<K>_m<M>_c<C>: the same harness, the
#                                 reference compiled with its makefile's flags
#                                 (makefile:2: -g, no -O) -- BASELINE.md's
#                                 "as shipped" CPU row
#   build_ref.sh full K M [C]     full_k<K>_m<M>_c<C>: the reference program as
#                                 shipped (its own main: bin, prune, expand,
#                                 unitig extension, print_kmers)
#   build_ref.sh dropin K M [C]   dropin_k<K>_m<M>_c<C>: the SAME reference
#                                 program, but its process_read/prune_data/
#                                 expand_read_id_list are
#                                 weakened and the GPU shim's strong definitions
#                                 (genome-assembly_amd/host/binning_gpu.c over
#                                 libkbin.so) win at link time -- the drop-in
#                                 integration described in INTEGRATION.md;
#                                 find_kmer_extensions is replaced as well
#                                 (genome-assembly_amd/host/unitig.c)
#   build_ref.sh dropinw K M [C]  dropinw_k<K>_m<M>_c<C>: the drop-in with the
#                                 reference's OWN find_kmer_extensions kept
#                                 (the unitig walk's timing baseline)
#   build_ref.sh unitig K M [C]   unitig_k<K>_m<M>_c<C>: the reference program
#                                 as shipped (its own process_read, prune,
#                                 expansion, print_kmers) with ONLY
#                                 find_kmer_extensions replaced by unitig.c --
#                                 CPU only: the unitig replay's parity test on
#                                 the reference's own tables
# No-op when /root/reference is absent (e.g. on the GPU box).
set -euo pipefail
MODE=harness
case "${1:-}" in full|dropin|dropinw|unitig|g) MODE=$1; shift ;; esac
K=${1:?K}; M=${2:?M}; C=${3:-1}
REF=${KB_REFERENCE_DIR:-/root/reference}
HERE="$(cd "$(dirname "$0")" && pwd)"
REPO="$(cd "$HERE/.." && pwd)"
OUT="$HERE/_ref"
RL=${KB_REF_READ_LENGTH:+_rl$KB_REF_READ_LENGTH}
case $MODE in
  harness) BIN="$OUT/ref_k${K}_m${M}_c${C}$RL" ;;
  g)       BIN="$OUT/refg_k${K}_m${M}_c${C}$RL" ;;
  full)    BIN="$OUT/full_k${K}_m${M}_c${C}$RL" ;;
  dropin)  BIN="$OUT/dropin_k${K}_m${M}_c${C}$RL" ;;
  dropinw) BIN="$OUT/dropinw_k${K}_m${M}_c${C}$RL" ;;
  unitig)  BIN="$OUT/unitig_k${K}_m${M}_c${C}$RL" ;;
esac
if [ ! -f "$REF/binning.c" ]; then
  echo "reference not present at $REF; skipping" >&2
  exit 0
fi
mkdir -p "$OUT"
# (a drop-in binary links the shim: rebuilt whenever the shim or the engine
# library is newer than it)
if [ -x "$BIN" ]; then
  if [ "$MODE" != dropin ] && [ "$MODE" != dropinw ] && [ "$MODE" != unitig ]; then exit 0; fi
  if [ ! "$REPO/genome-assembly_amd/host/binning_gpu.c" -nt "$BIN" ] && \
     [ ! "$REPO/genome-assembly_amd/host/unitig.c" -nt "$BIN" ] && \
     [ ! "$REPO/genome-assembly_amd/lib/libkbin.so" -nt "$BIN" ]; then exit 0; fi
fi
TMP="$(mktemp -d)"
trap 'rm -rf "$TMP"' EXIT
sed -e 's/^#define MMER_SIZE \(.*\)$/#ifndef MMER_SIZE\n#define MMER_SIZE \1\n#endif/' \
    -e 's/^#define KMER_SIZE \(.*\)$/#ifndef KMER_SIZE\n#define KMER_SIZE \1\n#endif/' \
    -e 's/^#define ABUNDANCE_CUTOFF \(.*\)$/#ifndef ABUNDANCE_CUTOFF\n#define ABUNDANCE_CUTOFF \1\n#endif/' \
    -e 's/^#define READ_LENGTH \(.*\)$/#ifndef READ_LENGTH\n#define READ_LENGTH \1\n#endif/' \
    "$REF/binning.c" > "$TMP/binning_guarded.c"
DEFS="-DKMER_SIZE=$K -DMMER_SIZE=$M -DABUNDANCE_CUTOFF=$C"
# KB_REF_READ_LENGTH=<n>: the fgets chunk size (binning.c:13, 101 as shipped);
# the binary name then ends in _rl<n>
if [ -n "${KB_REF_READ_LENGTH:-}" ]; then DEFS="$DEFS -DREAD_LENGTH=$KB_REF_READ_LENGTH"; fi
case $MODE in
  harness)
    gcc -O2 -w -I"$REF" $DEFS -Dmain=binning_main -c "$TMP/binning_guarded.c" -o "$TMP/binning.o"
    gcc -O2 -w -I"$REF" -c "$REF/zhash.c" -o "$TMP/zhash.o"
    gcc -O2 -w -I"$REF" -c "$REF/llist.c" -o "$TMP/llist.o"
    gcc -O2 -w -I"$REF" $DEFS -c "$HERE/ref_harness.c" -o "$TMP/harness.o"
    gcc -O2 "$TMP/binning.o" "$TMP/zhash.o" "$TMP/llist.o" "$TMP/harness.o" -o "$BIN"
    ;;
  g)
    gcc -g -w -I"$REF" $DEFS -Dmain=binning_main -c "$TMP/binning_guarded.c" -o "$TMP/binning.o"
    gcc -g -w -I"$REF" -c "$REF/zhash.c" -o "$TMP/zhash.o"
    gcc -g -w -I"$REF" -c "$REF/llist.c" -o "$TMP/llist.o"
    gcc -O2 -w -I"$REF" $DEFS -c "$HERE/ref_harness.c" -o "$TMP/harness.o"
    gcc "$TMP/binning.o" "$TMP/zhash.o" "$TMP/llist.o" "$TMP/harness.o" -o "$BIN"
    ;;
  unitig)
    gcc -g -O0 -fno-inline -w -I"$REF" $DEFS -c "$TMP/binning_guarded.c" -o "$TMP/binning.o"
    gcc -g -O0 -w -I"$REF" -c "$REF/zhash.c" -o "$TMP/zhash.o"
    gcc -g -O0 -w -I"$REF" -c "$REF/llist.c" -o "$TMP/llist.o"
    objcopy --weaken-symbol=find_kmer_extensions "$TMP/binning.o"
    gcc -O2 -w $DEFS -c "$REPO/genome-assembly_amd/host/unitig.c" -o "$TMP/unitig.o"
    gcc "$TMP/binning.o" "$TMP/zhash.o" "$TMP/llist.o" "$TMP/unitig.o" -o "$BIN"
    ;;
  full|dropin|dropinw)
    # makefile:2-5 flags (-g, no -O): calls stay relocations against the
    # global symbols, so a strong definition elsewhere can replace them
    gcc -g -O0 -fno-inline -w -I"$REF" $DEFS -c "$TMP/binning_guarded.c" -o "$TMP/binning.o"
    gcc -g -O0 -w -I"$REF" -c "$REF/zhash.c" -o "$TMP/zhash.o"
    gcc -g -O0 -w -I"$REF" -c "$REF/llist.c" -o "$TMP/llist.o"
    if [ "$MODE" = full ]; then
      gcc "$TMP/binning.o" "$TMP/zhash.o" "$TMP/llist.o" -o "$BIN"
    else
      LIB="$REPO/genome-assembly_amd/lib"
      [ -f "$LIB/libkbin.so" ] || { echo "build libkbin.so first" >&2; exit 1; }
      objcopy --weaken-symbol=process_read --weaken-symbol=prune_data --weaken-symbol=expand_read_id_list "$TMP/binning.o"
      # the shim includes our kb_zhash.h (same layout as zhash.h/llist.h); its
      # container calls resolve to the reference's zhash.o / llist.o
      gcc -O2 -w -pthread $DEFS -c "$REPO/genome-assembly_amd/host/binning_gpu.c" -o "$TMP/shim.o"
      OBJS="$TMP/shim.o"
      if [ "$MODE" = dropin ]; then
        objcopy --weaken-symbol=find_kmer_extensions "$TMP/binning.o"
        gcc -O2 -w $DEFS -c "$REPO/genome-assembly_amd/host/unitig.c" -o "$TMP/unitig.o"
        OBJS="$OBJS $TMP/unitig.o"
      fi
      gcc -pthread "$TMP/binning.o" "$TMP/zhash.o" "$TMP/llist.o" $OBJS -L"$LIB" -lkbin \
          -Wl,-rpath,"\$ORIGIN/../../genome-assembly_amd/lib" -o "$BIN"
    fi
    ;;
esac
echo "built $BIN"
