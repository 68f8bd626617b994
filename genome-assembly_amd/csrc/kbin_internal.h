// kbin_internal.h -- shared declarations between the HIP kernels
// (kbin_kernels.hip) and the host C-ABI (kbin_api.hip).  Not installed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kb {

// Slot layouts of the open-addressed (mmer, kmer) table.  EMPTY slot = all 0.
//  KW=1 (K <= 31):  w0 = kmer_code + 1 (claim word, CAS), w1 = tag | cnt << 32
//  KW=2 (K <= 63):  w0 = (code >> 63) + 1 (claim), w1 = (code & 2^63-1) | PUB,
//                   w2 = tag | cnt << 32, w3 = pad
// tag = mmer_code + 1 (non-zero marks it published).  Every non-claim word
// carries its own "published" marker, so readers never need cross-word
// ordering ("Table protocol").
constexpr uint64_t PUB = 1ull << 63;
constexpr uint32_t NONE = 0xFFFFFFFFu;

// status bits written by kernels
constexpr uint32_t ST_TABLE_FULL = 1u;   // distinct keys exceeded the load limit
constexpr uint32_t ST_PROBE_LIMIT = 2u;  // a probe sequence exceeded max_probe
constexpr uint32_t ST_ALPHABET = 4u;     // byte outside ACGT in packed input

struct ScanArgs {
    const uint64_t* words;     // packed reads, RW words per read
    const uint32_t* lens;      // bases per read
    const uint64_t* kmer_base; // [n_reads+1] first occurrence index of read r
    uint64_t n_reads;
    uint64_t* table;           // slots * SW words
    uint64_t mask;             // slots - 1
    uint32_t* occ_slot;        // [n_kmers of batch] slot of each occurrence
    uint32_t* n_distinct;      // global distinct-key counter
    uint32_t* status;
    uint32_t max_distinct;
    uint32_t max_probe;
    int RW;                    // words per read
    int K, M;
};

struct PlaceArgs {
    const uint32_t* occ_slot;
    const uint64_t* kmer_base; // [n_reads+1]
    uint64_t n_reads;
    uint64_t n_occ;
    const uint32_t* slot_entry;
    const uint64_t* e_off;
    uint32_t* cursor;
    uint32_t* ids_ord;         // ordinals placed per entry
    uint32_t ord_base;
};

// launch helpers implemented in kbin_kernels.hip (all asynchronous on `s`)
hipError_t launch_pack(const uint8_t* d_bases, const uint64_t* d_off, uint64_t n_reads,
                       int RW, uint64_t* d_words, uint32_t* d_lens, uint32_t* d_status,
                       hipStream_t s);
hipError_t launch_kmer_base(const uint32_t* d_lens, uint64_t n_reads, int K,
                            uint64_t* d_kmer_base, uint64_t* d_scratch, uint64_t scratch_n,
                            hipStream_t s);
uint64_t kmer_base_scratch_elems(uint64_t n_reads);
hipError_t launch_scan_insert(const ScanArgs& a, int KW, hipStream_t s);
hipError_t launch_compact(const uint64_t* table, uint64_t slots, int KW, int K,
                          uint32_t cutoff_keep_gt, uint32_t* slot_entry,
                          uint32_t* e_mmer, uint64_t* e_hi, uint64_t* e_lo,
                          uint32_t* e_cnt, uint64_t* e_off,
                          uint64_t* scratch, uint64_t scratch_n,
                          uint64_t* d_totals, hipStream_t s);
uint64_t compact_scratch_elems(uint64_t slots);
hipError_t launch_place(const PlaceArgs& a, hipStream_t s);
hipError_t launch_sort(const uint64_t* e_off, const uint32_t* e_cnt, uint64_t n_entries,
                       uint32_t* ids_ord, uint32_t* ids_tmp, const int32_t* read_ids,
                       int32_t* ids_out, uint32_t* lists, uint32_t* list_counts,
                       hipStream_t s);
hipError_t launch_fill_ids(int32_t* d_ids, uint64_t n, int32_t first, hipStream_t s);
hipError_t launch_generate(uint64_t* d_words, uint32_t* d_lens, uint64_t n_reads,
                           uint32_t read_len, uint64_t genome_len, uint32_t err_ppm,
                           uint64_t seed, hipStream_t s);
hipError_t launch_unpack(const uint64_t* d_words, const uint32_t* d_lens, uint64_t n_reads,
                         int RW, const uint64_t* d_off, uint8_t* d_bases, hipStream_t s);

}  // namespace kb
