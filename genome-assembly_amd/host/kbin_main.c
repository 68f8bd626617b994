/*
 * kbin_main.c -- command-line driver equivalent to the reference `main`
 * (binning.c:1147-1169) up to the hot-path boundary: read loop with fgets
 * chunking, process_read per chunk, prune_data, then the canonical dump of the
 * materialised two-level table (instead of the reference's unitig steps).
 *
 *   kbin_main <reads-file> <K> <M> <READ_LENGTH> <cutoff> <prune 0|1> [device] [--gpus N|d0,d1,..] [--unitigs]
 *
 * --unitigs: instead of the dump, the rest of the reference's main
 * (binning.c:1171-1180): expand_read_id_list, find_kmer_extensions forward
 * and backward (the exact replay, unitig.c), print_kmers -- the reference
 * program's own stdout.
 *
 * --gpus: bin on several GPUs through one multi-GPU group (mmer-sharded,
 * records exchanged over RCCL; kbh_configure_gpus); the dump is identical.
 *
 * KBH_TIMING=1 in the environment: one JSON line of wall-clock phases on
 * stderr (read loop = fgets + process_read; then prune_data's phases);
 * KBH_NODUMP=1 skips the dump (timing runs).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/binning_gpu.h"

int main(int argc, char **argv)
{
    /* (--gpus anywhere after the positional arguments) */
    int gpus[64], ng = 0, pos = argc, unitigs = 0;
    for (int i = 1; i < argc; i++)
        if (!strcmp(argv[i], "--unitigs")) {
            unitigs = 1;
            if (pos == argc) pos = i;
        } else if (!strcmp(argv[i], "--gpus")) {
            if (i + 1 >= argc) return 2;
            const char *q = argv[i + 1];
            if (!strchr(q, ',')) {
                ng = atoi(q);
                for (int g = 0; g < ng && g < 64; g++) gpus[g] = g;
            } else {
                for (; q && ng < 64; q = strchr(q, ',') ? strchr(q, ',') + 1 : NULL) gpus[ng++] = atoi(q);
            }
            if (pos == argc) pos = i;
        }
    if (pos < 7) {
        fprintf(stderr, "usage: %s <reads> <K> <M> <READ_LENGTH> <cutoff> <prune 0|1> [device] [--gpus N|d0,d1,..]\n",
                argv[0]);
        return 2;
    }
    const int K = atoi(argv[2]), M = atoi(argv[3]), rl = atoi(argv[4]);
    const int cutoff = atoi(argv[5]), prune = atoi(argv[6]);
    kbh_configure(K, M, cutoff, pos > 7 ? atoi(argv[7]) : 0);
    if (ng > 1 && kbh_configure_gpus(ng, gpus) != 0) {
        fprintf(stderr, "bad --gpus\n");
        return 2;
    }

    FILE *file = fopen(argv[1], "r");
    if (!file) {
        perror(argv[1]);
        return 2;
    }
    const char *tenv = getenv("KBH_TIMING"), *denv = getenv("KBH_NODUMP");
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    struct ZHashTable *hash_table = zcreate_hash_table();
    char *read = malloc((size_t)rl + 1);
    int read_id = 0;
    long long kmers = 0;
    while (fgets(read, rl, file) != NULL) { /* binning.c:1158-1166 */
        int len = (int)strlen(read);
        read[--len] = '\0';
        if (len >= K) kmers += len - K + 1;
        process_read(hash_table, read, read_id++);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    fclose(file);
    free(read);
    if (prune)
        prune_data(hash_table);
    else
        kbh_finish_unpruned(hash_table);
    if (tenv && *tenv == '1') {
        kbh_times t;
        kbh_last_times(&t);
        const double loop = (t1.tv_sec - t0.tv_sec) * 1e3 + (t1.tv_nsec - t0.tv_nsec) * 1e-6;
        fprintf(stderr,
                "{\"reads\": %d, \"kmers\": %lld, \"read_loop_ms\": %.3f, \"finalize_ms\": %.3f, "
                "\"export_ms\": %.3f, \"materialise_ms\": %.3f, \"prune_ms\": %.3f, \"total_ms\": %.3f, "
                "\"entries\": %llu, \"ids\": %llu, \"nodes\": %llu, \"materialise_order_ms\": %.3f, "
                "\"materialise_group_ms\": %.3f, \"materialise_fill_ms\": %.3f, \"release_ms\": %.3f}\n",
                read_id, kmers, loop, t.finalize_ms, t.export_ms, t.materialise_ms, t.prune_ms, loop + t.total_ms,
                (unsigned long long)t.entries, (unsigned long long)t.ids, (unsigned long long)t.nodes, t.order_ms,
                t.group_ms, t.fill_ms, t.release_ms);
    }
    if (unitigs) { /* binning.c:1171-1180 */
        struct timespec u0, u1, u2;
        clock_gettime(CLOCK_MONOTONIC, &u0);
        expand_read_id_list(hash_table);
        clock_gettime(CLOCK_MONOTONIC, &u1);
        find_kmer_extensions(hash_table, true);
        find_kmer_extensions(hash_table, false);
        clock_gettime(CLOCK_MONOTONIC, &u2);
        if (tenv && *tenv == '1') {
            kbh_unitig_stats us;
            kbh_unitig_stats_get(&us);
            fprintf(stderr,
                    "{\"expand_ms\": %.3f, \"unitig_ms\": %.3f, \"unitig_index_ms\": %.3f, \"unitigs\": %llu, "
                    "\"merges\": %llu, \"u1_events\": %llu}\n",
                    (u1.tv_sec - u0.tv_sec) * 1e3 + (u1.tv_nsec - u0.tv_nsec) * 1e-6,
                    (u2.tv_sec - u1.tv_sec) * 1e3 + (u2.tv_nsec - u1.tv_nsec) * 1e-6, us.index_ms,
                    (unsigned long long)us.unitigs, (unsigned long long)us.merges,
                    (unsigned long long)us.u1_events);
        }
        if (!(denv && *denv == '1')) kbh_print_kmers(hash_table, stdout);
        return 0;
    }
    if (!(denv && *denv == '1')) kbh_dump_table(hash_table, stdout);
    return 0;
}
