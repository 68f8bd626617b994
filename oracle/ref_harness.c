/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * A `main` that drives the *reference* binning.c (compiled from
 * /root/reference with its `main` renamed to `binning_main`, see build_ref.sh)
 * up to the hot-path boundary and prints the canonical post-prune dump
 * (SURVEY.md §8(c)):
 *
 *     mmer \t kmer \t count \t id1,id2,...\n      (ids in list order)
 *
 * The read loop restates binning.c:1150-1166 exactly (fgets with a buffer of
 * READ_LENGTH bytes, unconditional strip of the last byte, read_id++ per
 * chunk), except that READ_LENGTH is a run-time argument here because the
 * harness owns the buffer.  K, M and the cutoff stay compile-time in the
 * reference, so build_ref.sh builds one binary per (K, M, cutoff).
 *
 * Usage:  ref_kK_mM_cC <reads-file> <READ_LENGTH> <prune 0|1> [time]
 * Output is unsorted (hash-bucket order); callers sort bytewise.
 * With "time" the dump is skipped and one line goes to stdout instead:
 *     kmers=<n> bin_s=<fgets+process_read loop> prune_s=<prune_data>
 * (the timed region of BASELINE.md; bench.py's cpu_baseline "reference" leg).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdbool.h>
#include <time.h>

#include "zhash.h"
#include "llist.h"

/* reference entry points (binning.c) */
struct ZHashTable *process_read(struct ZHashTable *hash_table, char *read, int read_id);
struct ZHashTable *prune_data(struct ZHashTable *hash_table);
void *iterate_level_one_hash(struct ZHashTable *hash_table, bool indirection, bool remove_current);
void *iterate_level_two_hash(struct ZHashTable *hash_table, bool indirection, bool remove_current);

int main(int argc, char **argv)
{
    if (argc < 4) {
        fprintf(stderr, "usage: %s <reads-file> <READ_LENGTH> <prune 0|1>\n", argv[0]);
        return 2;
    }
    FILE *file = fopen(argv[1], "r");
    if (!file) { perror(argv[1]); return 2; }
    int rl = atoi(argv[2]);
    int do_prune = atoi(argv[3]);
    int timing = argc > 4 && strcmp(argv[4], "time") == 0;
    struct timespec t0, t1, t2;
    long long kmers = 0;
    char *read = malloc((size_t)rl + 1);
    struct ZHashTable *hash_table = zcreate_hash_table();
    int read_id = 0;

    clock_gettime(CLOCK_MONOTONIC, &t0);
    /* binning.c:1158-1166 */
    while (fgets(read, rl, file) != NULL) {
        int len = strlen(read);
        read[--len] = '\0';
        if (len >= KMER_SIZE) kmers += len - KMER_SIZE + 1;
        process_read(hash_table, read, read_id++);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    fclose(file);

    if (do_prune)
        prune_data(hash_table); /* binning.c:1169 */
    clock_gettime(CLOCK_MONOTONIC, &t2);
    if (timing) {
        printf("kmers=%lld bin_s=%.6f prune_s=%.6f\n", kmers,
               (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec),
               (t2.tv_sec - t1.tv_sec) + 1e-9 * (t2.tv_nsec - t1.tv_nsec));
        free(read);
        return 0;
    }

    struct ZHashEntry *me, *ke;
    while ((me = iterate_level_one_hash(hash_table, false, false)) != NULL) {
        struct ZHashTable *kt = me->val;
        while ((ke = iterate_level_two_hash(kt, false, false)) != NULL) {
            ll_node *n = ke->val;
            int cnt = 0;
            for (ll_node *t = n; t; t = t->next) cnt++;
            printf("%s\t%s\t%d\t", me->key, ke->key, cnt);
            for (ll_node *t = n; t; t = t->next)
                printf(t->next ? "%d," : "%d", t->read_id);
            putchar('\n');
        }
    }
    free(read);
    return 0;
}
