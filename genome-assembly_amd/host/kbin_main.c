/*
 * kbin_main.c -- command-line driver equivalent to the reference `main`
 * (binning.c:1147-1169) up to the hot-path boundary: read loop with fgets
 * chunking, process_read per chunk, prune_data, then the canonical dump of the
 * materialised two-level table (instead of the reference's unitig steps).
 *
 *   kbin_main <reads-file> <K> <M> <READ_LENGTH> <cutoff> <prune 0|1> [device]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/binning_gpu.h"

int main(int argc, char **argv)
{
    if (argc < 7) {
        fprintf(stderr, "usage: %s <reads> <K> <M> <READ_LENGTH> <cutoff> <prune 0|1> [device]\n",
                argv[0]);
        return 2;
    }
    const int K = atoi(argv[2]), M = atoi(argv[3]), rl = atoi(argv[4]);
    const int cutoff = atoi(argv[5]), prune = atoi(argv[6]);
    kbh_configure(K, M, cutoff, argc > 7 ? atoi(argv[7]) : 0);

    FILE *file = fopen(argv[1], "r");
    if (!file) {
        perror(argv[1]);
        return 2;
    }
    struct ZHashTable *hash_table = zcreate_hash_table();
    char *read = malloc((size_t)rl + 1);
    int read_id = 0;
    while (fgets(read, rl, file) != NULL) { /* binning.c:1158-1166 */
        int len = (int)strlen(read);
        read[--len] = '\0';
        process_read(hash_table, read, read_id++);
    }
    fclose(file);
    free(read);
    if (prune)
        prune_data(hash_table);
    else
        kbh_finish_unpruned(hash_table);
    kbh_dump_table(hash_table, stdout);
    return 0;
}
