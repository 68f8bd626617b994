/* host_surface_check.c -- CPU check of the reference calling surface that
 * libkbin_host exports besides process_read / prune_data (VERDICT r04 item
 * 7): getbp / getval / getscore (binning.c:69-124) and prune_kmers
 * (binning.c:1085-1123).  Links ONLY libkbin_host + libkbin, like a standalone
 * C host; touches no GPU.
 *
 * Prints "score <string> <getscore>" lines for the pytest to compare with its
 * own base-4 values, then checks prune_kmers on tables built by zhash_set:
 * survivors keep their bucket and relative chain order, the table is not
 * resized, entry_count drops by the pruned keys, and an all-pruned table
 * comes back NULL.  Exit status 0 and a final "ok" line on success. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/binning_gpu.h"
#include "../../include/kb_zhash.h"

#define CHECK(c)                                                      \
    do {                                                              \
        if (!(c)) {                                                   \
            fprintf(stderr, "check failed at line %d: %s\n", __LINE__, #c); \
            return 1;                                                 \
        }                                                             \
    } while (0)

static uint64_t rng = 88172645463325252ull;
static uint64_t next(void)
{
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng;
}

typedef struct {
    size_t bucket;
    char key[40];
    int n;
} walk_rec;

static size_t walk(struct ZHashTable *t, walk_rec *out)
{
    size_t k = 0;
    for (size_t b = 0; b < kb_zhash_sizes[t->size_index]; b++)
        for (struct ZHashEntry *e = t->entries[b]; e; e = e->next) {
            int n = 0;
            for (ll_node *x = e->val; x; x = x->next) n++;
            out[k].bucket = b;
            strcpy(out[k].key, e->key);
            out[k].n = n;
            k++;
        }
    return k;
}

int main(void)
{
    /* the encoding */
    for (int v = 0; v < 4; v++) CHECK(getval(getbp(v)) == v);
    CHECK(getbp(7) == 'A' && getbp(-1) == 'A');
    CHECK(getval('N') == 3 && getval('a') == 3);
    const char *strs[] = {"T", "A", "GATTACA", "CTTTTTT", "ACGTACGTACGTACG", "AAAAAAAAAAAAAAAA", ""};
    for (size_t i = 0; i < sizeof strs / sizeof *strs; i++)
        printf("score %s %d\n", strs[i][0] ? strs[i] : "-", getscore((char *)strs[i]));

    const int cutoff = 2;
    kbh_configure(31, 7, cutoff, 0);
    for (int round = 0; round < 4; round++) {
        const int nkeys = round == 3 ? 40 : 3000;
        struct ZHashTable *t = zcreate_hash_table();
        for (int i = 0; i < nkeys; i++) {
            char key[32];
            for (int j = 0; j < 31; j++) key[j] = getbp((int)(next() & 3));
            key[31] = '\0';
            if (zhash_exists(t, key)) continue;
            /* lists of 1..5 ids (round 3: all <= cutoff, the table empties) */
            const int n = round == 3 ? 1 + (int)(next() % cutoff) : 1 + (int)(next() % 5);
            ll_node *head = NULL;
            for (int j = 0; j < n; j++) {
                ll_node *x = create_node_num((int)(next() % 100000));
                x->next = head;
                head = x;
            }
            zhash_set(t, key, head);
        }
        walk_rec *before = malloc(t->entry_count * sizeof(walk_rec));
        const size_t nb = walk(t, before);
        const size_t step = t->size_index, count = t->entry_count;
        CHECK(nb == count);
        size_t kept = 0;
        for (size_t i = 0; i < nb; i++) kept += before[i].n > cutoff;
        struct ZHashTable *r = prune_kmers(t);
        if (kept == 0) {
            CHECK(r == NULL);
            printf("round %d: %zu keys, all pruned -> NULL\n", round, nb);
        } else {
            CHECK(r == t);
            CHECK(t->size_index == step);
            CHECK(t->entry_count == kept);
            walk_rec *after = malloc(kept * sizeof(walk_rec));
            CHECK(walk(t, after) == kept);
            size_t j = 0;
            for (size_t i = 0; i < nb; i++) {
                if (before[i].n <= cutoff) continue;
                CHECK(after[j].bucket == before[i].bucket);
                CHECK(strcmp(after[j].key, before[i].key) == 0);
                CHECK(after[j].n == before[i].n);
                j++;
            }
            printf("round %d: %zu keys, %zu kept, step %zu\n", round, nb, kept, step);
            free(after);
            zfree_hash_table(t);
        }
        free(before);
        (void)count;
    }
    printf("ok\n");
    return 0;
}
