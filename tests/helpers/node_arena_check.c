/* node_arena_check.c -- CPU check of the drop-in's list-node arena
 * (binning_gpu.c: node_new / free interposition), linked like the drop-in:
 * this executable links libkbin_host.so, whose free() then is the process's.
 * Materialises a synthetic CSR (kbh_materialise_csr, prune on), expands it
 * (expand_read_id_list), prints a digest of every entry's outer list and
 * copied id lists, then frees every node the way free_llist does (llist.c:
 * 101-108) and prints whether the nodes came from the arena.  The pytest
 * runs it with KBH_NODE_ARENA unset and =0: same digest, arena 1 then 0. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../include/binning_gpu.h"
#include "../../include/kb_zhash.h"

static uint64_t mix(uint64_t x)
{
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    return x;
}

int main(int argc, char **argv)
{
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 20000;
    const int K = 31, M = 7;
    uint32_t *mmer = malloc(n * 4), *count = malloc(n * 4);
    uint64_t *hi = calloc(n, 8), *lo = malloc(n * 8), *off = malloc((n + 1) * 8), *first = malloc(n * 8);
    off[0] = 0;
    for (uint64_t i = 0; i < n; i++) {
        mmer[i] = (uint32_t)(mix(i) % (1u << (2 * M)));
        lo[i] = (mix(i + 77) & ((1ull << 40) - 1)) | (i << 40);
        lo[i] &= (1ull << (2 * K)) - 1;
        count[i] = 1 + (uint32_t)(mix(i + 5) % 5); /* 1 is pruned at cutoff 1 */
        off[i + 1] = off[i] + count[i];
        first[i] = i << 16;
    }
    int32_t *ids = malloc(off[n] * 4);
    for (uint64_t k = 0; k < off[n]; k++) ids[k] = (int32_t)(mix(k + 999) % 1000000);
    kb_csr c = {n, off[n], 0, 0, mmer, hi, lo, count, off, ids, first};
    if (kbh_configure(K, M, 1, 0) != 0) return 2;
    struct ZHashTable *h = zcreate_hash_table();
    if (kbh_materialise_csr(h, &c, 1, 0) != 0) return 3;
    expand_read_id_list(h);
    uint64_t dig = 0, outer_n = 0, id_n = 0;
    for (size_t b1 = 0; b1 < (size_t)kb_zhash_sizes[h->size_index]; b1++)
        for (struct ZHashEntry *me = h->entries[b1]; me; me = me->next) {
            struct ZHashTable *t = me->val;
            for (size_t b2 = 0; b2 < (size_t)kb_zhash_sizes[t->size_index]; b2++)
                for (struct ZHashEntry *ke = t->entries[b2]; ke; ke = ke->next) {
                    uint64_t kd = 0;
                    for (const char *p = ke->key; *p; p++) kd = mix(kd + (uint64_t)*p);
                    uint64_t pos = 0;
                    for (ll_node *o = ke->val; o; o = o->next, outer_n++, pos++)
                        for (ll_node *x = o->item; x; x = x->next, id_n++)
                            dig += mix(kd ^ (pos << 40) ^ (uint64_t)(uint32_t)x->read_id);
                    /* free the lists as free_llist does: every node its own block */
                    for (ll_node *o = ke->val; o;) {
                        ll_node *on = o->next;
                        for (ll_node *x = o->item; x;) {
                            ll_node *xn = x->next;
                            free(x);
                            x = xn;
                        }
                        free(o);
                        o = on;
                    }
                    ke->val = NULL;
                }
        }
    printf("digest %016llx outer %llu ids %llu arena %d\n", (unsigned long long)dig, (unsigned long long)outer_n,
           (unsigned long long)id_n, kbh_node_arena_active());
    return 0;
}
