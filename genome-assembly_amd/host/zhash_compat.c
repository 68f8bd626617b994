/*
 * zhash_compat.c -- clean-room implementation of the reference container API
 * (twitu/genome-assembly zhash.h / llist.h), used when the reference's own
 * zhash.c / llist.c are not linked (our tests, the kbin_main CLI).
 *
 * Behaviour restated from the reference so materialised tables have the same
 * shape: separate chaining over the prime ladder of zhash.c:13-17; bucket of a
 * key = fold of (17*h + byte) mod size over its bytes (zhash.c:171-182); new
 * entries are pushed on the chain head (zhash.c:148-161); the table moves one
 * ladder step up once entry_count exceeds half the bucket count (zhash.c:77-79)
 * and one step down on delete below an eighth (zhash.c:128-130); a rehash walks
 * the old buckets in index order, pushing each entry onto its new chain
 * (zhash.c:184-214).  Keys are copied, values are borrowed.
 */
#include <stdlib.h>
#include <string.h>

#include "../../include/kb_zhash.h"

const size_t kb_zhash_sizes[23] = {
    53, 101, 211, 503, 1553, 3407, 6803, 12503, 25013, 50261, 104729, 250007,
    500009, 1000003, 2000029, 4000037, 10000019, 25000009, 50000047, 104395301,
    217645177, 512927357, 1000000007};

#define LADDER_TOP (sizeof(kb_zhash_sizes) / sizeof(kb_zhash_sizes[0]))

static void *must(void *p)
{
    if (!p) exit(EXIT_FAILURE); /* the reference's OOM convention */
    return p;
}

static struct ZHashTable *table_at(size_t step)
{
    struct ZHashTable *t = must(malloc(sizeof *t));
    t->size_index = step;
    t->entry_count = 0;
    t->entries = must(calloc(kb_zhash_sizes[step], sizeof(struct ZHashEntry *)));
    return t;
}

struct ZHashTable *zcreate_hash_table(void) { return table_at(0); }

size_t zgenerate_hash(struct ZHashTable *t, char *key)
{
    const size_t m = kb_zhash_sizes[t->size_index];
    size_t h = 0;
    for (const unsigned char *p = (const unsigned char *)key; *p; p++)
        h = (h * 17 + (size_t)(char)*p) % m;
    return h;
}

struct ZHashEntry *zcreate_entry(char *key, void *val)
{
    size_t n = strlen(key) + 1;
    struct ZHashEntry *e = must(malloc(sizeof *e));
    e->key = must(malloc(n));
    memcpy(e->key, key, n);
    e->val = val;
    e->next = NULL;
    return e;
}

void zfree_entry(struct ZHashEntry *e, bool recursive)
{
    while (e) {
        struct ZHashEntry *nx = recursive ? e->next : NULL;
        free(e->key);
        free(e);
        e = nx;
    }
}

void zfree_hash_table(struct ZHashTable *t)
{
    const size_t m = kb_zhash_sizes[t->size_index];
    for (size_t b = 0; b < m; b++)
        zfree_entry(t->entries[b], true);
    free(t->entries);
    free(t);
}

void zhash_rehash(struct ZHashTable *t, size_t step)
{
    if (step == t->size_index) return;
    const size_t old_m = kb_zhash_sizes[t->size_index];
    struct ZHashEntry **old = t->entries;
    t->size_index = step;
    t->entries = must(calloc(kb_zhash_sizes[step], sizeof(struct ZHashEntry *)));
    for (size_t b = 0; b < old_m; b++) {
        struct ZHashEntry *e = old[b];
        while (e) {
            struct ZHashEntry *nx = e->next;
            size_t h = zgenerate_hash(t, e->key);
            e->next = t->entries[h];
            t->entries[h] = e;
            e = nx;
        }
    }
    free(old);
}

static struct ZHashEntry *find(struct ZHashTable *t, char *key)
{
    struct ZHashEntry *e = t->entries[zgenerate_hash(t, key)];
    while (e && strcmp(e->key, key) != 0) e = e->next;
    return e;
}

void zhash_set(struct ZHashTable *t, char *key, void *val)
{
    struct ZHashEntry *e = find(t, key);
    if (e) {
        e->val = val;
        return;
    }
    size_t h = zgenerate_hash(t, key);
    e = zcreate_entry(key, val);
    e->next = t->entries[h];
    t->entries[h] = e;
    t->entry_count++;
    if (t->entry_count > kb_zhash_sizes[t->size_index] / 2) {
        size_t up = t->size_index + 1 < LADDER_TOP ? t->size_index + 1 : t->size_index;
        zhash_rehash(t, up);
    }
}

void *zhash_get(struct ZHashTable *t, char *key)
{
    struct ZHashEntry *e = find(t, key);
    return e ? e->val : NULL;
}

bool zhash_exists(struct ZHashTable *t, char *key) { return find(t, key) != NULL; }

void *zhash_delete(struct ZHashTable *t, char *key)
{
    struct ZHashEntry **link = &t->entries[zgenerate_hash(t, key)];
    while (*link && strcmp((*link)->key, key) != 0) link = &(*link)->next;
    struct ZHashEntry *e = *link;
    if (!e) return NULL;
    *link = e->next;
    void *val = e->val;
    zfree_entry(e, false);
    t->entry_count--;
    if (t->entry_count < kb_zhash_sizes[t->size_index] / 8 && t->size_index > 0)
        zhash_rehash(t, t->size_index - 1);
    return val;
}

/* llist.h:21-33 subset used by the materialiser and downstream code */
ll_node *create_node_num(int id)
{
    ll_node *n = must(malloc(sizeof *n));
    n->next = NULL;
    n->read_id = id;
    return n;
}

ll_node *create_node_item(void *item)
{
    ll_node *n = must(malloc(sizeof *n));
    n->next = NULL;
    n->item = item;
    return n;
}

void free_llist(ll_node *list)
{
    while (list) {
        ll_node *nx = list->next;
        free(list);
        list = nx;
    }
}
