/*
 * kb_zhash.h -- container types of the reference's public surface, declared
 * with the SAME layout and function names as twitu/genome-assembly
 *   zhash.h:14-44  struct ZHashEntry / struct ZHashTable, zcreate_hash_table,
 *                  zhash_set, zhash_get, ... (chained string hash)
 *   llist.h:7-33   ll_node (read-id list node), create_node_num, ...
 * so that code written against the reference (binning.c's iterators,
 * expand_read_id_list, find_kmer_extensions, print_kmers) can walk the tables
 * that prune_data() materialises from the GPU result.
 *
 * When the reference's own zhash.c / llist.c are linked (the drop-in case,
 * INTEGRATION.md) they provide these symbols; otherwise
 * genome-assembly_amd/host/zhash_compat.c provides a clean-room
 * implementation with the same hash function and size ladder.
 */
#ifndef KB_ZHASH_H
#define KB_ZHASH_H

#include <stdbool.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef ZHASH_H /* the reference header may already be included */
struct ZHashEntry {
    char *key;
    void *val;
    struct ZHashEntry *next;
};

struct ZHashTable {
    size_t size_index;
    size_t entry_count;
    struct ZHashEntry **entries;
};

struct ZHashTable *zcreate_hash_table(void);
void zfree_hash_table(struct ZHashTable *hash_table);
void zhash_set(struct ZHashTable *hash_table, char *key, void *val);
void *zhash_get(struct ZHashTable *hash_table, char *key);
void *zhash_delete(struct ZHashTable *hash_table, char *key);
bool zhash_exists(struct ZHashTable *hash_table, char *key);
struct ZHashEntry *zcreate_entry(char *key, void *val);
void zfree_entry(struct ZHashEntry *entry, bool recursive);
size_t zgenerate_hash(struct ZHashTable *hash, char *key);
void zhash_rehash(struct ZHashTable *hash_table, size_t size_index);
#endif

#ifndef LLIST_H
typedef struct ll_node {
    struct ll_node *next;
    union {
        int read_id;
        void *item;
    };
} ll_node;

ll_node *create_node_num(int id);
ll_node *create_node_item(void *item);
void free_llist(ll_node *list);
#endif

/* prime ladder of zhash.c:13-17 (exported so walkers can size iterations) */
extern const size_t kb_zhash_sizes[23];

#ifdef __cplusplus
}
#endif
#endif
