/*
 * pyset.c -- CPython 3.10 set-table model for int keys (TEST INFRASTRUCTURE ONLY).
 * Behaviour modelled: Objects/setobject.c of CPython 3.10 (set_add_entry,
 * set_insert_clean, set_table_resize, set_merge, set_difference,
 * set_copy_and_difference, set_or, set_pop).  See pyset.h for why.
 */
#include "pyset.h"
#include <stdlib.h>
#include <string.h>

#define LINEAR_PROBES 9
#define PERTURB_SHIFT 5

static inline int64_t py_hash_int(int64_t x) { return x == -1 ? -2 : x; }

static pyentry *alloc_table(int64_t size) { return (pyentry *)calloc((size_t)size, sizeof(pyentry)); }

void pyset_init(pyset *s) {
    s->mask = PYSET_MINSIZE - 1;
    s->fill = s->used = s->finger = 0;
    s->table = alloc_table(PYSET_MINSIZE);
}

void pyset_free(pyset *s) {
    free(s->table);
    s->table = NULL;
}

static void insert_clean(pyentry *table, uint64_t mask, int64_t key, int64_t hash) {
    uint64_t perturb = (uint64_t)hash;
    uint64_t i = (uint64_t)hash & mask;
    for (;;) {
        pyentry *e = &table[i];
        if (e->key == 0) { e->key = key; e->hash = hash; return; }
        if (i + LINEAR_PROBES <= mask) {
            for (int j = 0; j < LINEAR_PROBES; j++) {
                e++;
                if (e->key == 0) { e->key = key; e->hash = hash; return; }
            }
        }
        perturb >>= PERTURB_SHIFT;
        i = (i * 5 + 1 + perturb) & mask;
    }
}

static void table_resize(pyset *s, int64_t minused) {
    int64_t newsize = PYSET_MINSIZE;
    while (newsize <= minused) newsize <<= 1;
    pyentry *old = s->table;
    int64_t oldmask = s->mask;
    /* small table kept and no dummies: CPython returns without touching it */
    if (newsize == PYSET_MINSIZE && oldmask == PYSET_MINSIZE - 1 && s->fill == s->used) return;
    pyentry *nt = alloc_table(newsize);
    s->mask = newsize - 1;
    s->table = nt;
    for (int64_t k = 0; k <= oldmask; k++) {
        pyentry *e = &old[k];
        if (e->key != 0 && e->key != PYSET_DUMMY) insert_clean(nt, (uint64_t)s->mask, e->key, e->hash);
    }
    s->fill = s->used;
    free(old);
}

static void add_entry(pyset *s, int64_t key, int64_t hash) {
    uint64_t mask = (uint64_t)s->mask;
    uint64_t i = (uint64_t)hash & mask;
    pyentry *e = &s->table[i];
    pyentry *freeslot = NULL;
    uint64_t perturb;
    if (e->key == 0) goto found_unused;
    perturb = (uint64_t)hash;
    for (;;) {
        if (e->hash == hash && e->key == key) return;          /* found_active */
        else if (e->hash == -1 && e->key == PYSET_DUMMY) freeslot = e;
        if (i + LINEAR_PROBES <= mask) {
            for (int j = 0; j < LINEAR_PROBES; j++) {
                e++;
                if (e->hash == 0 && e->key == 0) goto found_unused_or_dummy;
                if (e->hash == hash && e->key == key) return;
                else if (e->hash == -1 && e->key == PYSET_DUMMY) freeslot = e;
            }
        }
        perturb >>= PERTURB_SHIFT;
        i = (i * 5 + 1 + perturb) & mask;
        e = &s->table[i];
        if (e->key == 0) goto found_unused_or_dummy;
    }
found_unused_or_dummy:
    if (freeslot == NULL) goto found_unused;
    s->used++;
    freeslot->key = key; freeslot->hash = hash;
    return;
found_unused:
    s->fill++; s->used++;
    e->key = key; e->hash = hash;
    if ((uint64_t)s->fill * 5 < mask * 3) return;
    table_resize(s, s->used > 50000 ? s->used * 2 : s->used * 4);
}

void pyset_add(pyset *s, int64_t key) { add_entry(s, key, py_hash_int(key)); }
void pyset_add_hashed(pyset *s, int64_t key, int64_t hash) { add_entry(s, key, hash); }

int pyset_contains(const pyset *s, int64_t key) {
    int64_t hash = py_hash_int(key);
    uint64_t mask = (uint64_t)s->mask, i = (uint64_t)hash & mask, perturb = (uint64_t)hash;
    const pyentry *e = &s->table[i];
    if (e->key == 0) return 0;
    for (;;) {
        if (e->hash == hash && e->key == key) return 1;
        if (i + LINEAR_PROBES <= mask) {
            for (int j = 0; j < LINEAR_PROBES; j++) {
                e++;
                if (e->hash == 0 && e->key == 0) return 0;
                if (e->hash == hash && e->key == key) return 1;
            }
        }
        perturb >>= PERTURB_SHIFT;
        i = (i * 5 + 1 + perturb) & mask;
        e = &s->table[i];
        if (e->key == 0) return 0;
    }
}

void pyset_from_array(pyset *s, const int64_t *keys, int n) {
    pyset_init(s);
    for (int k = 0; k < n; k++) pyset_add(s, keys[k]);
}

/* set_merge(so, other) */
static void merge(pyset *so, const pyset *other) {
    if (other == so || other->used == 0) return;
    if ((so->fill + other->used) * 5 >= so->mask * 3) table_resize(so, (so->used + other->used) * 2);
    if (so->fill == 0 && so->mask == other->mask && other->fill == other->used) {
        memcpy(so->table, other->table, sizeof(pyentry) * (size_t)(other->mask + 1));
        so->fill = other->fill; so->used = other->used;
        return;
    }
    if (so->fill == 0) {
        so->fill = other->used; so->used = other->used;
        for (int64_t k = 0; k <= other->mask; k++) {
            const pyentry *e = &other->table[k];
            if (e->key != 0 && e->key != PYSET_DUMMY) insert_clean(so->table, (uint64_t)so->mask, e->key, e->hash);
        }
        return;
    }
    for (int64_t k = 0; k <= other->mask; k++) {
        const pyentry *e = &other->table[k];
        if (e->key != 0 && e->key != PYSET_DUMMY) add_entry(so, e->key, e->hash);
    }
}

void pyset_copy(pyset *dst, const pyset *src) {
    pyset_init(dst);
    merge(dst, src);
}

static void discard_hashed(pyset *s, int64_t key, int64_t hash);
static void discard(pyset *s, int64_t key) { discard_hashed(s, key, py_hash_int(key)); }
int pyset_discard_hashed(pyset *s, int64_t key, int64_t hash) {
    const int64_t before = s->used;
    discard_hashed(s, key, hash);
    return s->used < before;
}
static void discard_hashed(pyset *s, int64_t key, int64_t hash) {
    uint64_t mask = (uint64_t)s->mask, i = (uint64_t)hash & mask, perturb = (uint64_t)hash;
    pyentry *e = &s->table[i];
    if (e->key == 0) return;
    for (;;) {
        if (e->hash == hash && e->key == key) goto found;
        if (i + LINEAR_PROBES <= mask) {
            for (int j = 0; j < LINEAR_PROBES; j++) {
                e++;
                if (e->hash == 0 && e->key == 0) return;
                if (e->hash == hash && e->key == key) goto found;
            }
        }
        perturb >>= PERTURB_SHIFT;
        i = (i * 5 + 1 + perturb) & mask;
        e = &s->table[i];
        if (e->key == 0) return;
    }
found:
    e->key = PYSET_DUMMY; e->hash = -1; s->used--;
}

void pyset_difference(pyset *dst, const pyset *a, const pyset *b) {
    if ((a->used >> 2) > b->used) {          /* set_copy_and_difference */
        pyset_copy(dst, a);
        for (int64_t k = 0; k <= b->mask; k++) {
            const pyentry *e = &b->table[k];
            if (e->key != 0 && e->key != PYSET_DUMMY) discard(dst, e->key);
        }
        return;
    }
    pyset_init(dst);
    for (int64_t k = 0; k <= a->mask; k++) {
        const pyentry *e = &a->table[k];
        if (e->key != 0 && e->key != PYSET_DUMMY && !pyset_contains(b, e->key)) add_entry(dst, e->key, e->hash);
    }
}

void pyset_or(pyset *dst, const pyset *a, const pyset *b) {
    pyset_copy(dst, a);
    if (a == b) return;
    merge(dst, b);
}

int pyset_items(const pyset *s, int64_t *out) {
    int n = 0;
    for (int64_t k = 0; k <= s->mask; k++) {
        const pyentry *e = &s->table[k];
        if (e->key != 0 && e->key != PYSET_DUMMY) out[n++] = e->key;
    }
    return n;
}

int64_t pyset_pop(pyset *s) {
    int64_t k = s->finger & s->mask;
    while (s->table[k].key == 0 || s->table[k].key == PYSET_DUMMY) {
        k++;
        if (k > s->mask) k = 0;
    }
    int64_t key = s->table[k].key;
    s->table[k].key = PYSET_DUMMY; s->table[k].hash = -1;
    s->used--;
    s->finger = k + 1;
    return key;
}

int pyset_issuperset(const pyset *a, const pyset *b) {
    if (b->used > a->used) return 0;
    for (int64_t k = 0; k <= b->mask; k++) {
        const pyentry *e = &b->table[k];
        if (e->key != 0 && e->key != PYSET_DUMMY && !pyset_contains(a, e->key)) return 0;
    }
    return 1;
}

/* ---- exported probes used by tests/test_pyset_model.py ---- */
/* Build set(list) for `n` keys and write its iteration order. */
int pyset_probe_from_list(const int64_t *keys, int n, int64_t *out) {
    pyset s; pyset_from_array(&s, keys, n);
    int m = pyset_items(&s, out); pyset_free(&s); return m;
}
/* (set(A) - {x}) | (set(B) - {y})  -- the resolvent construction of REF.py:114 */
int pyset_probe_resolvent(const int64_t *a, int na, int64_t x, const int64_t *b, int nb, int64_t y, int64_t *out) {
    pyset A, B, X, Y, AX, BY, R;
    pyset_from_array(&A, a, na); pyset_from_array(&B, b, nb);
    pyset_from_array(&X, &x, 1); pyset_from_array(&Y, &y, 1);
    pyset_difference(&AX, &A, &X); pyset_difference(&BY, &B, &Y);
    pyset_or(&R, &AX, &BY);
    int m = pyset_items(&R, out);
    pyset_free(&A); pyset_free(&B); pyset_free(&X); pyset_free(&Y);
    pyset_free(&AX); pyset_free(&BY); pyset_free(&R);
    return m;
}
/* {abs(l) for each list in lists for l in set(list)} then pop() */
int64_t pyset_probe_var_pop(const int64_t *lits, const int *off, int nlists) {
    pyset V; pyset_init(&V);
    int64_t buf[4096];
    for (int c = 0; c < nlists; c++) {
        pyset C; pyset_from_array(&C, lits + off[c], off[c + 1] - off[c]);
        int m = pyset_items(&C, buf);
        for (int k = 0; k < m; k++) pyset_add(&V, buf[k] < 0 ? -buf[k] : buf[k]);
        pyset_free(&C);
    }
    int64_t r = V.used ? pyset_pop(&V) : 0;
    pyset_free(&V);
    return r;
}
