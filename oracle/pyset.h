/*
 * pyset.h -- a model of CPython 3.10's `set` object restricted to small int keys.
 *
 * TEST INFRASTRUCTURE ONLY (see sat_oracle.c header).
 *
 * Why: the reference's Davis-Putnam solver picks the variable to eliminate with
 * `variables.pop()` on a set built from Python sets of literals (REF.py:100-103,
 * :128).  Which element `pop()` returns is decided by the hash-table layout of
 * that set, which depends on the order clauses' literal sets iterate, which in
 * turn depends on how each clause set was built ( set(list), `pc - {var}`,
 * `a | b` at REF.py:64/99/114 ).  To reproduce the reference's elimination order
 * (and therefore its intermediate resolvent sets) we model CPython's set table:
 * open addressing with 9 linear probes then perturbed probing, fill/used
 * accounting with dummies, and its resize policy.  The model is checked against
 * the real interpreter in tests/test_pyset_model.py.
 */
#ifndef SATMI_ORACLE_PYSET_H
#define SATMI_ORACLE_PYSET_H
#include <stdint.h>

typedef struct {
    int64_t key;   /* 0 = unused slot (keys are never 0), PYSET_DUMMY = deleted */
    int64_t hash;  /* CPython hash of key; -1 marks a dummy                      */
} pyentry;

#define PYSET_DUMMY INT64_MIN
#define PYSET_MINSIZE 8

typedef struct {
    int64_t mask, fill, used, finger;
    pyentry *table;
} pyset;

void pyset_init(pyset *s);                        /* empty set (8 slots) */
void pyset_free(pyset *s);
void pyset_add(pyset *s, int64_t key);            /* set_add_key          */
/* the same with the caller's hash: keys stored as x + 1 (0 marks an unused slot)
 * for non-negative ints x, whose CPython hash is x */
void pyset_add_hashed(pyset *s, int64_t key, int64_t hash);
int  pyset_discard_hashed(pyset *s, int64_t key, int64_t hash);   /* 1 if it was present */
int  pyset_contains(const pyset *s, int64_t key); /* `key in s`           */
void pyset_from_array(pyset *s, const int64_t *keys, int n);   /* set(list)  */
void pyset_copy(pyset *dst, const pyset *src);    /* set_copy / make_new_set(src) */
void pyset_difference(pyset *dst, const pyset *a, const pyset *b);   /* a - b  */
void pyset_or(pyset *dst, const pyset *a, const pyset *b);           /* a | b  */
int  pyset_items(const pyset *s, int64_t *out);   /* iteration order; returns count */
int64_t pyset_pop(pyset *s);                      /* set.pop()            */
int  pyset_issuperset(const pyset *a, const pyset *b);

#endif
