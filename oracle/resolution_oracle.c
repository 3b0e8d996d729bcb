/*
 * resolution_oracle.c -- CPU restatement of resolution_solver (REF.py:63-95).
 * TEST INFRASTRUCTURE ONLY (see sat_oracle.c header).
 *
 * Saturation in passes: every pass resolves every pair (i < j) of the current
 * clause list on every clashing literal, skips tautologies, stops with False on
 * an empty resolvent, and adds the resolvents not seen before; True when a pass
 * adds nothing.  Each pass's new-clause *set* is independent of iteration order,
 * so clauses are kept canonical (sorted, de-duplicated literals).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { int32_t *lits; int64_t nl, capl; int64_t *off; int64_t n, capn; } cstore;

static void cs_init(cstore *s) { memset(s, 0, sizeof(*s)); s->capn = 64; s->off = (int64_t *)calloc(65, sizeof(int64_t)); }
static void cs_free(cstore *s) { free(s->lits); free(s->off); }
static int64_t cs_add(cstore *s, const int32_t *l, int n) {
    if (s->nl + n > s->capl) { s->capl = (s->nl + n) * 2 + 64; s->lits = (int32_t *)realloc(s->lits, sizeof(int32_t) * (size_t)s->capl); }
    if (s->n + 1 >= s->capn) { s->capn *= 2; s->off = (int64_t *)realloc(s->off, sizeof(int64_t) * (size_t)(s->capn + 1)); }
    memcpy(s->lits + s->nl, l, sizeof(int32_t) * (size_t)n);
    s->nl += n; s->n++; s->off[s->n] = s->nl;
    return s->n - 1;
}

/* hash set of canonical clauses (indices into a cstore) */
typedef struct { int64_t *slot; uint64_t mask; int64_t used; } chash;
static uint64_t clause_hash(const int32_t *l, int n) {
    uint64_t h = 1469598103934665603ULL ^ (uint64_t)n;
    for (int i = 0; i < n; i++) { h ^= (uint64_t)(uint32_t)l[i]; h *= 1099511628211ULL; h ^= h >> 29; }
    return h;
}
static void ch_init(chash *h, uint64_t cap) { uint64_t c = 64; while (c < cap * 2) c <<= 1; h->slot = (int64_t *)malloc(sizeof(int64_t) * c); memset(h->slot, 0xff, sizeof(int64_t) * c); h->mask = c - 1; h->used = 0; }
static int ch_find_or_insert(chash *h, cstore *st, const int32_t *l, int n, int insert);
static void ch_grow(chash *h, cstore *st) {
    chash g; ch_init(&g, (h->mask + 1));
    for (uint64_t i = 0; i <= h->mask; i++) if (h->slot[i] >= 0) {
        int64_t id = h->slot[i];
        const int32_t *l = st->lits + st->off[id]; int n = (int)(st->off[id + 1] - st->off[id]);
        uint64_t k = clause_hash(l, n) & g.mask;
        while (g.slot[k] >= 0) k = (k + 1) & g.mask;
        g.slot[k] = id; g.used++;
    }
    free(h->slot); *h = g;
}
/* returns 1 if present; if absent and insert: stores into st and returns 0 */
static int ch_find_or_insert(chash *h, cstore *st, const int32_t *l, int n, int insert) {
    uint64_t k = clause_hash(l, n) & h->mask;
    while (h->slot[k] >= 0) {
        int64_t id = h->slot[k];
        if (st->off[id + 1] - st->off[id] == n && memcmp(st->lits + st->off[id], l, sizeof(int32_t) * (size_t)n) == 0) return 1;
        k = (k + 1) & h->mask;
    }
    if (!insert) return 0;
    h->slot[k] = cs_add(st, l, n); h->used++;
    if ((uint64_t)h->used * 2 > h->mask) ch_grow(h, st);
    return 0;
}

static int cmp_i32(const void *a, const void *b) { int32_t x = *(const int32_t *)a, y = *(const int32_t *)b; return (x > y) - (x < y); }
static int canon(int32_t *l, int n) {   /* sort + unique -> new length */
    qsort(l, (size_t)n, sizeof(int32_t), cmp_i32);
    int m = 0;
    for (int i = 0; i < n; i++) if (m == 0 || l[m - 1] != l[i]) l[m++] = l[i];
    return m;
}

/*
 * Returns 1 (True), 0 (False), -1 (aborted by pass/clause limits).
 * pass_new[p] = size of the new-clause set added by completed pass p.
 * If rec_lits != NULL, the canonical new clauses of each completed pass are
 * appended in sorted order (rec_pass_off indexes rec_clause_off).
 */
int oracle_resolution(int nclauses, const int32_t *off, const int32_t *lits,
                      int max_passes, int64_t clause_limit,
                      int64_t *pass_new, int pass_cap, int *n_passes,
                      int32_t *rec_lits, int64_t rec_lit_cap, int64_t *rec_clause_off, int64_t rec_clause_cap,
                      int64_t *rec_pass_off, int rec_pass_cap) {
    cstore list; cs_init(&list);      /* `clauses` (REF.py:64), canonical */
    cstore seenst; cs_init(&seenst);
    chash seen; ch_init(&seen, (uint64_t)nclauses + 16);
    int32_t *buf = NULL; int bufcap = 0;
    for (int c = 0; c < nclauses; c++) {
        int n = off[c + 1] - off[c];
        if (n + 1 > bufcap) { bufcap = n + 64; buf = (int32_t *)realloc(buf, sizeof(int32_t) * (size_t)bufcap); }
        memcpy(buf, lits + off[c], sizeof(int32_t) * (size_t)n);
        n = canon(buf, n);
        cs_add(&list, buf, n);
        ch_find_or_insert(&seen, &seenst, buf, n, 1);
    }
    int64_t rl = 0, rc = 0; int rp = 0;
    if (rec_pass_off) rec_pass_off[0] = 0;
    if (rec_clause_off) rec_clause_off[0] = 0;
    int passes = 0, result = -1;
    for (;;) {
        if (max_passes > 0 && passes >= max_passes) { result = -1; break; }
        cstore fresh; cs_init(&fresh);
        chash freshh; ch_init(&freshh, 64);
        int64_t n = list.n;
        int empty = 0, too_big = 0;
        for (int64_t i = 0; i < n && !empty && !too_big; i++) {
            const int32_t *ci = list.lits + list.off[i]; int ni = (int)(list.off[i + 1] - list.off[i]);
            for (int64_t j = i + 1; j < n && !empty && !too_big; j++) {
                const int32_t *cj = list.lits + list.off[j]; int nj = (int)(list.off[j + 1] - list.off[j]);
                for (int a = 0; a < ni; a++) {
                    int32_t lit = ci[a];
                    int clash = 0;
                    for (int b = 0; b < nj; b++) if (cj[b] == -lit) { clash = 1; break; }
                    if (!clash) continue;
                    /* resolvent = (ci | cj) - {lit, -lit} */
                    if (ni + nj + 1 > bufcap) { bufcap = ni + nj + 64; buf = (int32_t *)realloc(buf, sizeof(int32_t) * (size_t)bufcap); }
                    int m = 0;
                    for (int b = 0; b < ni; b++) if (ci[b] != lit && ci[b] != -lit) buf[m++] = ci[b];
                    for (int b = 0; b < nj; b++) if (cj[b] != lit && cj[b] != -lit) buf[m++] = cj[b];
                    m = canon(buf, m);
                    int taut = 0;   /* sorted: x and -x both present? */
                    for (int b = 0; b < m && !taut; b++)
                        if (buf[b] < 0) { for (int e = m - 1; e >= 0 && buf[e] > 0; e--) if (buf[e] == -buf[b]) { taut = 1; break; } }
                    if (taut) continue;
                    if (m == 0) { empty = 1; break; }
                    if (ch_find_or_insert(&seen, &seenst, buf, m, 0)) continue;
                    ch_find_or_insert(&freshh, &fresh, buf, m, 1);
                    if (clause_limit > 0 && list.n + fresh.n > clause_limit) { too_big = 1; break; }
                }
            }
        }
        if (empty) { result = 0; cs_free(&fresh); free(freshh.slot); break; }
        if (too_big) { result = -1; cs_free(&fresh); free(freshh.slot); break; }
        if (fresh.n == 0) { result = 1; cs_free(&fresh); free(freshh.slot); break; }
        if (passes < pass_cap && pass_new) pass_new[passes] = fresh.n;
        /* seen.update(new_clauses); clauses.extend(...) */
        int64_t *order = (int64_t *)malloc(sizeof(int64_t) * (size_t)fresh.n);
        for (int64_t k = 0; k < fresh.n; k++) order[k] = k;
        /* record sorted (lexicographic on the sorted literal lists, like Python's sorted()) */
        if (rec_lits && rp < rec_pass_cap) {
            /* insertion sort is fine for the small passes that get recorded */
            for (int64_t x = 1; x < fresh.n; x++) {
                int64_t key = order[x], y = x - 1;
                while (y >= 0) {
                    const int32_t *A = fresh.lits + fresh.off[order[y]]; int na = (int)(fresh.off[order[y] + 1] - fresh.off[order[y]]);
                    const int32_t *B = fresh.lits + fresh.off[key]; int nb = (int)(fresh.off[key + 1] - fresh.off[key]);
                    int c = 0, t = 0;
                    while (t < na && t < nb && c == 0) { c = (A[t] > B[t]) - (A[t] < B[t]); t++; }
                    if (c == 0) c = (na > nb) - (na < nb);
                    if (c <= 0) break;
                    order[y + 1] = order[y]; y--;
                }
                order[y + 1] = key;
            }
            for (int64_t k = 0; k < fresh.n && rc < rec_clause_cap; k++) {
                int64_t id = order[k];
                for (int64_t t = fresh.off[id]; t < fresh.off[id + 1] && rl < rec_lit_cap; t++) rec_lits[rl++] = fresh.lits[t];
                rec_clause_off[++rc] = rl;
            }
            rec_pass_off[++rp] = rc;
        }
        for (int64_t k = 0; k < fresh.n; k++) {
            const int32_t *l = fresh.lits + fresh.off[k]; int m = (int)(fresh.off[k + 1] - fresh.off[k]);
            ch_find_or_insert(&seen, &seenst, l, m, 1);
            cs_add(&list, l, m);
        }
        free(order);
        cs_free(&fresh); free(freshh.slot);
        passes++;
    }
    if (n_passes) *n_passes = passes;
    cs_free(&list); cs_free(&seenst); free(seen.slot); free(buf);
    return result;
}
