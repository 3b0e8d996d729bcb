/*
 * dp_oracle.c -- CPU restatement of davis_putnam_solver (REF.py:98-130).
 * TEST INFRASTRUCTURE ONLY (see sat_oracle.c header).
 *
 * Every clause is held as a modelled CPython set (pyset.h) so the elimination
 * order chosen by `variables.pop()` (REF.py:103) and the iteration order of every
 * clause match the reference exactly.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "pyset.h"

typedef struct { pyset *v; int n, cap; } setlist;

static void sl_push(setlist *l, pyset s) {
    if (l->n == l->cap) { l->cap = l->cap ? l->cap * 2 : 64; l->v = (pyset *)realloc(l->v, sizeof(pyset) * (size_t)l->cap); }
    l->v[l->n++] = s;
}

/* variables = {abs(lit) for clause in clauses for lit in clause}  (REF.py:100/128) */
static void build_vars(pyset *V, pyset *const *cl, int n) {
    pyset_init(V);
    for (int c = 0; c < n; c++) {
        const pyset *s = cl[c];
        for (int64_t k = 0; k <= s->mask; k++) {
            int64_t key = s->table[k].key;
            if (key != 0 && key != PYSET_DUMMY) pyset_add(V, key < 0 ? -key : key);
        }
    }
}

static int is_tautology(const pyset *r) {
    /* any(lit in resolvent and -lit in resolvent for lit in resolvent) (REF.py:115) */
    for (int64_t k = 0; k <= r->mask; k++) {
        int64_t key = r->table[k].key;
        if (key != 0 && key != PYSET_DUMMY && pyset_contains(r, -key)) return 1;
    }
    return 0;
}

/*
 * Returns 1 (True = satisfiable), 0 (False), -1 (aborted: step or size limit).
 * trace_vars[k] = variable eliminated at step k (up to trace_cap), *n_steps = steps run.
 * If rec_lits != NULL, the clause list after each completed step is appended
 * (clauses in list order, literals in set-iteration order):
 *   rec_step_off[s] .. rec_step_off[s+1] index clauses in rec_clause_off.
 */
int oracle_dp(int nclauses, const int32_t *off, const int32_t *lits,
              int64_t step_limit, int64_t clause_limit,
              int32_t *trace_vars, int trace_cap, int *n_steps,
              int32_t *rec_lits, int64_t rec_lit_cap, int64_t *rec_clause_off, int64_t rec_clause_cap,
              int64_t *rec_step_off, int rec_step_cap) {
    pyset **clauses = (pyset **)malloc(sizeof(pyset *) * (size_t)(nclauses > 0 ? nclauses : 1));
    int ncl = nclauses;
    for (int c = 0; c < nclauses; c++) {       /* clauses = [set(clause) ...] (REF.py:99) */
        clauses[c] = (pyset *)malloc(sizeof(pyset));
        int n = off[c + 1] - off[c];
        int64_t *tmp = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
        for (int j = 0; j < n; j++) tmp[j] = lits[off[c] + j];
        pyset_from_array(clauses[c], tmp, n);
        free(tmp);
    }
    int64_t rl = 0, rc = 0; int rs = 0;
    if (rec_step_off) { rec_step_off[0] = 0; }
    if (rec_clause_off) rec_clause_off[0] = 0;
    int steps = 0, result = 1;
    pyset V; build_vars(&V, clauses, ncl);
    while (V.used > 0) {                       /* while variables: */
        if (step_limit > 0 && steps >= step_limit) { result = -1; break; }
        int64_t var = pyset_pop(&V);           /* var = variables.pop() */
        if (steps < trace_cap && trace_vars) trace_vars[steps] = (int32_t)var;
        steps++;
        /* split (REF.py:106-108) -- list order preserved */
        pyset **pos = (pyset **)malloc(sizeof(pyset *) * (size_t)(ncl + 1));
        pyset **neg = (pyset **)malloc(sizeof(pyset *) * (size_t)(ncl + 1));
        pyset **rem = (pyset **)malloc(sizeof(pyset *) * (size_t)(ncl + 1));
        int np = 0, nn = 0, nr = 0;
        for (int c = 0; c < ncl; c++) if (pyset_contains(clauses[c], var)) pos[np++] = clauses[c];
        for (int c = 0; c < ncl; c++) if (pyset_contains(clauses[c], -var)) neg[nn++] = clauses[c];
        for (int c = 0; c < ncl; c++)
            if (!pyset_contains(clauses[c], var) && !pyset_contains(clauses[c], -var)) rem[nr++] = clauses[c];
        /* resolution (REF.py:111-119) */
        setlist nw = {0};
        pyset sv, snv; int64_t one = var, mone = -var;
        pyset_from_array(&sv, &one, 1); pyset_from_array(&snv, &mone, 1);
        int empty = 0, too_big = 0;
        for (int i = 0; i < np && !empty && !too_big; i++)
            for (int j = 0; j < nn; j++) {
                pyset a, b, r;
                pyset_difference(&a, pos[i], &sv);
                pyset_difference(&b, neg[j], &snv);
                pyset_or(&r, &a, &b);
                pyset_free(&a); pyset_free(&b);
                if (is_tautology(&r)) { pyset_free(&r); continue; }
                if (r.used == 0) { pyset_free(&r); empty = 1; break; }
                sl_push(&nw, r);
                if (clause_limit > 0 && nr + nw.n > clause_limit) { too_big = 1; break; }
            }
        pyset_free(&sv); pyset_free(&snv);
        if (empty || too_big) {
            for (int k = 0; k < nw.n; k++) pyset_free(&nw.v[k]);
            free(nw.v); free(pos); free(neg); free(rem);
            result = empty ? 0 : -1;
            break;
        }
        /* unique_new (REF.py:122-125): greedy, against remaining + unique_new */
        pyset **nextc = (pyset **)malloc(sizeof(pyset *) * (size_t)(nr + nw.n + 1));
        int nnext = 0;
        for (int k = 0; k < nr; k++) nextc[nnext++] = rem[k];
        for (int k = 0; k < nw.n; k++) {
            int sub = 0;
            for (int e = 0; e < nnext && !sub; e++)
                if (pyset_issuperset(&nw.v[k], nextc[e])) sub = 1;
            if (sub) { pyset_free(&nw.v[k]); continue; }
            pyset *keep = (pyset *)malloc(sizeof(pyset));
            *keep = nw.v[k];
            nextc[nnext++] = keep;
        }
        free(nw.v);
        /* free the clauses that left the formula (pos/neg sets) */
        for (int c = 0; c < ncl; c++)
            if (pyset_contains(clauses[c], var) || pyset_contains(clauses[c], -var)) { pyset_free(clauses[c]); free(clauses[c]); }
        free(pos); free(neg); free(rem); free(clauses);
        clauses = nextc; ncl = nnext;           /* clauses = remaining_clauses + unique_new */
        if (rec_lits && rs < rec_step_cap) {
            for (int c = 0; c < ncl && rc < rec_clause_cap; c++) {
                const pyset *s = clauses[c];
                for (int64_t k = 0; k <= s->mask; k++) {
                    int64_t key = s->table[k].key;
                    if (key != 0 && key != PYSET_DUMMY && rl < rec_lit_cap) rec_lits[rl++] = (int32_t)key;
                }
                rec_clause_off[++rc] = rl;
            }
            rec_step_off[++rs] = rc;
        }
        pyset_free(&V);
        build_vars(&V, clauses, ncl);
    }
    pyset_free(&V);
    for (int c = 0; c < ncl; c++) { pyset_free(clauses[c]); free(clauses[c]); }
    free(clauses);
    if (n_steps) *n_steps = steps;
    return result;
}
