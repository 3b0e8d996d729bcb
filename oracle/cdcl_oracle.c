/*
 * cdcl_oracle.c -- C restatement of the reference's CDCLSolver / cdcl_solve
 * (REF.py:217-384).  TEST INFRASTRUCTURE ONLY: the checker of the GPU CDCL
 * kernel (csrc/cdcl.hip), pinned against tests/golden/cdcl_ref.json (produced
 * by running the reference's own class, tests/golden/make_golden_cdcl.py).
 * The product never links it.
 *
 * Every Python container whose iteration order decides the search is modelled:
 *   watch_list   defaultdict(set): keys in insertion order (dict), each value a
 *                CPython set of clause indices (pyset.c, key idx + 1, hash idx)
 *                -- REF.py:272 iterates the keys, :276 a snapshot of one set;
 *   assignment   dict: insertion stamps (a deleted key re-enters at the end),
 *                the model is returned in that order (REF.py:258, :262);
 *   activity     float64 arithmetic exactly as Python's (REF.py:355-357, :378).
 * The solve loop stops after `max_iter` iterations (REF.py:247 has none; the
 * reference's caller times it out after 60 s, REF.py:417-437).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "pyset.h"

typedef struct {
    int32_t *lits;
    int32_t len;
} cl_t;

typedef struct {
    /* formula (REF.py:221), grows by learned clauses (REF.py:349-350) */
    cl_t *f;
    int64_t nf, capf;
    int maxv;            /* max(abs(l)) over the formula (REF.py:372) */
    /* assignment / levels / antecedents dicts */
    int8_t *val;         /* -1 absent, 0 False, 1 True */
    int64_t *ord;        /* insertion stamp of the assignment key */
    int64_t next_ord;
    int32_t *lev;
    int64_t *ante;       /* -2 absent; else clause index or -1 (REF.py:244, :304) */
    double *act;         /* activity, 0.0 when absent */
    double var_inc, var_decay;
    int32_t level;
    /* watch_list: keys in insertion order, a set per key */
    int32_t *klit;
    pyset *kset;
    int32_t nk, capk;
    int32_t *kidx;       /* literal code -> key index + 1 (0 = absent) */
} cdcl_t;

static inline int lcode(int32_t lit) { return (lit < 0 ? -lit : lit) * 2 + (lit < 0); }
static inline int iabs(int32_t x) { return x < 0 ? -x : x; }

static int key_of(cdcl_t *S, int32_t lit, int create) {
    int k = S->kidx[lcode(lit)];
    if (k || !create) return k - 1;
    if (S->nk == S->capk) {
        S->capk = S->capk ? 2 * S->capk : 16;
        S->klit = (int32_t *)realloc(S->klit, sizeof(int32_t) * (size_t)S->capk);
        S->kset = (pyset *)realloc(S->kset, sizeof(pyset) * (size_t)S->capk);
    }
    S->klit[S->nk] = lit;
    pyset_init(&S->kset[S->nk]);
    S->kidx[lcode(lit)] = ++S->nk;
    return S->nk - 1;
}

static void watch_add(cdcl_t *S, int32_t lit, int64_t idx) {
    const int k = key_of(S, lit, 1);
    pyset_add_hashed(&S->kset[k], idx + 1, idx);
}

static void assign(cdcl_t *S, int v, int value, int32_t level, int64_t ante) {
    if (S->val[v] < 0) S->ord[v] = S->next_ord++;   /* a new dict key goes last */
    S->val[v] = (int8_t)value;
    S->lev[v] = level;
    S->ante[v] = ante;
}

static void append_clause(cdcl_t *S, const int32_t *lits, int32_t len) {
    if (S->nf == S->capf) {
        S->capf = S->capf ? 2 * S->capf : 64;
        S->f = (cl_t *)realloc(S->f, sizeof(cl_t) * (size_t)S->capf);
    }
    S->f[S->nf].lits = (int32_t *)malloc(sizeof(int32_t) * (size_t)(len > 0 ? len : 1));
    memcpy(S->f[S->nf].lits, lits, sizeof(int32_t) * (size_t)len);
    S->f[S->nf].len = len;
    S->nf++;
}

/* REF.py:233-244 */
static void setup_watch_list(cdcl_t *S) {
    for (int64_t i = 0; i < S->nf; ++i) {
        const cl_t *c = &S->f[i];
        if (c->len > 1) {
            watch_add(S, c->lits[0], i);
            watch_add(S, c->lits[1], i);
        } else if (c->len == 1) {
            const int v = iabs(c->lits[0]);
            if (S->val[v] < 0) assign(S, v, c->lits[0] > 0, 0, i);
        }
    }
}

/* REF.py:269-304.  Returns 1 with the conflict clause in (*cl, *cn), else 0. */
static int propagate(cdcl_t *S, int64_t **snap, int64_t *snapcap, int32_t *unitbuf, const int32_t **cl, int32_t *cn) {
    for (;;) {
        int32_t unit = 0;
        const int nk0 = S->nk;   /* list(self.watch_list): keys added during the pass are not visited */
        for (int ki = 0; ki < nk0; ++ki) {
            const int32_t lit = S->klit[ki];
            const int v = iabs(lit);
            if (S->val[v] < 0 || (lit > 0) == S->val[v]) continue;
            pyset *ws = &S->kset[ki];
            if (*snapcap < ws->used + 1) {
                *snapcap = 2 * (ws->used + 1);
                *snap = (int64_t *)realloc(*snap, sizeof(int64_t) * (size_t)*snapcap);
            }
            const int n = pyset_items(ws, *snap);   /* list(self.watch_list[lit]) */
            for (int t = 0; t < n; ++t) {
                const int64_t idx = (*snap)[t] - 1;
                const cl_t *c = &S->f[idx];
                int found = 0;
                for (int j = 0; j < c->len; ++j) {
                    const int32_t o = c->lits[j];
                    if (o == lit) continue;
                    const int ov = iabs(o);
                    if (S->val[ov] < 0 || (o > 0) == S->val[ov]) {
                        pyset_discard_hashed(&S->kset[ki], idx + 1, idx);
                        watch_add(S, o, idx);
                        ws = &S->kset[ki];   /* kset may have moved */
                        found = 1;
                        break;
                    }
                }
                if (!found) {
                    if (c->len == 1) {
                        unit = c->lits[0];
                    } else {
                        *cl = c->lits;
                        *cn = c->len;
                        return 1;
                    }
                }
            }
        }
        if (unit == 0) return 0;
        const int v = iabs(unit);
        if (S->val[v] >= 0) {
            if ((unit > 0) != S->val[v]) {
                unitbuf[0] = unit;
                *cl = unitbuf;
                *cn = 1;
                return 1;
            }
        } else {
            assign(S, v, unit > 0, S->level, -1);
        }
    }
}

static int level_max(const cdcl_t *S, const int32_t *lits, int n, int *second, int *distinct) {
    int mx = -1, sc = -1, d = 0;
    for (int i = 0; i < n; ++i) {
        const int l = S->lev[iabs(lits[i])];
        int seen = 0;
        for (int j = 0; j < i; ++j)
            if (S->lev[iabs(lits[j])] == l) seen = 1;
        if (seen) continue;
        ++d;
        if (l > mx) {
            sc = mx;
            mx = l;
        } else if (l > sc) {
            sc = l;
        }
    }
    *second = sc;
    *distinct = d;
    return mx;
}

static int in_list(const int32_t *a, int n, int32_t x) {
    for (int i = 0; i < n; ++i)
        if (a[i] == x) return 1;
    return 0;
}

/* REF.py:306-345.  Learned literals into *out (len *on), backtrack level into
 * *bt.  Returns -1 where the reference raises KeyError (an unassigned variable
 * in self.levels[...]). */
static int analyze_conflict(cdcl_t *S, const int32_t *conflict, int32_t cn, int32_t **out, int32_t *on,
                            int32_t *bt) {
    int32_t *lits = (int32_t *)malloc(sizeof(int32_t) * (size_t)(cn > 0 ? cn : 1));
    int n = 0;
    for (int i = 0; i < cn; ++i) {
        if (S->val[iabs(conflict[i])] < 0) {
            free(lits);
            return -1;
        }
        lits[n++] = conflict[i];
    }
    int second, distinct;
    int mx = level_max(S, lits, n, &second, &distinct);
    while (distinct > 1) {
        int32_t last = 0;
        for (int i = 0; i < n; ++i)
            if (S->lev[iabs(lits[i])] == mx) {
                last = lits[i];
                break;
            }
        if (last == 0) break;
        const int64_t a = S->ante[iabs(last)];
        if (a < 0) break;   /* None (absent) or -1 */
        const cl_t *ac = &S->f[a];
        int32_t *nl = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n + ac->len + 1));
        int m = 0;
        for (int i = 0; i < n; ++i)
            if (lits[i] != last && !in_list(ac->lits, ac->len, -lits[i])) nl[m++] = lits[i];
        for (int i = 0; i < ac->len; ++i)
            if (ac->lits[i] != -last && !in_list(nl, m, ac->lits[i])) nl[m++] = ac->lits[i];
        free(lits);
        lits = nl;
        n = m;
        for (int i = 0; i < n; ++i)
            if (S->val[iabs(lits[i])] < 0) {
                free(lits);
                return -1;
            }
        mx = level_max(S, lits, n, &second, &distinct);
    }
    *bt = distinct > 1 ? second : 0;
    *out = lits;
    *on = n;
    return 0;
}

/* REF.py:347-357 */
static void learn_clause(cdcl_t *S, const int32_t *c, int32_t n) {
    if (n == 0) return;
    const int64_t idx = S->nf;
    append_clause(S, c, n);
    if (n > 1) {
        watch_add(S, c[0], idx);
        watch_add(S, c[1], idx);
    }
    S->var_inc *= 1.0 / S->var_decay;
    for (int i = 0; i < n; ++i) S->act[iabs(c[i])] += S->var_inc;
}

/* REF.py:359-368 */
static void backtrack(cdcl_t *S, int32_t level) {
    for (int v = 1; v <= S->maxv; ++v)
        if (S->val[v] >= 0 && S->lev[v] > level) {
            S->val[v] = -1;
            S->ante[v] = -2;
        }
    S->level = level;
}

/* REF.py:370-379 */
static int select_variable(cdcl_t *S) {
    int best = 0;
    double bk = 0.0;
    for (int v = 1; v <= S->maxv; ++v) {
        if (S->val[v] >= 0) continue;
        if (best == 0 || S->act[v] > bk) {
            best = v;
            bk = S->act[v];
        }
    }
    if (best == 0) return 0;
    S->var_inc *= S->var_decay;
    return best;
}

/*
 * cdcl_solve(formula) (REF.py:382-384) on CSR clauses.
 * Returns 1 (True), 0 (False), -1 (max_iter iterations of the solve loop
 * passed), -2 (the reference raises: KeyError in analyze_conflict, or
 * max() over no literal in select_variable).  model: the assignment dict as
 * signed literals in its insertion order (*model_len of them, <= nvars) -- the
 * returned model for result 1, else the live dict where the run ended.
 * stats[0..6] = solve-loop iterations, conflicts analysed, decisions, learned
 * clauses, final formula length, watch-list keys, decision level; *var_inc.
 */
int oracle_cdcl(int nclauses, const int32_t *off, const int32_t *lits, int64_t max_iter, int32_t *model,
                int32_t *model_len, int64_t *stats, double *var_inc) {
    cdcl_t S;
    memset(&S, 0, sizeof(S));
    int maxv = 0;
    for (int64_t i = 0; i < (nclauses > 0 ? off[nclauses] : 0); ++i)
        if (iabs(lits[i]) > maxv) maxv = iabs(lits[i]);
    S.maxv = maxv;
    S.val = (int8_t *)malloc((size_t)maxv + 1);
    memset(S.val, -1, (size_t)maxv + 1);
    S.ord = (int64_t *)calloc((size_t)maxv + 1, sizeof(int64_t));
    S.lev = (int32_t *)calloc((size_t)maxv + 1, sizeof(int32_t));
    S.ante = (int64_t *)malloc(sizeof(int64_t) * ((size_t)maxv + 1));
    for (int v = 0; v <= maxv; ++v) S.ante[v] = -2;
    S.act = (double *)calloc((size_t)maxv + 1, sizeof(double));
    S.kidx = (int32_t *)calloc(2 * ((size_t)maxv + 1), sizeof(int32_t));
    S.var_inc = 1.0;
    S.var_decay = 0.95;
    for (int c = 0; c < nclauses; ++c) append_clause(&S, lits + off[c], off[c + 1] - off[c]);
    setup_watch_list(&S);
    int64_t *snap = NULL, snapcap = 0;
    int32_t unitbuf[1];
    int64_t it = 0, conflicts = 0, decisions = 0, learned = 0;
    int result = -1;
    while (max_iter <= 0 || it < max_iter) {
        ++it;
        const int32_t *cl = NULL;
        int32_t cn = 0;
        if (propagate(&S, &snap, &snapcap, unitbuf, &cl, &cn)) {
            if (S.level == 0) {
                result = 0;
                break;
            }
            int32_t *lc = NULL, ln = 0, bt = 0;
            ++conflicts;
            if (analyze_conflict(&S, cl, cn, &lc, &ln, &bt) < 0) {
                result = -2;
                break;
            }
            learn_clause(&S, lc, ln);
            learned += ln > 0;
            free(lc);
            backtrack(&S, bt);
        } else {
            int all = 1;   /* REF.py:257 */
            for (int64_t c = 0; c < S.nf && all; ++c)
                for (int j = 0; j < S.f[c].len; ++j)
                    if (S.val[iabs(S.f[c].lits[j])] < 0) {
                        all = 0;
                        break;
                    }
            if (all) {
                result = 1;
                break;
            }
            const int v = select_variable(&S);
            if (v == 0) {
                result = 1;
                break;
            }
            S.level += 1;
            ++decisions;
            assign(&S, v, 1, S.level, -2);
        }
    }
    int n = 0;
    {
        /* the dict's insertion order: assigned variables by stamp */
        for (int v = 1; v <= maxv; ++v)
            if (S.val[v] >= 0) {
                int k = n++;
                while (k > 0 && S.ord[iabs(model[k - 1])] > S.ord[v]) {
                    model[k] = model[k - 1];
                    --k;
                }
                model[k] = S.val[v] ? v : -v;
            }
    }
    *model_len = n;
    if (stats) {
        stats[0] = it;
        stats[1] = conflicts;
        stats[2] = decisions;
        stats[3] = learned;
        stats[4] = S.nf;
        stats[5] = S.nk;
        stats[6] = S.level;
    }
    if (var_inc) *var_inc = S.var_inc;
    for (int64_t c = 0; c < S.nf; ++c) free(S.f[c].lits);
    for (int k = 0; k < S.nk; ++k) pyset_free(&S.kset[k]);
    free(S.f);
    free(S.klit);
    free(S.kset);
    free(S.kidx);
    free(S.val);
    free(S.ord);
    free(S.lev);
    free(S.ante);
    free(S.act);
    free(snap);
    return result;
}
