/*
 * sat_oracle.c -- CPU restatement of the reference's clause-set solvers.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (sat-mpi-stana-andrei_amd/)
 * links, loads or calls this file.  It is used by tests/ as the checker, by
 * __graft_entry__.smoke() as the checker and by bench.py's cpu_baseline leg.
 *
 * Reference: /root/reference/"comparatie intre algoritmii de rezolvare a seturilor
 * de clauze.py" (called REF.py below).  Each function cites the lines it restates.
 *
 * This is a deliberately *literal* restatement: formulas are explicit clause
 * lists that are copied/filtered exactly like the Python lists in REF.py, the
 * recursion is real recursion, unit clauses are processed one at a time in the
 * order the reference processes them.  The GPU kernels use a very different
 * formulation (assignment-state bitmaps, time-stamped conflict detection, an
 * explicit trail stack), so agreement between the two is meaningful.
 *
 * Pinning: the JSON files in tests/golden hold outputs of the reference functions themselves
 * (run here by tests/golden/make_golden.py, with per-call counters observed via
 * sys.settrace); tests/test_oracle_golden.py checks this file against them.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* formula = list of clauses, clause = list of ints (REF.py:11-13)     */
/* ------------------------------------------------------------------ */
typedef struct {
    int nc;        /* number of clauses                 */
    int *len;      /* len[i]                            */
    int **cl;      /* cl[i] -> literals                 */
    int *pool;     /* owned literal storage             */
} formula;

static formula *f_alloc(int nc, long nlits) {
    formula *f = (formula *)calloc(1, sizeof(formula));
    f->nc = 0;
    f->len = (int *)malloc(sizeof(int) * (size_t)(nc > 0 ? nc : 1));
    f->cl = (int **)malloc(sizeof(int *) * (size_t)(nc > 0 ? nc : 1));
    f->pool = (int *)malloc(sizeof(int) * (size_t)(nlits > 0 ? nlits : 1));
    return f;
}
static void f_free(formula *f) {
    if (!f) return;
    free(f->len); free(f->cl); free(f->pool); free(f);
}
static long f_nlits(const formula *f) {
    long s = 0;
    for (int i = 0; i < f->nc; i++) s += f->len[i];
    return s;
}
static formula *f_copy_append_unit(const formula *f, int unit_lit) {
    long nl = f_nlits(f);
    formula *g = f_alloc(f->nc + 1, nl + 1);
    int *p = g->pool;
    for (int i = 0; i < f->nc; i++) {
        memcpy(p, f->cl[i], sizeof(int) * (size_t)f->len[i]);
        g->cl[g->nc] = p; g->len[g->nc] = f->len[i]; g->nc++;
        p += f->len[i];
    }
    p[0] = unit_lit;
    g->cl[g->nc] = p; g->len[g->nc] = 1; g->nc++;
    return g;
}

/* ------------------------------------------------------------------ */
/* ordered assignment: Dict[int,bool] with insertion order (REF.py:14) */
/* ------------------------------------------------------------------ */
typedef struct {
    int n;               /* entries                          */
    int *order;          /* signed literal per entry, in insertion order */
    signed char *val;    /* val[var] = 0 unassigned, +1 True, -1 False   */
} assign_t;

typedef struct {
    int nvars;
    int mode;            /* 0 = REF semantics, 1 = SOUND (decisions as unit clauses) */
    int64_t max_solutions, node_limit;
    int stop;            /* 1 = max_solutions reached, 2 = node limit */
    int64_t nodes, decisions, unit_props, pure_assigns, conflicts, solutions;
    /* solution output */
    int32_t *sol_lits; int64_t sol_cap_lits, sol_used_lits;
    int64_t *sol_off; int64_t sol_cap, sol_stored;
    /* root assignment after the root's unit_propagate (dict mutated in place) */
    int32_t *root_assign; int *root_len; int root_done;
} dctx;

static assign_t *a_new(int nvars) {
    assign_t *a = (assign_t *)calloc(1, sizeof(assign_t));
    a->order = (int *)malloc(sizeof(int) * (size_t)(nvars + 1));
    a->val = (signed char *)calloc((size_t)nvars + 1, 1);
    return a;
}
static assign_t *a_copy(const assign_t *a, int nvars) {
    assign_t *b = a_new(nvars);
    b->n = a->n;
    memcpy(b->order, a->order, sizeof(int) * (size_t)a->n);
    memcpy(b->val, a->val, (size_t)nvars + 1);
    return b;
}
static void a_free(assign_t *a) {
    if (!a) return;
    free(a->order); free(a->val); free(a);
}
static void a_set(assign_t *a, int lit) {
    int v = lit > 0 ? lit : -lit;
    a->val[v] = lit > 0 ? 1 : -1;
    a->order[a->n++] = lit;
}

static void emit_solution(dctx *c, const assign_t *a) {
    c->solutions++;
    if (c->sol_off && c->sol_stored < c->sol_cap &&
        c->sol_used_lits + a->n <= c->sol_cap_lits) {
        memcpy(c->sol_lits + c->sol_used_lits, a->order, sizeof(int32_t) * (size_t)a->n);
        c->sol_used_lits += a->n;
        c->sol_stored++;
        c->sol_off[c->sol_stored] = c->sol_used_lits;
    }
    if (c->max_solutions > 0 && c->solutions >= c->max_solutions) c->stop = 1;
}

/* unit_propagate, REF.py:139-165.  Returns the (possibly new) formula, or NULL
 * on conflict.  `f_in` is never freed here; a returned formula != f_in is owned
 * by the caller.  `skip_first_count`: SOUND decision children do not count the
 * propagation of the decision literal itself as a unit propagation. */
static formula *unit_propagate(dctx *c, const formula *f_in, assign_t *a, int skip_first_count) {
    const formula *f = f_in;
    formula *owned = NULL;
    int changed = 1;
    int *units = NULL; int ucap = 0;
    while (changed) {
        changed = 0;
        /* unit_clauses = [c for c in f if len(c) == 1]   (REF.py:143) */
        int nu = 0;
        if (ucap < f->nc) { ucap = f->nc + 1; units = (int *)realloc(units, sizeof(int) * (size_t)ucap); }
        for (int i = 0; i < f->nc; i++)
            if (f->len[i] == 1) units[nu++] = f->cl[i][0];
        for (int k = 0; k < nu; k++) {
            int lit = units[k];
            int var = lit > 0 ? lit : -lit;
            int val = lit > 0 ? 1 : -1;
            if (a->val[var] != 0) {                      /* REF.py:149-152 */
                if (a->val[var] != val) { free(units); f_free(owned); return NULL; }
                continue;
            }
            a_set(a, lit);                               /* REF.py:154 */
            if (skip_first_count) skip_first_count = 0; else c->unit_props++;
            changed = 1;
            /* new_f (REF.py:156-164) */
            formula *g = f_alloc(f->nc, f_nlits(f));
            int *p = g->pool;
            for (int i = 0; i < f->nc; i++) {
                const int *ci = f->cl[i];
                int li = f->len[i], has = 0;
                for (int j = 0; j < li; j++) if (ci[j] == lit) { has = 1; break; }
                if (has) continue;
                int n = 0;
                for (int j = 0; j < li; j++) if (ci[j] != -lit) p[n++] = ci[j];
                if (n == 0) { f_free(g); free(units); f_free(owned); return NULL; }
                g->cl[g->nc] = p; g->len[g->nc] = n; g->nc++;
                p += n;
            }
            f_free(owned);
            owned = g; f = g;
        }
    }
    free(units);
    if (!owned) {   /* unchanged: hand back a private copy to keep ownership simple */
        formula *g = f_alloc(f->nc, f_nlits(f));
        int *p = g->pool;
        for (int i = 0; i < f->nc; i++) {
            memcpy(p, f->cl[i], sizeof(int) * (size_t)f->len[i]);
            g->cl[g->nc] = p; g->len[g->nc] = f->len[i]; g->nc++; p += f->len[i];
        }
        owned = g;
    }
    return owned;
}

/* dpll_optimized, REF.py:133-214 (mode 0).  Mode 1 (SOUND) replaces the branch
 * of REF.py:210-213 by a recursion on `formula + [[lit]]` with the assignment
 * copied *without* var, i.e. the decision is applied to the formula as a unit
 * clause and is propagated by REF.py's own unit_propagate. */
static void dpll_node(dctx *c, const formula *F, assign_t *a, int is_decision_child, int is_root) {
    if (c->stop) return;
    c->nodes++;
    if (c->node_limit > 0 && c->nodes > c->node_limit) { c->stop = 2; return; }

    formula *f = unit_propagate(c, F, a, is_decision_child && c->mode == 1);
    if (is_root && c->root_assign) {
        memcpy(c->root_assign, a->order, sizeof(int32_t) * (size_t)a->n);
        *c->root_len = a->n;
    }
    if (!f) { c->conflicts++; return; }                 /* REF.py:168-169 */
    if (f->nc == 0) { emit_solution(c, a); f_free(f); return; }   /* REF.py:170-171 */

    int nv = c->nvars;
    /* literal_sign = defaultdict(set), REF.py:174-179 (dict order = first occurrence) */
    int *order = (int *)malloc(sizeof(int) * (size_t)(nv + 1));
    unsigned char *signs = (unsigned char *)calloc((size_t)nv + 1, 1);   /* bit0 True, bit1 False */
    int *cnt = (int *)calloc((size_t)nv + 1, sizeof(int));
    int norder = 0;
    for (int i = 0; i < f->nc; i++)
        for (int j = 0; j < f->len[i]; j++) {
            int lit = f->cl[i][j], var = lit > 0 ? lit : -lit;
            if (a->val[var] == 0) {
                if (signs[var] == 0) order[norder++] = var;
                signs[var] |= (lit > 0) ? 1 : 2;
                cnt[var]++;
            }
        }
    /* pure_literals, REF.py:181-184 */
    int *pure = (int *)malloc(sizeof(int) * (size_t)(nv + 1));
    int npure = 0;
    for (int k = 0; k < norder; k++) {
        int var = order[k];
        if (signs[var] == 1) pure[npure++] = var;
        else if (signs[var] == 2) pure[npure++] = -var;
    }
    if (npure > 0) {                                     /* REF.py:186-195 */
        assign_t *na = a_copy(a, nv);
        for (int k = 0; k < npure; k++) a_set(na, pure[k]);
        c->pure_assigns += npure;
        /* membership tests against the pure list */
        signed char *ispure = (signed char *)calloc((size_t)nv + 1, 1);
        for (int k = 0; k < npure; k++) ispure[pure[k] > 0 ? pure[k] : -pure[k]] = pure[k] > 0 ? 1 : -1;
        formula *g = f_alloc(f->nc, f_nlits(f));
        int *p = g->pool;
        for (int i = 0; i < f->nc; i++) {
            int drop = 0;
            for (int j = 0; j < f->len[i] && !drop; j++) {
                int lit = f->cl[i][j], var = lit > 0 ? lit : -lit;
                if (ispure[var] == (lit > 0 ? 1 : -1)) drop = 1;      /* lit in pure_literals */
            }
            if (drop) continue;
            int n = 0;
            for (int j = 0; j < f->len[i]; j++) {
                int lit = f->cl[i][j], var = lit > 0 ? lit : -lit;
                if (ispure[var] == (lit > 0 ? -1 : 1)) continue;       /* -lit in pure_literals */
                p[n++] = lit;
            }
            g->cl[g->nc] = p; g->len[g->nc] = n; g->nc++; p += n;
        }
        free(ispure);
        free(order); free(signs); free(cnt); free(pure);
        f_free(f);
        dpll_node(c, g, na, 0, 0);
        f_free(g); a_free(na);
        return;
    }
    free(pure);
    /* var_counts + max(... key=count), REF.py:198-208: first maximal in dict order */
    if (norder == 0) {                                   /* REF.py:205-206 */
        emit_solution(c, a);
        free(order); free(signs); free(cnt); f_free(f);
        return;
    }
    int best = order[0];
    for (int k = 1; k < norder; k++)
        if (cnt[order[k]] > cnt[best]) best = order[k];
    free(order); free(signs); free(cnt);
    for (int t = 0; t < 2 && !c->stop; t++) {            /* for val in [True, False] */
        int lit = t == 0 ? best : -best;
        assign_t *na = a_copy(a, nv);
        c->decisions++;
        if (c->mode == 0) {
            a_set(na, lit);                               /* new_assignment[var] = val */
            dpll_node(c, f, na, 1, 0);
        } else {
            formula *g = f_copy_append_unit(f, lit);
            dpll_node(c, g, na, 1, 0);
            f_free(g);
        }
        a_free(na);
    }
    f_free(f);
}

typedef struct {
    int64_t nodes, decisions, unit_props, pure_assigns, conflicts, solutions;
} oracle_counters;

/* Returns 0 = search complete, 1 = stopped after max_solutions, 2 = node limit. */
int oracle_dpll(int nvars, int nclauses, const int32_t *clause_off, const int32_t *lits,
                int mode, int64_t max_solutions, int64_t node_limit,
                const int32_t *init_assign, int n_init,
                int32_t *sol_lits, int64_t sol_cap_lits, int64_t *sol_off, int64_t sol_cap,
                int32_t *root_assign, int *root_len, oracle_counters *ctr) {
    int nv = nvars;
    for (int i = 0; i < n_init; i++) { int v = init_assign[i] > 0 ? init_assign[i] : -init_assign[i]; if (v > nv) nv = v; }
    for (long i = 0; i < clause_off[nclauses]; i++) { int v = lits[i] > 0 ? lits[i] : -lits[i]; if (v > nv) nv = v; }
    dctx c; memset(&c, 0, sizeof(c));
    c.nvars = nv; c.mode = mode; c.max_solutions = max_solutions; c.node_limit = node_limit;
    c.sol_lits = sol_lits; c.sol_cap_lits = sol_cap_lits; c.sol_off = sol_off; c.sol_cap = sol_cap;
    if (sol_off) sol_off[0] = 0;
    c.root_assign = root_assign; c.root_len = root_len;
    if (root_len) *root_len = 0;

    formula *F = f_alloc(nclauses, clause_off[nclauses]);
    memcpy(F->pool, lits, sizeof(int) * (size_t)clause_off[nclauses]);
    for (int i = 0; i < nclauses; i++) { F->cl[i] = F->pool + clause_off[i]; F->len[i] = clause_off[i + 1] - clause_off[i]; }
    F->nc = nclauses;
    assign_t *a = a_new(nv);
    for (int i = 0; i < n_init; i++) {   /* a caller-supplied dict: later keys overwrite, order kept */
        int lit = init_assign[i], v = lit > 0 ? lit : -lit;
        if (a->val[v] != 0) { a->val[v] = lit > 0 ? 1 : -1;
            for (int k = 0; k < a->n; k++) if ((a->order[k] > 0 ? a->order[k] : -a->order[k]) == v) a->order[k] = lit;
        } else a_set(a, lit);
    }
    dpll_node(&c, F, a, 0, 1);
    a_free(a); f_free(F);
    if (ctr) {
        ctr->nodes = c.nodes; ctr->decisions = c.decisions; ctr->unit_props = c.unit_props;
        ctr->pure_assigns = c.pure_assigns; ctr->conflicts = c.conflicts; ctr->solutions = c.solutions;
    }
    return c.stop;
}
