// dpll.hip -- batched DPLL for gfx950: one instance per wavefront.
//
// Replaces dpll_optimized (REF.py:133-214) for batches of CNF formulas.
//
// Formulation (not the reference's list copying):
//   * The instance (literals as 16-bit codes var<<1|neg, clause offsets) is
//     staged once into the wave's LDS slice; the search never re-reads HBM.
//   * The formula the reference keeps as filtered Python lists is represented
//     implicitly by a per-variable state word vst[v]:
//        bit0 assigned, bit1 value, bit2 "effective", bits3.. batch time + 1.
//     A clause is in the reference's current formula iff none of its literals
//     is true under an *effective* assignment; a literal is still in its clause
//     iff it is not false under an effective assignment.  Unit propagation and
//     pure-literal assignments are effective (they rewrite the formula in
//     REF.py:156-164 / :190-194); in SATMI_MODE_REF a branch assignment is not
//     (REF.py:210-213 never rewrites the formula) and in SATMI_MODE_SOUND it is.
//   * unit_propagate (REF.py:139-165) processes a *snapshot* of unit clauses in
//     clause order, one by one, and returns None at the first emptied clause.
//     Here a round is: a wave-parallel clause scan that (a) finds the clauses
//     emptied by the previous batch and the *time* (batch index) at which each
//     was emptied -- the max time of its falsified literals -- and (b) collects
//     the next snapshot of unit clauses in clause order with ballot/popcount
//     compaction.  The batch itself is applied sequentially (it is short) so the
//     first-come semantics of `if var in a` (REF.py:149-152) hold exactly.  The
//     earliest emptied clause gives the exact stopping point, so assignment
//     counts match the reference one for one.
//   * Pure literals / branching (REF.py:174-208) use one clause-parallel scan
//     with LDS atomics (count, first occurrence, sign set); pure literals are
//     emitted in first-occurrence order through a position bitmap; the branch
//     variable is a 64-bit wave max over (count, -first position), which is the
//     reference's "first maximal key in dict order" tie-break.
//   * Recursion is an explicit frame stack + trail in LDS.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <mutex>
#include <string>
#include <vector>

#include "common.h"

namespace satmi {

constexpr uint32_t VS_ASSIGNED = 1u, VS_VALUE = 2u, VS_EFF = 4u, VS_FLAGS = 7u;
constexpr int VS_TIME_SHIFT = 3;
constexpr uint32_t PHASE_BIT = 0x8000u;

struct DpllLayout {
    uint32_t lit, coff, vst, trail, fvar, ftrail, units, cnt, first, sgn, posbits, bytes;
    int32_t lcap, mcap, ncap;
};

struct DpllArgs {
    const int32_t *inst_clause_begin;
    const int32_t *clause_lit_begin;
    const int32_t *lits;
    const int32_t *inst_nvars;
    const int32_t *init_begin;
    const int32_t *init_lits;
    int32_t num_instances;
    int32_t mode;
    int32_t sol_cap;
    int32_t sol_stride;
    int64_t max_solutions;
    int64_t node_limit;
    uint64_t time_limit_ticks;
    int32_t *status;
    int64_t *counters;
    int32_t *sol_len;
    int32_t *sol_lits;
    int32_t *root_len;
    int32_t *root_lits;
    uint32_t *work_counter;
    DpllLayout lay;
};

struct Lds {
    uint16_t *lit;      // [lcap]   literal codes
    uint16_t *coff;     // [mcap+1] clause offsets into lit
    uint32_t *vst;      // [ncap+1] variable state
    uint16_t *trail;    // [ncap+1] assignment order (literal codes) == dict insertion order
    uint16_t *fvar;     // [ncap+1] decision frames: var | PHASE_BIT once the False branch runs
    uint16_t *ftrail;   // [ncap+1] trail length before the decision
    uint16_t *units;    // [mcap+1] current unit-clause snapshot (literal codes)
    uint32_t *cnt;      // [ncap+1] occurrence counts   (analyze scan)
    uint32_t *first;    // [ncap+1] first occurrence    (analyze scan)
    uint32_t *sgn;      // [ncap+1] sign set bit0 +, bit1 -
    uint64_t *posbits;  // [lcap/64] pure literals by first position
};

struct ScanRes {
    int nu;      // units collected for the next batch
    int e_min;   // earliest batch time at which a clause was emptied (INT_MAX: none)
};

// One unit-propagation scan over all clauses (see header).
__device__ ScanRes scan_round(const Lds &S, int m) {
    const int ln = lane_id();
    const uint64_t lt = lanemask_lt();
    int nu = 0;
    int e_loc = INT_MAX;
    for (int c0 = 0; c0 < m; c0 += 64) {
        const int c = c0 + ln;
        bool unit = false;
        uint32_t ucode = 0;
        if (c < m) {
            const int beg = S.coff[c], end = S.coff[c + 1];
            bool sat = false;
            int alive = 0, emax = -1;
            for (int j = beg; j < end; ++j) {
                const uint32_t code = S.lit[j];
                const uint32_t s = S.vst[code >> 1];
                if (s & VS_EFF) {
                    if (((s >> 1) ^ code) & 1u) {
                        sat = true;   // satisfied (before or during the batch): never empty, never unit
                    } else {
                        emax = max(emax, (int)(s >> VS_TIME_SHIFT) - 1);
                    }
                } else {
                    ++alive;
                    ucode = code;
                }
            }
            if (!sat) {
                if (alive == 0) {
                    if (emax >= 0) e_loc = min(e_loc, emax);
                } else if (alive == 1) {
                    unit = true;
                }
            }
        }
        const uint64_t mk = __ballot(unit);
        if (unit) S.units[nu + __popcll(mk & lt)] = (uint16_t)ucode;
        nu += __popcll(mk);
    }
    wave_sync();
    return {nu, wave_min_i32(e_loc)};
}

// unit_propagate (REF.py:139-165).  Returns true on conflict.  `trail_len` is
// advanced by every assignment made; `*exact_len` receives the trail length at
// the exact point the reference stops (used for the root record).
__device__ bool propagate(const Lds &S, int m, bool has_empty, int &trail_len, int nu, bool do_scan,
                          bool decision_round, int64_t &props, int64_t &rounds, int *exact_len) {
    const int ln = lane_id();
    if (do_scan) {
        ScanRes r = scan_round(S, m);
        ++rounds;
        nu = r.nu;
    }
    bool dec = decision_round;
    // Every round that does not stop assigns at least one new variable, so at
    // most nvars+1 rounds run; `guard` makes that bound structural.
    for (int guard = 0; nu > 0 && guard <= 32768; ++guard) {
        const int round_start = trail_len;
        bool mismatch = false;
        int nassign = 0, first_k = -1;
        for (int k = 0; k < nu; ++k) {
            const uint32_t code = uniform_u32(S.units[k]);
            const uint32_t v = code >> 1;
            const uint32_t want = (code & 1u) ? 0u : VS_VALUE;
            const uint32_t s = uniform_u32(S.vst[v]);
            if (s & VS_ASSIGNED) {
                if ((s & VS_VALUE) != want) { mismatch = true; break; }
                continue;
            }
            if (ln == 0) {
                S.vst[v] = VS_ASSIGNED | VS_EFF | want | ((uint32_t)(k + 1) << VS_TIME_SHIFT);
                S.trail[trail_len] = (uint16_t)code;
            }
            if (first_k < 0) first_k = k;
            ++trail_len;
            ++nassign;
            wave_sync();
        }
        wave_sync();
        if (nassign == 0 && !mismatch) break;   // `changed` stayed False (REF.py:141-142)
        ScanRes r = scan_round(S, m);
        ++rounds;
        int e_min = r.e_min;
        if (has_empty && nassign > 0) e_min = min(e_min, first_k);
        if (e_min != INT_MAX) {
            int cnt = 0;
            for (int i0 = round_start; i0 < trail_len; i0 += 64) {
                const int i = i0 + ln;
                bool p = false;
                if (i < trail_len) {
                    const uint32_t s = S.vst[S.trail[i] >> 1];
                    p = (int)(s >> VS_TIME_SHIFT) - 1 <= e_min;
                }
                cnt += __popcll(__ballot(p));
            }
            props += cnt - (dec ? 1 : 0);
            *exact_len = round_start + cnt;
            return true;
        }
        props += nassign - (dec ? 1 : 0);
        for (int i = round_start + ln; i < trail_len; i += 64) {
            const uint32_t v = S.trail[i] >> 1;
            S.vst[v] &= VS_FLAGS;
        }
        wave_sync();
        if (mismatch) {
            *exact_len = trail_len;
            return true;
        }
        dec = false;
        nu = r.nu;
    }
    *exact_len = trail_len;
    return false;
}

struct AnRes {
    int nactive;
    int npure;
    uint32_t best_var;   // 0 = no unassigned variable occurs (REF.py:205)
};

// literal_sign / pure_literals / var_counts (REF.py:174-208) in one scan.
__device__ AnRes analyze(const Lds &S, int m, int n) {
    const int ln = lane_id();
    for (int v = ln; v <= n; v += 64) {
        S.cnt[v] = 0;
        S.first[v] = 0xFFFFFFFFu;
        S.sgn[v] = 0;
    }
    wave_sync();
    int nactive = 0;
    for (int c0 = 0; c0 < m; c0 += 64) {
        const int c = c0 + ln;
        bool active = false;
        if (c < m) {
            const int beg = S.coff[c], end = S.coff[c + 1];
            active = true;
            for (int j = beg; j < end; ++j) {
                const uint32_t code = S.lit[j];
                const uint32_t s = S.vst[code >> 1];
                if ((s & VS_EFF) && (((s >> 1) ^ code) & 1u)) { active = false; break; }
            }
            if (active) {
                for (int j = beg; j < end; ++j) {
                    const uint32_t code = S.lit[j];
                    const uint32_t v = code >> 1;
                    if (!(S.vst[v] & VS_ASSIGNED)) {
                        atomicAdd(&S.cnt[v], 1u);
                        atomicMin(&S.first[v], (uint32_t)j);
                        atomicOr(&S.sgn[v], 1u << (code & 1u));
                    }
                }
            }
        }
        nactive += __popcll(__ballot(active));
    }
    wave_sync();
    int npure = 0;
    uint64_t best = 0;
    for (int v0 = 1; v0 <= n; v0 += 64) {
        const int v = v0 + ln;
        bool pure = false;
        if (v <= n) {
            const uint32_t c = S.cnt[v];
            if (c > 0) {
                const uint32_t f = S.first[v];
                pure = S.sgn[v] != 3u;
                if (pure) atomicOr((unsigned long long *)&S.posbits[f >> 6], 1ull << (f & 63));
                const uint64_t key = ((uint64_t)c << 32) | (uint64_t)(0xFFFFFFFFu - f);
                best = key > best ? key : best;
            }
        }
        npure += __popcll(__ballot(pure));
    }
    best = wave_max_u64(best);
    wave_sync();
    uint32_t best_var = 0;
    if (best) best_var = uniform_u32(S.lit[0xFFFFFFFFu - (uint32_t)best] >> 1);
    return {nactive, npure, best_var};
}

// Append the pure literals to the trail in first-occurrence order (REF.py:187-189).
__device__ int assign_pures(const Lds &S, int L, int trail_len) {
    const int ln = lane_id();
    const int W = (L + 63) >> 6;
    int base = 0;
    for (int w0 = 0; w0 < W; w0 += 64) {
        const int w = w0 + ln;
        uint64_t bits = w < W ? S.posbits[w] : 0ull;
        const int c = __popcll(bits);
        const int incl = wave_incl_scan(c);
        int pos = trail_len + base + incl - c;
        while (bits) {
            const int bit = __ffsll((unsigned long long)bits) - 1;
            bits &= bits - 1;
            const uint32_t p = (uint32_t)(w * 64 + bit);
            const uint32_t v = S.lit[p] >> 1;
            const bool positive = S.sgn[v] == 1u;
            S.trail[pos++] = (uint16_t)((v << 1) | (positive ? 0u : 1u));
            S.vst[v] = VS_ASSIGNED | VS_EFF | (positive ? VS_VALUE : 0u);
        }
        if (w < W) S.posbits[w] = 0ull;
        base += __shfl(incl, 63, 64);
    }
    wave_sync();
    return trail_len + uniform_i32(base);
}

__device__ void store_assignment(const Lds &S, int trail_len, int32_t *out) {
    for (int i = lane_id(); i < trail_len; i += 64) {
        const uint32_t code = S.trail[i];
        const int v = (int)(code >> 1);
        out[i] = (code & 1u) ? -v : v;
    }
}

enum { ST_PROP_SCAN = 0, ST_PROP_PENDING = 1, ST_ANALYZE = 2, ST_BACKTRACK = 3, ST_DONE = 4 };

__device__ void solve_instance(const DpllArgs &A, const Lds &S, int b) {
    const int ln = lane_id();
    const int cb = A.inst_clause_begin[b], ce = A.inst_clause_begin[b + 1];
    const int m = ce - cb;
    const int lb = A.clause_lit_begin[cb], le = A.clause_lit_begin[ce];
    const int L = le - lb;
    const int n = A.inst_nvars[b];
    const int ib = A.init_begin ? A.init_begin[b] : 0;
    const int nin = A.init_begin ? A.init_begin[b + 1] - ib : 0;
    int64_t *ctr = A.counters + (int64_t)b * SATMI_NCOUNTERS;
    if (m > A.lay.mcap || L > A.lay.lcap || n > A.lay.ncap || n < 0) {
        if (ln < SATMI_NCOUNTERS) ctr[ln] = 0;
        if (ln == 0) {
            A.status[b] = SATMI_DPLL_TOO_LARGE;
            if (A.root_len) A.root_len[b] = 0;
        }
        return;
    }
    // ---- stage the instance into LDS
    for (int i = ln; i < L; i += 64) {
        const int x = A.lits[lb + i];
        const uint32_t v = (uint32_t)(x < 0 ? -x : x);
        S.lit[i] = (uint16_t)((v << 1) | (x < 0 ? 1u : 0u));
    }
    for (int i = ln; i <= m; i += 64) S.coff[i] = (uint16_t)(A.clause_lit_begin[cb + i] - lb);
    for (int v = ln; v <= n; v += 64) S.vst[v] = 0;
    for (int w = ln; w < ((L + 63) >> 6); w += 64) S.posbits[w] = 0ull;
    wave_sync();
    int trail_len = 0;
    if (nin > 0) {   // caller-supplied dict: later keys overwrite the value, keep their slot
        int tl = 0;
        if (ln == 0) {
            for (int i = 0; i < nin; ++i) {
                const int x = A.init_lits[ib + i];
                const uint32_t v = (uint32_t)(x < 0 ? -x : x);
                const uint32_t code = (v << 1) | (x < 0 ? 1u : 0u);
                if (S.vst[v] & VS_ASSIGNED) {
                    for (int t = 0; t < tl; ++t)
                        if ((S.trail[t] >> 1) == v) S.trail[t] = (uint16_t)code;
                } else {
                    S.trail[tl++] = (uint16_t)code;
                }
                S.vst[v] = VS_ASSIGNED | (x > 0 ? VS_VALUE : 0u);
            }
        }
        trail_len = uniform_i32(tl);
        wave_sync();
    }
    bool has_empty = false;
    for (int c0 = 0; c0 < m; c0 += 64) {
        const int c = c0 + ln;
        const bool e = c < m && S.coff[c + 1] == S.coff[c];
        if (__ballot(e)) has_empty = true;
    }

    const bool sound = A.mode == SATMI_MODE_SOUND;
    int64_t nodes = 1, decisions = 0, props = 0, pures = 0, conflicts = 0, sols = 0, rounds = 0;
    int depth = 0, nu = 0;
    int status = SATMI_DPLL_EXHAUSTED;
    bool decision_round = false, at_root = true;
    int state = ST_PROP_SCAN;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();

    while (state != ST_DONE) {
        if (state == ST_PROP_SCAN || state == ST_PROP_PENDING) {
            int exact_len = trail_len;
            const bool conflict = propagate(S, m, has_empty, trail_len, nu, state == ST_PROP_SCAN,
                                            decision_round, props, rounds, &exact_len);
            decision_round = false;
            if (at_root) {
                at_root = false;
                if (A.root_lits) store_assignment(S, exact_len, A.root_lits + (int64_t)b * A.sol_stride);
                if (A.root_len && ln == 0) A.root_len[b] = exact_len;
            }
            if (conflict) {
                ++conflicts;
                state = ST_BACKTRACK;
            } else {
                state = ST_ANALYZE;
            }
            continue;
        }
        if (state == ST_ANALYZE) {
            const AnRes r = analyze(S, m, n);
            bool leaf = false;
            if (r.nactive == 0) {
                leaf = true;                                  // REF.py:170-171
            } else if (r.npure > 0) {                         // REF.py:186-195
                trail_len = assign_pures(S, L, trail_len);
                pures += r.npure;
                ++nodes;                                      // recursive call; its unit_propagate is a no-op
            } else if (r.best_var == 0) {
                leaf = true;                                  // REF.py:205-206
            } else {                                          // REF.py:208-213
                const uint32_t v = r.best_var;
                if (ln == 0) {
                    S.fvar[depth] = (uint16_t)v;
                    S.ftrail[depth] = (uint16_t)trail_len;
                }
                ++depth;
                ++decisions;
                ++nodes;
                const uint32_t code = v << 1;                 // True first
                if (sound) {
                    if (ln == 0) S.units[0] = (uint16_t)code;
                    nu = 1;
                    decision_round = true;
                    state = ST_PROP_PENDING;
                } else {
                    if (ln == 0) {
                        S.vst[v] = VS_ASSIGNED | VS_VALUE;
                        S.trail[trail_len] = (uint16_t)code;
                    }
                    ++trail_len;
                }
                wave_sync();
            }
            if (leaf) {
                if (sols < A.sol_cap) {
                    store_assignment(S, trail_len,
                                     A.sol_lits + ((int64_t)b * A.sol_cap + sols) * A.sol_stride);
                    if (ln == 0) A.sol_len[(int64_t)b * A.sol_cap + sols] = trail_len;
                }
                ++sols;
                if (A.max_solutions > 0 && sols >= A.max_solutions) {
                    status = SATMI_DPLL_STOPPED;
                    state = ST_DONE;
                } else {
                    state = ST_BACKTRACK;
                }
            }
        }
        if (state == ST_BACKTRACK) {
            state = ST_DONE;
            while (depth > 0) {
                const int top = depth - 1;
                const uint32_t fv = uniform_u32(S.fvar[top]);
                const int ft = uniform_i32(S.ftrail[top]);
                for (int i = ft + ln; i < trail_len; i += 64) S.vst[S.trail[i] >> 1] = 0;
                wave_sync();
                trail_len = ft;
                if (!(fv & PHASE_BIT)) {
                    const uint32_t v = fv;
                    if (ln == 0) S.fvar[top] = (uint16_t)(v | PHASE_BIT);
                    ++decisions;
                    ++nodes;
                    const uint32_t code = (v << 1) | 1u;      // False
                    if (sound) {
                        if (ln == 0) S.units[0] = (uint16_t)code;
                        nu = 1;
                        decision_round = true;
                        state = ST_PROP_PENDING;
                    } else {
                        if (ln == 0) {
                            S.vst[v] = VS_ASSIGNED;
                            S.trail[trail_len] = (uint16_t)code;
                        }
                        ++trail_len;
                        state = ST_ANALYZE;
                    }
                    wave_sync();
                    break;
                }
                --depth;
            }
        }
        if (state != ST_DONE) {
            if (A.node_limit > 0 && nodes > A.node_limit) {
                status = SATMI_DPLL_NODE_LIMIT;
                state = ST_DONE;
            } else if (A.time_limit_ticks && __builtin_amdgcn_s_memrealtime() - t0 > A.time_limit_ticks) {
                status = SATMI_DPLL_TIMEOUT;
                state = ST_DONE;
            }
        }
    }
    if (ln == 0) {
        A.status[b] = status;
        ctr[SATMI_CTR_NODES] = nodes;
        ctr[SATMI_CTR_DECISIONS] = decisions;
        ctr[SATMI_CTR_UNIT_PROPS] = props;
        ctr[SATMI_CTR_PURE] = pures;
        ctr[SATMI_CTR_CONFLICTS] = conflicts;
        ctr[SATMI_CTR_SOLUTIONS] = sols;
        ctr[SATMI_CTR_ROUNDS] = rounds;
        ctr[SATMI_CTR_RESERVED] = 0;
    }
}

// Persistent grid: every wave pulls instance indices from a global counter until
// the batch is drained (instances differ wildly in search-tree size).
__global__ void __launch_bounds__(256) dpll_batch_kernel(DpllArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = threadIdx.x >> 6;
    unsigned char *base = smem + (size_t)wave * A.lay.bytes;
    Lds S;
    S.lit = (uint16_t *)(base + A.lay.lit);
    S.coff = (uint16_t *)(base + A.lay.coff);
    S.vst = (uint32_t *)(base + A.lay.vst);
    S.trail = (uint16_t *)(base + A.lay.trail);
    S.fvar = (uint16_t *)(base + A.lay.fvar);
    S.ftrail = (uint16_t *)(base + A.lay.ftrail);
    S.units = (uint16_t *)(base + A.lay.units);
    S.cnt = (uint32_t *)(base + A.lay.cnt);
    S.first = (uint32_t *)(base + A.lay.first);
    S.sgn = (uint32_t *)(base + A.lay.sgn);
    S.posbits = (uint64_t *)(base + A.lay.posbits);
    for (;;) {
        uint32_t b = 0;
        if (lane_id() == 0) b = atomicAdd(A.work_counter, 1u);
        b = uniform_u32(b);
        if (b >= (uint32_t)A.num_instances) break;
        solve_instance(A, S, (int)b);
        wave_sync();
    }
}

// ------------------------------------------------------------------ host side
static uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }

static bool make_layout(int max_vars, int max_clauses, int max_lits, DpllLayout *lay) {
    if (max_vars < 0 || max_clauses < 0 || max_lits < 0) return false;
    if (max_vars > 32767 || max_clauses > 65534 || max_lits > 65535) return false;
    const uint32_t N = (uint32_t)max_vars + 1, M = (uint32_t)max_clauses + 1, Lc = (uint32_t)max_lits + 1;
    uint32_t o = 0;
    lay->lit = o;     o = align16(o + 2 * Lc);
    lay->coff = o;    o = align16(o + 2 * M);
    lay->vst = o;     o = align16(o + 4 * N);
    lay->trail = o;   o = align16(o + 2 * N);
    lay->fvar = o;    o = align16(o + 2 * N);
    lay->ftrail = o;  o = align16(o + 2 * N);
    lay->units = o;   o = align16(o + 2 * M);
    lay->cnt = o;     o = align16(o + 4 * N);
    lay->first = o;   o = align16(o + 4 * N);
    lay->sgn = o;     o = align16(o + 4 * N);
    lay->posbits = o; o = align16(o + 8 * ((Lc + 63) / 64));
    lay->bytes = o;
    lay->lcap = max_lits;
    lay->mcap = max_clauses;
    lay->ncap = max_vars;
    return o <= 160u * 1024u;
}

struct DeviceWork {
    uint32_t *counter = nullptr;
    double ticks_per_s = 1e8;
};
static std::mutex g_work_mu;
static std::vector<DeviceWork> g_work;

static int device_work(DeviceWork **out) {
    int dev = 0;
    SATMI_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_work_mu);
    if ((int)g_work.size() <= dev) g_work.resize(dev + 1);
    DeviceWork &w = g_work[dev];
    if (!w.counter) {
        SATMI_HIP(hipMalloc(&w.counter, 256));
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) == hipSuccess && khz > 0)
            w.ticks_per_s = (double)khz * 1000.0;
    }
    *out = &w;
    return SATMI_OK;
}

}  // namespace satmi

using namespace satmi;

extern "C" uint64_t satmi_dpll_lds_bytes(int max_vars, int max_clauses, int max_lits) {
    DpllLayout lay;
    if (!make_layout(max_vars, max_clauses, max_lits, &lay)) return 0;
    return lay.bytes;
}

extern "C" int satmi_dpll_batch_device(int num_instances, const int32_t *d_inst_clause_begin,
                                       const int32_t *d_clause_lit_begin, const int32_t *d_lits,
                                       const int32_t *d_inst_nvars, int max_vars, int max_clauses,
                                       int max_lits, const int32_t *d_init_begin, const int32_t *d_init_lits,
                                       int mode, int64_t max_solutions, int64_t node_limit,
                                       double time_limit_s, int sol_cap, int sol_stride, int32_t *d_status,
                                       int64_t *d_counters, int32_t *d_sol_len, int32_t *d_sol_lits,
                                       int32_t *d_root_len, int32_t *d_root_lits, void *stream) {
    if (num_instances < 0 || !d_inst_clause_begin || !d_clause_lit_begin || !d_inst_nvars || !d_status ||
        !d_counters) {
        set_error("satmi_dpll_batch_device: bad arguments");
        return SATMI_ERR_ARG;
    }
    if (mode != SATMI_MODE_REF && mode != SATMI_MODE_SOUND) {
        set_error("satmi_dpll_batch_device: mode must be SATMI_MODE_REF or SATMI_MODE_SOUND");
        return SATMI_ERR_ARG;
    }
    if (sol_cap < 0 || (sol_cap > 0 && (!d_sol_len || !d_sol_lits || sol_stride < max_vars))) {
        set_error("satmi_dpll_batch_device: solution buffers too small (sol_stride < max_vars)");
        return SATMI_ERR_ARG;
    }
    if (d_root_lits && sol_stride < max_vars) {
        set_error("satmi_dpll_batch_device: root buffer stride < max_vars");
        return SATMI_ERR_ARG;
    }
    if (num_instances == 0) return SATMI_OK;
    DpllLayout lay;
    if (!make_layout(max_vars, max_clauses, max_lits, &lay)) {
        set_error("satmi_dpll_batch_device: instance too large for the LDS layout (vars <= 32767, "
                  "clauses <= 65534, literals <= 65535, <= 160 KiB per wave)");
        return SATMI_ERR_TOO_LARGE;
    }
    DeviceWork *w = nullptr;
    int rc = device_work(&w);
    if (rc) return rc;
    const int waves_per_wg = lay.bytes * 4 <= 160u * 1024u ? 4 : (lay.bytes * 2 <= 160u * 1024u ? 2 : 1);
    const uint32_t wg_lds = lay.bytes * (uint32_t)waves_per_wg;
    const int wg_per_cu = std::max(1, std::min(8, (int)((160u * 1024u) / wg_lds)));
    int dev = 0, cus = 256;
    SATMI_HIP(hipGetDevice(&dev));
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    const int need = (num_instances + waves_per_wg - 1) / waves_per_wg;
    const int grid = std::max(1, std::min(need, cus * wg_per_cu));

    DpllArgs A;
    A.inst_clause_begin = d_inst_clause_begin;
    A.clause_lit_begin = d_clause_lit_begin;
    A.lits = d_lits;
    A.inst_nvars = d_inst_nvars;
    A.init_begin = d_init_begin;
    A.init_lits = d_init_lits;
    A.num_instances = num_instances;
    A.mode = mode;
    A.sol_cap = sol_cap;
    A.sol_stride = sol_stride;
    A.max_solutions = max_solutions;
    A.node_limit = node_limit;
    A.time_limit_ticks = time_limit_s > 0 ? (uint64_t)(time_limit_s * w->ticks_per_s) : 0;
    A.status = d_status;
    A.counters = d_counters;
    A.sol_len = d_sol_len;
    A.sol_lits = d_sol_lits;
    A.root_len = d_root_len;
    A.root_lits = d_root_lits;
    A.work_counter = w->counter;
    A.lay = lay;

    hipStream_t s = (hipStream_t)stream;
    SATMI_HIP(hipMemsetAsync(w->counter, 0, sizeof(uint32_t), s));
    if (wg_lds > 64u * 1024u)
        SATMI_HIP(hipFuncSetAttribute((const void *)dpll_batch_kernel,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)wg_lds));
    hipLaunchKernelGGL(dpll_batch_kernel, dim3(grid), dim3(64 * waves_per_wg), wg_lds, s, A);
    SATMI_HIP(hipGetLastError());
    return SATMI_OK;
}

extern "C" int satmi_dpll_batch_host(int num_instances, const int32_t *h_inst_clause_begin,
                                     const int32_t *h_clause_lit_begin, const int32_t *h_lits,
                                     const int32_t *h_inst_nvars, const int32_t *h_init_begin,
                                     const int32_t *h_init_lits, int mode, int64_t max_solutions,
                                     int64_t node_limit, double time_limit_s, int sol_cap, int sol_stride,
                                     int32_t *h_status, int64_t *h_counters, int32_t *h_sol_len,
                                     int32_t *h_sol_lits, int32_t *h_root_len, int32_t *h_root_lits) {
    if (num_instances < 0 || !h_inst_clause_begin || !h_clause_lit_begin || !h_inst_nvars) {
        set_error("satmi_dpll_batch_host: bad arguments");
        return SATMI_ERR_ARG;
    }
    if (num_instances == 0) return SATMI_OK;
    const int C = h_inst_clause_begin[num_instances];
    const int Ltot = h_clause_lit_begin[C];
    int max_vars = 0, max_clauses = 0, max_lits = 0;
    for (int b = 0; b < num_instances; ++b) {
        const int cb = h_inst_clause_begin[b], ce = h_inst_clause_begin[b + 1];
        max_clauses = std::max(max_clauses, ce - cb);
        max_lits = std::max(max_lits, h_clause_lit_begin[ce] - h_clause_lit_begin[cb]);
        max_vars = std::max(max_vars, h_inst_nvars[b]);
    }
    const int Itot = h_init_begin ? h_init_begin[num_instances] : 0;
    if (h_init_begin)
        for (int i = 0; i < Itot; ++i) max_vars = std::max(max_vars, std::abs(h_init_lits[i]));
    if (sol_stride < max_vars) {
        set_error("satmi_dpll_batch_host: sol_stride < number of variables");
        return SATMI_ERR_ARG;
    }
    // one allocation for everything
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_icb = 0;
    const size_t o_clb = o_icb + up(4 * (size_t)(num_instances + 1));
    const size_t o_lits = o_clb + up(4 * (size_t)(C + 1));
    const size_t o_nv = o_lits + up(4 * (size_t)std::max(Ltot, 1));
    const size_t o_ib = o_nv + up(4 * (size_t)num_instances);
    const size_t o_il = o_ib + up(4 * (size_t)(num_instances + 1));
    const size_t o_st = o_il + up(4 * (size_t)std::max(Itot, 1));
    const size_t o_ctr = o_st + up(4 * (size_t)num_instances);
    const size_t o_sl = o_ctr + up(8 * (size_t)num_instances * SATMI_NCOUNTERS);
    const size_t o_sol = o_sl + up(4 * (size_t)num_instances * std::max(sol_cap, 1));
    const size_t o_rl = o_sol + up(4 * (size_t)num_instances * std::max(sol_cap, 1) * std::max(sol_stride, 1));
    const size_t o_rlits = o_rl + up(4 * (size_t)num_instances);
    const size_t total = o_rlits + up(4 * (size_t)num_instances * std::max(sol_stride, 1));
    unsigned char *d = nullptr;
    SATMI_HIP(hipMalloc(&d, total));
    int rc = SATMI_OK;
    hipStream_t s = nullptr;
    auto h2d = [&](size_t off, const void *src, size_t bytes) -> int {
        if (bytes) SATMI_HIP(hipMemcpyAsync(d + off, src, bytes, hipMemcpyHostToDevice, s));
        return SATMI_OK;
    };
    auto d2h = [&](void *dst, size_t off, size_t bytes) -> int {
        if (dst && bytes) SATMI_HIP(hipMemcpyAsync(dst, d + off, bytes, hipMemcpyDeviceToHost, s));
        return SATMI_OK;
    };
    do {
        if ((rc = h2d(o_icb, h_inst_clause_begin, 4 * (size_t)(num_instances + 1)))) break;
        if ((rc = h2d(o_clb, h_clause_lit_begin, 4 * (size_t)(C + 1)))) break;
        if ((rc = h2d(o_lits, h_lits, 4 * (size_t)Ltot))) break;
        if ((rc = h2d(o_nv, h_inst_nvars, 4 * (size_t)num_instances))) break;
        if (h_init_begin) {
            if ((rc = h2d(o_ib, h_init_begin, 4 * (size_t)(num_instances + 1)))) break;
            if ((rc = h2d(o_il, h_init_lits, 4 * (size_t)Itot))) break;
        }
        rc = satmi_dpll_batch_device(
            num_instances, (const int32_t *)(d + o_icb), (const int32_t *)(d + o_clb),
            (const int32_t *)(d + o_lits), (const int32_t *)(d + o_nv), max_vars, max_clauses, max_lits,
            h_init_begin ? (const int32_t *)(d + o_ib) : nullptr,
            h_init_begin ? (const int32_t *)(d + o_il) : nullptr, mode, max_solutions, node_limit,
            time_limit_s, sol_cap, sol_stride, (int32_t *)(d + o_st), (int64_t *)(d + o_ctr),
            (int32_t *)(d + o_sl), (int32_t *)(d + o_sol), (int32_t *)(d + o_rl), (int32_t *)(d + o_rlits), s);
        if (rc) break;
        if ((rc = d2h(h_status, o_st, 4 * (size_t)num_instances))) break;
        if ((rc = d2h(h_counters, o_ctr, 8 * (size_t)num_instances * SATMI_NCOUNTERS))) break;
        if (sol_cap > 0) {
            if ((rc = d2h(h_sol_len, o_sl, 4 * (size_t)num_instances * sol_cap))) break;
            if ((rc = d2h(h_sol_lits, o_sol, 4 * (size_t)num_instances * sol_cap * sol_stride))) break;
        }
        if ((rc = d2h(h_root_len, o_rl, 4 * (size_t)num_instances))) break;
        if ((rc = d2h(h_root_lits, o_rlits, 4 * (size_t)num_instances * sol_stride))) break;
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "hipStreamSynchronize");
    } while (0);
    (void)hipFree(d);
    return rc;
}
