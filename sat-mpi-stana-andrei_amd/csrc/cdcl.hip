// cdcl.hip -- the reference's CDCLSolver / cdcl_solve (REF.py:217-384) on gfx950,
// batched: one wavefront per instance, the solver state in a per-wave HBM arena.
//
// The reference's search is decided by the iteration order of its Python
// containers, so the kernel keeps their layouts, not just their contents:
//   * watch_list (defaultdict(set), REF.py:227): the keys in insertion order
//     (klit[]), each value a CPython 3.10 set table of clause indices -- int
//     keys i hash to i, stored as i + 1 (0 = an unused slot, INT32_MIN = a
//     dummy); add / discard / resize follow Objects/setobject.c (set_add_entry,
//     set_discard_entry, set_table_resize, set_insert_clean), so
//     `list(self.watch_list[lit])` (REF.py:276) iterates in the reference's order;
//   * assignment (dict, REF.py:222): a value and an insertion stamp per
//     variable; a deleted key re-enters last (REF.py:362), the model comes out
//     in stamp order (REF.py:258, :262);
//   * activity / var_inc: IEEE double arithmetic in the reference's order
//     (REF.py:355-357, :378), max() keeping the first maximal variable.
// What runs across the wave's 64 lanes (the rest runs on lane 0, every lane
// keeping the same scalar state):
//   * propagate (REF.py:269-304): the tables of all false watch literals are
//     read as one stream in the reference's visiting order, one slot per lane;
//     the replacement watch of every member (its first other literal that is
//     free or true) is found in parallel; the first member without one is the
//     conflict; the removals are dummy marks at known slots (no resize on
//     discard), the adds go in order (they may create keys);
//   * the set tables' adds: each linear-probe run read at once (one lane per
//     slot) and settled by ballots; a resize clears the new table across the
//     lanes and re-inserts against an occupancy bitmap in registers;
//   * the all-assigned test (REF.py:257) over a bitmap of the variables that
//     occur; select_variable's max over activities (REF.py:370-379);
//     backtracking (REF.py:359-368); the model's dict order (a rank per stamp).
// The solve loop (REF.py:247-267) has no bound in the reference (its caller
// kills it after 60 s, REF.py:417-437): here a launch stops an instance after
// max_iter iterations, at its time limit, or when its arena is full.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <mutex>
#include <vector>

#include "common.h"

namespace satmi {
namespace {

constexpr int32_t WS_EMPTY = 0, WS_DUMMY = INT32_MIN;
constexpr int WS_MINSIZE = 8, WS_PROBES = 9, WS_PERTURB = 5;
constexpr int32_t ANTE_ABSENT = -2;
constexpr double VAR_DECAY = 0.95;

enum { CD_FALSE = 0, CD_TRUE = 1, CD_LIMIT = -1, CD_ERROR = -2, CD_FULL = -3 };

// Per-wave arena layout (offsets in bytes), sized on the host for the batch.
struct CdclLayout {
    uint64_t coff, lits, val, ord, lev, ante, act, appears, klit, kidx, woff, wmask, wfill, wused, pool, scratch,
        bytes;
    int64_t clause_cap, lit_cap, pool_cap;
    int32_t ncap;   // variables
    int32_t lcap;   // one learned-literal list in scratch: 2 x variables + the longest clause (repeats)
    // the per-variable and per-key arrays ([val, pool) of the arena) and the
    // learned-literal scratch, in the wave's LDS when they fit (lds_bytes > 0):
    // the lane-0 watch-list adds and conflict analysis are chains of dependent
    // reads of exactly these arrays
    uint32_t lds_bytes, lds_scratch;
};

struct CdclArgs {
    const int32_t *inst_clause_begin, *clause_lit_begin, *lits, *inst_nvars;
    int32_t num_instances;
    int64_t max_iter;
    uint64_t time_limit_ticks;
    int32_t *status, *assign_len, *assign;   // assign: [B x assign_stride] signed literals, dict order
    int32_t assign_stride;
    int64_t *stats;                          // [B x CDCL_NSTATS]
    double *var_inc;                         // [B]
    unsigned char *arena;
    CdclLayout lay;
    uint32_t *work_counter;
};

struct St {   // views into one wave's arena
    int32_t *coff;   // (32-bit offsets and indices: make_cdcl_layout bounds the arena below 2^31 entries)
    int32_t *lits;
    int8_t *val;
    int64_t *ord;
    int32_t *lev;
    int32_t *ante;
    double *act;
    uint64_t *appears;
    int32_t *klit, *kidx;
    int32_t *woff;
    int32_t *wmask, *wfill, *wused;
    int32_t *pool, *scratch;
#ifdef SATMI_CDCL_PHASES
    uint64_t *clk;   // diagnostic build: per-phase shader clocks and counts (lane 0), [7] = last stamp
#endif
};

// Diagnostic build only (make variant VFLAGS=-DSATMI_CDCL_PHASES, read by
// tools/cdcl_probe.py): per-phase clocks of a solve written over stats[4..7]
// (snapshot, replacement watches, watch-list moves, everything between
// propagate calls) and counts over stats[1..3] (moves, snapshot entries, false
// watch lists visited).
#ifdef SATMI_CDCL_PHASES
#define CDCL_CLK(S, i)                                             \
    do {                                                           \
        if (lane_id() == 0) {                                      \
            const uint64_t _t = __builtin_amdgcn_s_memtime();      \
            (S).clk[i] += _t - (S).clk[7];                         \
            (S).clk[7] = _t;                                       \
        }                                                          \
    } while (0)
#else
#define CDCL_CLK(S, i) \
    do {               \
    } while (0)
#endif

__device__ __forceinline__ int iabs(int x) { return x < 0 ? -x : x; }
__device__ __forceinline__ int lcode(int lit) { return (iabs(lit) << 1) | (lit < 0 ? 1 : 0); }

// The solver's scalar state, kept identical on every lane (it changes only in
// wave-uniform code).
struct Seq {
    int64_t nf;        // formula length (clauses)
    int64_t nlits;     // literals stored
    int64_t pool_top;  // set-table pool in use (slots)
    int32_t nk;        // watch-list keys
    int64_t next_ord;
    int32_t level;
    double var_inc;
    bool full;         // the arena ran out
};

// The set-table operations below are wave-uniform: every lane calls them with
// the same arguments and keeps the same Seq (no broadcast needed afterwards);
// the probes read a whole linear-probe run at once (one lane per slot), the
// writes are made by lane 0, a resize clears and rebuilds the table across the
// lanes.
__device__ __forceinline__ bool ws_alloc(const CdclArgs &A, Seq &q, int64_t slots, int64_t *off) {
    if (q.pool_top + slots > A.lay.pool_cap) {
        q.full = true;
        return false;
    }
    *off = q.pool_top;
    q.pool_top += slots;
    return true;
}

// set_insert_clean (lane 0; tables beyond the register bitmap of ws_resize)
__device__ void ws_insert_clean(int32_t *t, uint64_t mask, int32_t key) {
    const uint64_t h = (uint64_t)(int64_t)(key - 1);
    uint64_t perturb = h, i = h & mask;
    for (;;) {
        if (t[i] == WS_EMPTY) {
            t[i] = key;
            return;
        }
        if (i + WS_PROBES <= mask)
            for (int j = 1; j <= WS_PROBES; ++j)
                if (t[i + j] == WS_EMPTY) {
                    t[i + j] = key;
                    return;
                }
        perturb >>= WS_PERTURB;
        i = (i * 5 + 1 + perturb) & mask;
    }
}

constexpr int64_t WS_BITMAP_SLOTS = 64 * 64;   // new tables up to this size: occupancy bits in registers

// set_table_resize(so, minused) (wave-uniform): the new table cleared by all
// lanes, the old members read 64 at a time and re-inserted in slot order
// (set_insert_clean) against an occupancy bitmap held in registers (lane L:
// slots [64L, 64L + 64)), so a probe costs no memory round trip
__device__ void ws_resize(const CdclArgs &A, const St &S, Seq &q, int k, int64_t minused) {
    const int ln = lane_id();
    int64_t newsize = WS_MINSIZE;
    while (newsize <= minused) newsize <<= 1;
    const int32_t mask = S.wmask[k];
    if (newsize == WS_MINSIZE && mask == WS_MINSIZE - 1 && S.wfill[k] == S.wused[k]) return;
    int64_t off;
    if (!ws_alloc(A, q, newsize, &off)) return;
#ifdef SATMI_CDCL_PHASES
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    if (ln == 0) {
        S.clk[10] += 1;
        S.clk[11] += (uint64_t)S.wused[k];
    }
#endif
    int32_t *nt = S.pool + off;
    const int32_t *ot = S.pool + S.woff[k];
    const uint64_t nmask = (uint64_t)(newsize - 1);
    for (int64_t i = ln; i < newsize; i += 64) nt[i] = WS_EMPTY;
    __builtin_amdgcn_s_waitcnt(0);   // the cleared slots land before the keys written over them
    if (newsize <= WS_BITMAP_SLOTS) {
        uint64_t occ = 0;   // this lane's 64 slots of the new table
        for (int i0 = 0; i0 <= mask; i0 += 64) {
            const int32_t x = i0 + ln <= mask ? ot[i0 + ln] : WS_EMPTY;
            for (uint64_t am = __ballot(x != WS_EMPTY && x != WS_DUMMY); am; am &= am - 1) {
                const int32_t key = __builtin_amdgcn_readlane(x, __builtin_ctzll(am));
                const uint64_t h = (uint64_t)(int64_t)(key - 1);
                uint64_t perturb = h, i = h & nmask, at;
                for (;;) {
                    // bits i .. i + WS_PROBES (a run never passes the table's end)
                    const int w = (int)(i >> 6), sh = (int)(i & 63);
                    const uint64_t lo = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)occ, w) |
                                        ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(occ >> 32), w) << 32);
                    uint64_t run = ~lo >> sh;   // free slots from i on
                    if (sh > 0 && w + 1 < 64) {
                        const uint64_t hi =
                            (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)occ, w + 1) |
                            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(occ >> 32), w + 1) << 32);
                        run |= ~hi << (64 - sh);
                    }
                    const int len = i + WS_PROBES <= nmask ? WS_PROBES + 1 : 1;
                    run &= (len == 64 ? ~0ull : (1ull << len) - 1);
                    if (run) {
                        at = i + (uint64_t)__builtin_ctzll(run);
                        break;
                    }
                    perturb >>= WS_PERTURB;
                    i = (i * 5 + 1 + perturb) & nmask;
                }
                if (ln == (int)(at >> 6)) occ |= 1ull << (at & 63);
                if (ln == 0) nt[at] = key;
            }
        }
    } else if (ln == 0) {
        for (int64_t i = 0; i <= mask; ++i)
            if (ot[i] != WS_EMPTY && ot[i] != WS_DUMMY) ws_insert_clean(nt, nmask, ot[i]);
    }
    if (ln == 0) {
        S.woff[k] = (int32_t)off;
        S.wmask[k] = (int32_t)nmask;
        S.wfill[k] = S.wused[k];
    }
    wave_sync();
#ifdef SATMI_CDCL_PHASES
    if (ln == 0) S.clk[9] += __builtin_amdgcn_s_memtime() - t0;
#endif
}

// set_add_entry(so, key, hash = key - 1) (wave-uniform): each linear-probe run
// (the slot and the WS_PROBES after it, when they fit) is read at once, one
// lane per slot, and settled by ballots in probe order: the first empty slot
// or the key itself ends the search; CPython 3.10 keeps the LAST dummy probed
// before it as the slot to reuse
__device__ void ws_add(const CdclArgs &A, const St &S, Seq &q, int k, int32_t key) {
    const int ln = lane_id();
    const int64_t h = (int64_t)(key - 1);
    int32_t *t = S.pool + S.woff[k];
    const uint64_t mask = (uint64_t)S.wmask[k];
    uint64_t i = (uint64_t)h & mask, perturb = (uint64_t)h;
    int64_t freeslot = -1, slot;
    for (;;) {
        const int probes = i + WS_PROBES <= mask ? WS_PROBES : 0;
        const bool in = ln <= probes;
        const int32_t x = in ? t[i + ln] : 0;
        const uint64_t em = __ballot(in && x == WS_EMPTY), km = __ballot(in && x == key),
                       dm = __ballot(in && x == WS_DUMMY);
        const uint64_t stop = em | km;
        const uint64_t before = stop ? (1ull << __builtin_ctzll(stop)) - 1 : ~0ull;
        if (dm & before) freeslot = (int64_t)(i + 63 - __builtin_clzll(dm & before));
        if (stop) {
            if (km & (stop & (0 - stop))) return;   // already a member
            slot = (int64_t)(i + __builtin_ctzll(stop));
            break;
        }
        perturb >>= WS_PERTURB;
        i = (i * 5 + 1 + perturb) & mask;
    }
    if (freeslot >= 0) {   // found_unused_or_dummy with a dummy on the way
        if (ln == 0) {
            S.wused[k]++;
            t[freeslot] = key;
        }
        wave_sync();
        return;
    }
    const int32_t fill = S.wfill[k] + 1, used = S.wused[k] + 1;
    if (ln == 0) {
        S.wfill[k] = fill;
        S.wused[k] = used;
        t[slot] = key;
    }
    wave_sync();
    if ((uint64_t)fill * 5 < mask * 3) return;
    ws_resize(A, S, q, k, used > 50000 ? (int64_t)used * 2 : (int64_t)used * 4);
}

// self.watch_list[lit] (defaultdict: a missing key is created with an empty set)
__device__ int key_of(const CdclArgs &A, const St &S, Seq &q, int lit) {
    const int ln = lane_id();
    const int c = lcode(lit);
    int k = S.kidx[c] - 1;
    if (k >= 0) return k;
    int64_t off;
    if (!ws_alloc(A, q, WS_MINSIZE, &off)) return -1;
    k = q.nk++;
    if (ln == 0) {
        S.klit[k] = lit;
        S.kidx[c] = k + 1;
        S.woff[k] = (int32_t)off;
        S.wmask[k] = WS_MINSIZE - 1;
        S.wfill[k] = S.wused[k] = 0;
    }
    if (ln < WS_MINSIZE) S.pool[off + ln] = WS_EMPTY;
    wave_sync();
    return k;
}

// self.watch_list[lit].add(idx) (wave-uniform)
__device__ void watch_add(const CdclArgs &A, const St &S, Seq &q, int lit, int64_t idx) {
#ifdef SATMI_CDCL_PHASES
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
    lit = __builtin_amdgcn_readfirstlane(lit);
    const int32_t key = __builtin_amdgcn_readfirstlane((int32_t)(idx + 1));
    const int k = key_of(A, S, q, lit);
    if (k >= 0 && !q.full) ws_add(A, S, q, k, key);
#ifdef SATMI_CDCL_PHASES
    if (lane_id() == 0) {
        S.clk[8] += __builtin_amdgcn_s_memtime() - t0;
        S.clk[12] += 1;
    }
#endif
}

__device__ __forceinline__ bool lit_false(const St &S, int lit) {
    const int8_t v = S.val[iabs(lit)];
    return v >= 0 && (lit > 0) != (v != 0);
}

// propagate (REF.py:269-304): returns the conflict clause's index, -1 for none.
// (The reference's unit branch, REF.py:290-291 / :297-304, needs a watched
// clause of length 1; watched clauses are longer than 1 (REF.py:235, :351),
// so its pass ends either at a conflict or with `unit is None`.)
//
// Nothing the pass does changes what it reads: it assigns nothing, a
// replacement watch is never a false literal (so every add goes to the table
// of a literal the pass does not visit) and a removal only marks a slot of the
// visited table itself.  So the tables of all false watch literals are read as
// ONE stream -- keys in dict order, each table in slot order, which is the
// order REF.py:274-276 visits them -- in windows of up to 256 slots; every
// member of a window looks for its replacement watch at the same time; the
// first member without one (stream order) is the conflict (REF.py:292-293),
// and the members before it move: dummies at their slots, the adds in stream
// order (they may create keys and resize tables).  A launch's long
// solves are latency-bound chains of dependent memory reads, and one window
// covers the false lists of a typical pass at once.
// a member's first literals read at once (the menu formulas' clauses and their
// learned copies have 3; longer clauses read the rest one at a time): 3 measured
// +5 % over 4 (profiles/r05/steps/cdcl_owner_scan_ab.txt)
#ifndef CDCL_LITS_AHEAD
#define CDCL_LITS_AHEAD 3
#endif
#ifndef CDCL_WCH
#define CDCL_WCH 4          // 64-slot chunks per propagate window (reads in flight)
#endif
// own8 holds one window of 64 * 4 slots (cleared as 64 words) and the conflict
// scan's "none" sentinel is chunk 4: a wider window would overrun both
static_assert(CDCL_WCH >= 1 && CDCL_WCH <= 4, "CDCL_WCH: 1..4 chunks per propagate window");

__device__ int64_t propagate(const CdclArgs &A, const St &S, Seq &q) {
    __shared__ __attribute__((aligned(4))) uint8_t own8[256];   // window slot -> owning key lane (one-wave groups)
    const int ln = lane_id();
    CDCL_CLK(S, 3);
    const int nk0 = q.nk;   // list(self.watch_list): keys created during the pass are not visited
    for (int k0 = 0; k0 < nk0; k0 += 64) {
        const int kk = k0 + ln;
        const bool fl = kk < nk0 && lit_false(S, S.klit[kk]);
        const int size = fl ? S.wmask[kk] + 1 : 0;
        const int incl = wave_incl_scan(size);
        const int total = lane63(incl), excl = incl - size;
#ifdef SATMI_CDCL_PHASES
        const uint64_t fm = __ballot(fl);
        if (ln == 0) S.clk[6] += (uint64_t)__popcll(fm);
#endif
        for (int g0 = 0, nch; g0 < total; g0 += 64 * nch) {
            nch = min(CDCL_WCH, (total - g0 + 63) >> 6);   // one window when the stream fits 256 slots
            // the stream slot g of (u, lane): its key (the last false key whose
            // table starts at or before g) and the slot in that table.  Each
            // false key marks its table's first slot in an LDS byte map of the
            // window; a prefix max over the slots carries every mark to the
            // slots after it (tables come in key order, so the latest mark is
            // the owner) -- no serial loop over the false keys
            ((uint32_t *)own8)[ln] = 0xFFFFFFFFu;   // the window's 256 bytes: no mark
            if (fl && excl >= g0 && excl < g0 + 64 * nch) own8[excl - g0] = (uint8_t)ln;
            const uint64_t before = __ballot(fl && excl < g0);   // keys whose tables began in earlier windows
            int carry = before ? 63 - __builtin_clzll(before) : -1;
            int own[CDCL_WCH], ex[CDCL_WCH];
#pragma unroll
            for (int u = 0; u < CDCL_WCH; ++u) {
                own[u] = ex[u] = 0;
                if (u < nch) {
                    const int m8 = own8[64 * u + ln];
                    const int o = wave_incl_max(max(m8 == 0xFF ? -1 : m8, carry));
                    carry = __builtin_amdgcn_readlane(o, 63);
                    own[u] = max(o, 0);
                    ex[u] = __builtin_amdgcn_ds_bpermute(own[u] << 2, excl);
                }
            }
            int32_t x[CDCL_WCH], lit[CDCL_WCH];
            int at[CDCL_WCH];
#pragma unroll
            for (int u = 0; u < CDCL_WCH; ++u) {   // up to four table reads in flight
                const int g = g0 + 64 * u + ln;
                const bool in = u < nch && g < total;
                const int k = k0 + own[u];
                at[u] = in ? S.woff[k] + (g - ex[u]) : 0;
                lit[u] = in ? S.klit[k] : 0;
                x[u] = in ? S.pool[at[u]] : WS_EMPTY;
            }
            bool act[CDCL_WCH];
            int jb[CDCL_WCH], je[CDCL_WCH];
#pragma unroll
            for (int u = 0; u < CDCL_WCH; ++u) {
                act[u] = x[u] != WS_EMPTY && x[u] != WS_DUMMY;
                jb[u] = act[u] ? S.coff[x[u] - 1] : 0;
                je[u] = act[u] ? S.coff[x[u]] : 0;
            }
            CDCL_CLK(S, 0);
            // replacement watch: the clause's first literal other than lit that
            // is free or true (REF.py:279-286); the first CDCL_LITS_AHEAD of
            // every member are read together
            int r[CDCL_WCH];
            int o[CDCL_WCH][CDCL_LITS_AHEAD];
#pragma unroll
            for (int u = 0; u < CDCL_WCH; ++u)
#pragma unroll
                for (int t = 0; t < CDCL_LITS_AHEAD; ++t) o[u][t] = jb[u] + t < je[u] ? S.lits[jb[u] + t] : lit[u];
#pragma unroll
            for (int u = 0; u < CDCL_WCH; ++u) {
                r[u] = 0;
#pragma unroll
                for (int t = 0; t < CDCL_LITS_AHEAD; ++t) {
                    const int ot = o[u][t];
                    const int8_t v = S.val[iabs(ot)];
                    r[u] = (r[u] == 0 && ot != lit[u] && (v < 0 || (ot > 0) == (v != 0))) ? ot : r[u];
                }
                if (act[u] && r[u] == 0) {   // longer clauses: the rest one literal at a time
                    for (int j = jb[u] + CDCL_LITS_AHEAD; j < je[u]; ++j) {
                        const int ot = S.lits[j];
                        if (ot == lit[u]) continue;
                        const int8_t v = S.val[iabs(ot)];
                        if (v < 0 || (ot > 0) == (v != 0)) {
                            r[u] = ot;
                            break;
                        }
                    }
                }
            }
            // the first member without a replacement, in stream order (u, lane)
            int cu = 4, cl = 64;
            int64_t conflict = -1;
#pragma unroll
            for (int u = 0; u < CDCL_WCH; ++u) {
                const uint64_t nm = __ballot(act[u] && r[u] == 0);
                if (cu == 4 && nm) {
                    cu = u;
                    cl = __builtin_ctzll(nm);
                    conflict = (int64_t)__builtin_amdgcn_readlane(x[u], cl) - 1;
                }
            }
            CDCL_CLK(S, 1);
            // the moves: self.watch_list[lit].remove(idx) (a dummy at its slot),
            // self.watch_list[other_lit].add(idx) in stream order
#ifdef SATMI_CDCL_PHASES
            int nmv = 0;
#endif
#pragma unroll
            for (int u = 0; u < CDCL_WCH; ++u) {
                const bool mv = act[u] && r[u] != 0 && (u < cu || (u == cu && ln < cl));
                if (mv) S.pool[at[u]] = WS_DUMMY;
                uint64_t mm = __ballot(mv);
#ifdef SATMI_CDCL_PHASES
                nmv += __popcll(mm);
#endif
                for (; mm; mm &= mm - 1) {
                    const int l = __builtin_ctzll(mm);
                    const int rl = __builtin_amdgcn_readlane(r[u], l);
                    const int cx = __builtin_amdgcn_readlane(x[u], l);
                    const int kl = k0 + __builtin_amdgcn_readlane(own[u], l);
                    if (ln == 0) S.wused[kl] -= 1;
                    if (!q.full) watch_add(A, S, q, rl, (int64_t)cx - 1);
                }
            }
#ifdef SATMI_CDCL_PHASES
            {   // diagnostic counts: moves, members read
                int na = 0;
#pragma unroll
                for (int u = 0; u < CDCL_WCH; ++u) na += __popcll(__ballot(act[u]));
                if (ln == 0) {
                    S.clk[4] += (uint64_t)nmv;
                    S.clk[5] += (uint64_t)na;
                }
            }
#endif
            wave_sync();
            CDCL_CLK(S, 2);
            if (conflict >= 0 || q.full) return conflict;
        }
    }
    return -1;
}

// analyze_conflict (REF.py:306-345) across the wave: learned literals into
// S.scratch (returns their count, the same on every lane), the backtrack level
// into *bt; -1 where the reference raises KeyError (an unassigned variable
// reaching self.levels[...]); -2 if a list would pass `cap` entries (the arena
// is full: CD_FULL).  A list holds distinct literals plus the repeats of the
// conflict clause, so cap = 2 x variables + the longest clause is never
// reached.  Each resolution step keeps REF.py's list order: the kept literals
// in order, then the antecedent's literals in order that are not -last_lit,
// not among the kept ones and not a repeat of an earlier antecedent literal
// (a repeat is excluded exactly when its first occurrence was: same value,
// same tests) -- every membership test runs on the lanes in parallel.
__device__ int analyze_conflict(const St &S, int64_t conflict, int32_t cap, int32_t *bt) {
    const int ln = lane_id();
    const uint64_t lt = lanemask_lt();
    const int jb = S.coff[conflict], je = S.coff[conflict + 1];
    if (je - jb > cap) return -2;
    int32_t *L = S.scratch, *N = S.scratch + cap;
    int n = (int)(je - jb);
    bool bad = false;
    for (int i = ln; i < n; i += 64) {
        const int x = S.lits[jb + i];
        bad |= S.val[iabs(x)] < 0;
        L[i] = x;
    }
    if (__ballot(bad)) return -1;
    wave_sync();
    for (;;) {
        // max(levels) and max(levels - {max}) (-1: one level)
        int mx = -1;
        for (int i = ln; i < n; i += 64) mx = max(mx, S.lev[iabs(L[i])]);
        mx = wave_max_i32(mx);
        int sc = -1;
        for (int i = ln; i < n; i += 64) {
            const int l = S.lev[iabs(L[i])];
            if (l < mx) sc = max(sc, l);
        }
        sc = wave_max_i32(sc);
        if (sc < 0) {   // len(levels) <= 1
            *bt = 0;
            return n;
        }
        // the first literal at the maximal level
        int last = 0;
        for (int i0 = 0; i0 < n; i0 += 64) {
            const int i = i0 + ln;
            const uint64_t m = __ballot(i < n && S.lev[iabs(L[i < n ? i : 0])] == mx);
            if (m) {
                last = L[i0 + __builtin_ctzll(m)];
                break;
            }
        }
        const int a = S.ante[iabs(last)];
        if (a < 0) {   // None or -1
            *bt = sc;
            return n;
        }
        // resolve with the antecedent (REF.py:331-342): new list at scratch + cap
        const int ab = S.coff[a], ae = S.coff[a + 1];
        const int alen = (int)(ae - ab);
        int m = 0;
        for (int i0 = 0; i0 < n; i0 += 64) {   // kept literals, in order (m <= n <= cap)
            const int i = i0 + ln;
            const int x = i < n ? L[i] : 0;
            bool neg_in = false;
            for (int j = 0; j < alen; ++j) neg_in |= S.lits[ab + j] == -x;
            const bool keep = i < n && x != last && !neg_in;
            const uint64_t km = __ballot(keep);
            if (keep) N[m + __popcll(km & lt)] = x;
            m += __popcll(km);
        }
        wave_sync();
        const int m1 = m;
        for (int j0 = 0; j0 < alen; j0 += 64) {   // then the antecedent's new literals, in order
            const int j = j0 + ln;
            const int x = j < alen ? S.lits[ab + j] : 0;
            bool inc = j < alen && x != -last;
            for (int k = 0; k < m1; ++k) inc &= N[k] != x;
            const int kend = min(alen, j0 + 64);
            for (int k = 0; k < kend; ++k) inc &= !(k < j && S.lits[ab + k] == x);
            const uint64_t im = __ballot(inc);
            if (m + __popcll(im) > cap) return -2;
            if (inc) N[m + __popcll(im & lt)] = x;
            m += __popcll(im);
        }
        wave_sync();
        bad = false;
        for (int i = ln; i < m; i += 64) {
            const int x = N[i];
            bad |= S.val[iabs(x)] < 0;
            L[i] = x;
        }
        if (__ballot(bad)) return -1;
        wave_sync();
        n = m;
    }
}

__device__ void solve_one(const CdclArgs &A, const St &S, int b) {
    const int ln = lane_id();
    const int cb = A.inst_clause_begin[b], ce = A.inst_clause_begin[b + 1];
    const int m = ce - cb;
    const int lb = A.clause_lit_begin[cb], le = A.clause_lit_begin[ce];
    const int n = A.inst_nvars[b];
    int64_t *st = A.stats + (int64_t)b * SATMI_CDCL_NSTATS;
    int status = CD_LIMIT;
    if (m > A.lay.clause_cap || (le - lb) > A.lay.lit_cap || n > A.lay.ncap) {
        status = CD_FULL;
        if (ln == 0) {
            A.status[b] = status;
            A.assign_len[b] = 0;
            for (int i = 0; i < SATMI_CDCL_NSTATS; ++i) st[i] = 0;
            A.var_inc[b] = 1.0;
        }
        return;
    }
    // ---- stage: formula, empty dicts
    for (int i = ln; i <= m; i += 64) S.coff[i] = A.clause_lit_begin[cb + i] - lb;
    for (int i = ln; i < le - lb; i += 64) S.lits[i] = A.lits[lb + i];
    for (int v = ln; v <= n; v += 64) {
        S.val[v] = -1;
        S.ante[v] = ANTE_ABSENT;
        S.act[v] = 0.0;
        S.lev[v] = 0;
        S.ord[v] = 0;
        S.kidx[2 * v] = S.kidx[2 * v + 1] = 0;
    }
    for (int w = ln; w <= (n >> 6); w += 64) S.appears[w] = 0ull;
    wave_sync();
    for (int i = ln; i < le - lb; i += 64) {
        const int v = iabs(S.lits[i]);
        atomicOr((unsigned long long *)&S.appears[v >> 6], 1ull << (v & 63));
    }
    wave_sync();
    Seq q;
    q.nf = m;
    q.nlits = le - lb;
    q.pool_top = 0;
    q.nk = 0;
    q.next_ord = 0;
    q.level = 0;
    q.var_inc = 1.0;
    q.full = false;
    // setup_watch_list (REF.py:233-244), wave-uniform
    for (int64_t i = 0; i < m && !q.full; ++i) {
        const int jb = S.coff[i], len = S.coff[i + 1] - jb;
        if (len > 1) {
            watch_add(A, S, q, S.lits[jb], i);
            watch_add(A, S, q, S.lits[jb + 1], i);
        } else if (len == 1) {
            const int x = S.lits[jb], v = iabs(x);
            if (S.val[v] < 0) {
                if (ln == 0) {
                    S.val[v] = x > 0;
                    S.ord[v] = q.next_ord;
                    S.lev[v] = 0;
                    S.ante[v] = (int32_t)i;
                }
                ++q.next_ord;
            }
            wave_sync();
        }
    }
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
#ifdef SATMI_CDCL_PHASES
    if (ln == 0) {
        for (int i = 0; i < 16; ++i) S.clk[i] = 0;
        S.clk[7] = __builtin_amdgcn_s_memtime();
    }
#endif
    int64_t it = 0, conflicts = 0, decisions = 0, learned = 0;
    while (!q.full) {
        if (A.max_iter > 0 && it >= A.max_iter) break;
        if (A.time_limit_ticks && __builtin_amdgcn_s_memrealtime() - t0 > A.time_limit_ticks) break;
        ++it;
        const int64_t conflict = propagate(A, S, q);
        if (q.full) break;
        if (conflict >= 0) {
            if (q.level == 0) {
                status = CD_FALSE;
                break;
            }
            ++conflicts;
            int32_t bt = 0;
            int32_t cnt = analyze_conflict(S, conflict, A.lay.lcap, &bt);   // the whole wave
            cnt = __builtin_amdgcn_readfirstlane(cnt);
            bt = __builtin_amdgcn_readfirstlane(bt);
            CDCL_CLK(S, 13);
            if (cnt > 0) {   // learn_clause (REF.py:347-357), wave-uniform
                if (q.nf + 1 > A.lay.clause_cap || q.nlits + cnt > A.lay.lit_cap) {
                    q.full = true;
                } else {
                    const int64_t idx = q.nf;
                    for (int i = ln; i < cnt; i += 64) S.lits[q.nlits + i] = S.scratch[i];
                    q.nlits += cnt;
                    if (ln == 0) S.coff[idx + 1] = (int32_t)q.nlits;
                    q.nf = idx + 1;
                    if (cnt > 1) {
                        watch_add(A, S, q, S.scratch[0], idx);
                        watch_add(A, S, q, S.scratch[1], idx);
                    }
                    q.var_inc *= 1.0 / VAR_DECAY;
                    if (cnt <= 64) {
                        // a variable's increments in list order by the lane of its
                        // first occurrence (a repeated variable adds var_inc once
                        // per occurrence, REF.py:356-357)
                        const int v = ln < cnt ? iabs(S.scratch[ln]) : -1;
                        bool dup = false;
                        int mult = 0;
                        for (int j = 0; j < cnt; ++j) {
                            const int vj = __builtin_amdgcn_readlane(v, j);
                            dup |= j < ln && vj == v;
                            mult += vj == v ? 1 : 0;
                        }
                        if (ln < cnt && !dup) {
                            double a = S.act[v];
                            for (int t = 0; t < mult; ++t) a += q.var_inc;
                            S.act[v] = a;
                        }
                    } else if (ln == 0) {
                        for (int i = 0; i < cnt; ++i) S.act[iabs(S.scratch[i])] += q.var_inc;
                    }
                    wave_sync();
                }
            }
            CDCL_CLK(S, 14);
            if (cnt == -2) q.full = true;   // scratch list bound (see analyze_conflict)
            else if (cnt < 0) {
                status = CD_ERROR;
                break;
            }
            if (q.full) break;
            learned += cnt > 0 ? 1 : 0;
            // backtrack (REF.py:359-368)
            for (int v = 1 + ln; v <= n; v += 64)
                if (S.val[v] >= 0 && S.lev[v] > bt) {
                    S.val[v] = -1;
                    S.ante[v] = ANTE_ABSENT;
                }
            q.level = bt;
            wave_sync();
        } else {
            // all(abs(l) in self.assignment ...) (REF.py:257)
            bool miss = false;
            for (int v = 1 + ln; v <= n; v += 64)
                miss |= ((S.appears[v >> 6] >> (v & 63)) & 1ull) && S.val[v] < 0;
            if (!__ballot(miss)) {
                status = CD_TRUE;
                break;
            }
            // select_variable (REF.py:370-379): the first unassigned variable of
            // maximal activity among 1..max(abs(l)); n is that maximum
            // (activities are sums of positive increments: >= 0, possibly
            // +inf, never NaN, so their IEEE bit patterns order as unsigned
            // integers; three DPP reductions: high word, low word, first variable)
            uint64_t best = 0;
            int bv = INT_MAX;
            for (int v = 1 + ln; v <= n; v += 64)
                if (S.val[v] < 0) {
                    const uint64_t a = (uint64_t)__double_as_longlong(S.act[v]);
                    if (bv == INT_MAX || a > best) {
                        best = a;
                        bv = v;
                    }
                }
            const bool has = bv != INT_MAX;
            const uint32_t bh = (uint32_t)(best >> 32), bl = (uint32_t)best;
            const uint32_t mh = wave_max_u32(has ? bh : 0u);
            const bool on_h = has && bh == mh;
            const uint32_t ml = wave_max_u32(on_h ? bl : 0u);
            bv = wave_min_i32(on_h && bl == ml ? bv : INT_MAX);
            if (bv == INT_MAX) {   // no unassigned variable: True (REF.py:261-262)
                status = CD_TRUE;
                break;
            }
            q.var_inc *= VAR_DECAY;
            q.level += 1;
            ++decisions;
            if (ln == 0) {
                S.val[bv] = 1;
                S.ord[bv] = q.next_ord;
                S.lev[bv] = q.level;
                S.ante[bv] = ANTE_ABSENT;
            }
            ++q.next_ord;
            wave_sync();
        }
    }
    if (q.full) status = CD_FULL;
    // the assignment dict in insertion order: rank every assigned variable by stamp
    int na = 0;
    for (int v = 1 + ln; v <= n; v += 64) na += S.val[v] >= 0 ? 1 : 0;
    for (int off = 32; off >= 1; off >>= 1) na += __shfl_xor(na, off, 64);
    int32_t *out = A.assign + (int64_t)b * A.assign_stride;
    for (int v = 1 + ln; v <= n; v += 64) {
        if (S.val[v] < 0) continue;
        int r = 0;
        for (int u = 1; u <= n; ++u) r += (S.val[u] >= 0 && S.ord[u] < S.ord[v]) ? 1 : 0;
        if (r < A.assign_stride) out[r] = S.val[v] ? v : -v;
    }
    if (ln == 0) {
        A.status[b] = status;
        A.assign_len[b] = min(na, A.assign_stride);
        st[0] = it;
        st[1] = conflicts;
        st[2] = decisions;
        st[3] = learned;
        st[4] = q.nf;
        st[5] = q.nk;
        st[6] = q.level;
        st[7] = q.pool_top;
#ifdef SATMI_CDCL_PHASES
        for (int i = 0; i < 4; ++i) st[4 + i] = (int64_t)S.clk[i];
        for (int i = 0; i < 3; ++i) st[1 + i] = (int64_t)S.clk[4 + i];   // moves, entries, lists
        // (over the model row) clocks in watch adds, in resizes, resizes, entries moved by them, adds
        // then clocks in analyze_conflict and in learn_clause (their watch adds included)
        for (int i = 0; i < 7 && i < A.assign_stride; ++i)
            out[i] = (int32_t)min<uint64_t>(S.clk[8 + i], INT32_MAX);
#endif
        A.var_inc[b] = q.var_inc;
    }
}

// IN_LDS: [val, pool) of the layout and the learned-literal scratch live in
// the wave's LDS (A.lay.lds_bytes > 0).  A compile-time choice, so that every
// access is a ds_* or a global_* instruction: a pointer picked at run time
// between the two is generic, and flat instructions (both wait counters, no
// LDS fast path) were every access of the kernel.
template <bool IN_LDS>
__global__ void __launch_bounds__(64) cdcl_kernel(CdclArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char cdcl_lds[];
    unsigned char *base = A.arena + (size_t)blockIdx.x * (size_t)A.lay.bytes;
    // [val, pool) of the layout, relocated into LDS when it fits
    const auto small = [&](uint64_t off) -> unsigned char * {
        if constexpr (IN_LDS)
            return cdcl_lds + (off - A.lay.val);
        else
            return base + off;
    };
    St S;
    S.coff = (int32_t *)(base + A.lay.coff);
    S.lits = (int32_t *)(base + A.lay.lits);
    S.val = (int8_t *)small(A.lay.val);
    S.ord = (int64_t *)small(A.lay.ord);
    S.lev = (int32_t *)small(A.lay.lev);
    S.ante = (int32_t *)small(A.lay.ante);
    S.act = (double *)small(A.lay.act);
    S.appears = (uint64_t *)small(A.lay.appears);
    S.klit = (int32_t *)small(A.lay.klit);
    S.kidx = (int32_t *)small(A.lay.kidx);
    S.woff = (int32_t *)small(A.lay.woff);
    S.wmask = (int32_t *)small(A.lay.wmask);
    S.wfill = (int32_t *)small(A.lay.wfill);
    S.wused = (int32_t *)small(A.lay.wused);
    S.pool = (int32_t *)(base + A.lay.pool);
#ifdef SATMI_CDCL_PHASES
    __shared__ uint64_t clk_s[16];
    S.clk = clk_s;
#endif
    if constexpr (IN_LDS)
        S.scratch = (int32_t *)(cdcl_lds + A.lay.lds_scratch);
    else
        S.scratch = (int32_t *)(base + A.lay.scratch);
    span_begin(A.work_counter);
    uint64_t busy = 0;   // this wave's ticks spent solving (the rest of its residency is the launch's tail)
    for (;;) {
        uint32_t b = 0;
        if (lane_id() == 0) b = atomicAdd(A.work_counter, 1u);
        b = uniform_u32(b);
        if (b >= (uint32_t)A.num_instances) break;
        const uint64_t t = __builtin_amdgcn_s_memrealtime();
        solve_one(A, S, (int)b);
        busy += __builtin_amdgcn_s_memrealtime() - t;
        wave_sync();
    }
    if (lane_id() == 0) atomicAdd((unsigned long long *)A.work_counter + 3, (unsigned long long)busy);
    span_end(A.work_counter);
}

constexpr uint64_t CDCL_LDS_MAX = 32768;   // per wave (one-wave workgroups)

bool make_cdcl_layout(int max_vars, int64_t max_clauses, int64_t max_lits, int max_len, int64_t learn_cap,
                      CdclLayout *L) {
    const int64_t N = (int64_t)max_vars + 1;
    const int64_t C = max_clauses + learn_cap;               // clauses incl. learned
    const int64_t Lc = max_lits + learn_cap * (int64_t)std::max(max_len, 1);
    const int64_t K = 2 * N;                                 // watch-list keys
    // set tables: each clause sits in <= 2 sets; a table is < 8x its entries
    // over its lifetime (doubling tables, dummies until the next resize)
    const int64_t P = 16 * 2 * C + (int64_t)WS_MINSIZE * K;
    auto a = [](uint64_t x) { return (x + 255u) & ~(uint64_t)255u; };
    uint64_t o = 0;
    L->coff = o;    o = a(o + 4 * (uint64_t)(C + 1));
    L->lits = o;    o = a(o + 4 * (uint64_t)Lc);
    L->val = o;     o = a(o + (uint64_t)N);
    L->ord = o;     o = a(o + 8 * (uint64_t)N);
    L->lev = o;     o = a(o + 4 * (uint64_t)N);
    L->ante = o;    o = a(o + 4 * (uint64_t)N);
    L->act = o;     o = a(o + 8 * (uint64_t)N);
    L->appears = o; o = a(o + 8 * (uint64_t)(N / 64 + 1));
    L->klit = o;    o = a(o + 4 * (uint64_t)K);
    L->kidx = o;    o = a(o + 4 * (uint64_t)K);
    L->woff = o;    o = a(o + 4 * (uint64_t)K);
    L->wmask = o;   o = a(o + 4 * (uint64_t)K);
    L->wfill = o;   o = a(o + 4 * (uint64_t)K);
    L->wused = o;   o = a(o + 4 * (uint64_t)K);
    L->pool = o;    o = a(o + 4 * (uint64_t)P);
    L->lcap = (int32_t)std::min<int64_t>(2 * N + 2 + std::max(max_len, 1), INT32_MAX / 8);
    L->scratch = o; o = a(o + 4 * 2 * (uint64_t)L->lcap);   // two learned-literal lists
    L->bytes = o;
    const uint64_t small = L->pool - L->val, lds = small + 4 * 2 * (uint64_t)L->lcap;
    L->lds_bytes = lds <= CDCL_LDS_MAX ? (uint32_t)lds : 0u;
    L->lds_scratch = (uint32_t)small;
    L->clause_cap = C;
    L->lit_cap = Lc;
    L->pool_cap = P;
    L->ncap = max_vars;
    // clause offsets, literal indices and table offsets are 32-bit in the kernel
    return max_vars >= 0 && max_vars < (1 << 29) && C < INT32_MAX && Lc < INT32_MAX && P < INT32_MAX;
}

// Device memory of satmi_cdcl_batch_host, kept between calls (grow-only): the
// per-wave arenas of a batch are sized for max_iter learned clauses and reach
// gigabytes, whose hipMalloc / hipFree per call cost more than the solves of a
// menu-sized batch.  One slot per concurrent call (a call takes a free slot of
// its device or adds one, and returns it when done), each with its own
// non-blocking stream: calls from several host threads overlap on the device,
// so the waves a batch's few long solves leave idle run another batch.  The
// slots are bounded by the peak number of concurrent calls; never destroyed (no
// hipFree after the runtime's teardown).
struct CdclSlot {
    int dev = 0;
    bool busy = false;
    void *p = nullptr;
    size_t cap = 0;
    hipStream_t stream = nullptr;
};
struct CdclPool {
    std::mutex mu;
    std::vector<CdclSlot *> slots;
};
CdclPool &cdcl_pool() {
    static CdclPool *c = new CdclPool;
    return *c;
}
// a free slot of device `dev` (created with its stream when none is free)
CdclSlot *cdcl_acquire(int dev) {
    CdclPool &P = cdcl_pool();
    std::lock_guard<std::mutex> lk(P.mu);
    for (CdclSlot *c : P.slots)
        if (c->dev == dev && !c->busy) {
            c->busy = true;
            return c;
        }
    CdclSlot *c = new CdclSlot;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return nullptr;
    }
    c->dev = dev;
    c->busy = true;
    P.slots.push_back(c);
    return c;
}
// The calling thread's last satmi_cdcl_batch_host launch (satmi_cdcl_last_stats).
struct CdclStats {
    double span_s = 0.0, busy_wave_s = 0.0;
    int resident_waves = 0;
};
thread_local CdclStats g_cdcl_stats;

struct CdclSlotGuard {
    CdclSlot *c;
    ~CdclSlotGuard() {
        std::lock_guard<std::mutex> lk(cdcl_pool().mu);
        c->busy = false;
    }
};

}  // namespace
}  // namespace satmi

using namespace satmi;

extern "C" int satmi_cdcl_batch_host(int num_instances, const int32_t *h_inst_clause_begin,
                                     const int32_t *h_clause_lit_begin, const int32_t *h_lits, int64_t max_iter,
                                     int64_t learn_cap, double time_limit_s, int32_t *h_status,
                                     int32_t *h_assign_len, int32_t *h_assign, int assign_stride,
                                     int64_t *h_stats, double *h_var_inc) {
    if (num_instances < 0 || !h_inst_clause_begin || !h_clause_lit_begin || !h_status || !h_assign_len ||
        !h_assign || !h_stats || !h_var_inc || assign_stride < 0) {
        set_error("satmi_cdcl_batch_host: bad arguments");
        return SATMI_ERR_ARG;
    }
    if (num_instances == 0) return SATMI_OK;
    const int C = h_inst_clause_begin[num_instances];
    const int Ltot = h_clause_lit_begin[C];
    std::vector<int32_t> nv(num_instances, 0);
    int max_vars = 0, max_len = 0;
    int64_t max_clauses = 0, max_lits = 0;
    // (flat loops without early exits: the compiler vectorises them; a batch of
    // 32,768 menu formulas is ~5 M literals, scanned on the host every call)
    for (int c = 0; c < C; ++c) max_len = std::max(max_len, h_clause_lit_begin[c + 1] - h_clause_lit_begin[c]);
    int bad = 0;
    for (int b = 0; b < num_instances; ++b) {
        const int cb = h_inst_clause_begin[b], ce = h_inst_clause_begin[b + 1];
        const int lb = h_clause_lit_begin[cb], le = h_clause_lit_begin[ce];
        max_clauses = std::max<int64_t>(max_clauses, ce - cb);
        max_lits = std::max<int64_t>(max_lits, le - lb);
        uint32_t m = 0;
        for (int j = lb; j < le; ++j) {
            const int x = h_lits[j];
            bad |= (x == 0) | (x == INT32_MIN);
            m = std::max(m, x < 0 ? 0u - (uint32_t)x : (uint32_t)x);   // (INT32_MIN rejected below)
        }
        nv[b] = (int)std::min<uint32_t>(m, INT32_MAX);
        max_vars = std::max(max_vars, nv[b]);
    }
    if (bad) {
        set_error("satmi_cdcl_batch_host: literal 0 / INT32_MIN");
        return SATMI_ERR_ARG;
    }
    if (assign_stride < max_vars) {
        set_error("satmi_cdcl_batch_host: assign_stride < number of variables");
        return SATMI_ERR_ARG;
    }
    // learned clauses: one per conflict, at most one per iteration
    if (learn_cap <= 0) learn_cap = max_iter > 0 ? max_iter : (1 << 16);
    CdclLayout lay;
    if (!make_cdcl_layout(max_vars, max_clauses, max_lits, max_len, learn_cap, &lay)) {
        set_error("satmi_cdcl_batch_host: instance too large");
        return SATMI_ERR_TOO_LARGE;
    }
    int dev = 0, cus = 256;
    SATMI_HIP(hipGetDevice(&dev));
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    size_t free_b = 0, total_b = 0;
    SATMI_HIP(hipMemGetInfo(&free_b, &total_b));
    const size_t by_mem = (free_b / 2) / std::max<uint64_t>(lay.bytes, 1);
    if (by_mem < 1) {
        set_error("satmi_cdcl_batch_host: one instance's arena exceeds half the free device memory");
        return SATMI_ERR_NOMEM;
    }
    const int grid = (int)std::min<size_t>({(size_t)num_instances, (size_t)cus * 32, by_mem});
    int wclock = 0;
    double ticks_per_s = 1e8;
    if (hipDeviceGetAttribute(&wclock, hipDeviceAttributeWallClockRate, dev) == hipSuccess && wclock > 0)
        ticks_per_s = (double)wclock * 1000.0;
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_icb = 0, o_clb = o_icb + up(4 * (size_t)(num_instances + 1));
    const size_t o_lits = o_clb + up(4 * (size_t)(C + 1));
    const size_t o_nv = o_lits + up(4 * (size_t)std::max(Ltot, 1));
    const size_t o_st = o_nv + up(4 * (size_t)num_instances);
    const size_t o_al = o_st + up(4 * (size_t)num_instances);
    const size_t o_as = o_al + up(4 * (size_t)num_instances);
    const size_t o_stats = o_as + up(4 * (size_t)num_instances * std::max(assign_stride, 1));
    const size_t o_vi = o_stats + up(8 * (size_t)num_instances * SATMI_CDCL_NSTATS);
    const size_t o_wc = o_vi + up(8 * (size_t)num_instances);
    const size_t o_arena = o_wc + 256;
    const size_t total = o_arena + (size_t)grid * (size_t)lay.bytes;
    CdclSlot *slot = cdcl_acquire(dev);
    if (!slot) {
        set_error("satmi_cdcl_batch_host: hipStreamCreate failed");
        return SATMI_ERR_HIP;
    }
    CdclSlotGuard guard{slot};
    if (slot->cap < total) {
        if (slot->p) (void)hipFree(slot->p);
        slot->p = nullptr;
        slot->cap = 0;
        void *p = nullptr;
        SATMI_HIP(hipMalloc(&p, total));
        slot->p = p;
        slot->cap = total;
    }
    unsigned char *d = (unsigned char *)slot->p;
    hipStream_t s = slot->stream;
    int rc = SATMI_OK;
    do {
        auto h2d = [&](size_t off, const void *src, size_t bytes) {
            return bytes ? hipMemcpyAsync(d + off, src, bytes, hipMemcpyHostToDevice, s) : hipSuccess;
        };
        if (h2d(o_icb, h_inst_clause_begin, 4 * (size_t)(num_instances + 1)) != hipSuccess ||
            h2d(o_clb, h_clause_lit_begin, 4 * (size_t)(C + 1)) != hipSuccess ||
            h2d(o_lits, h_lits, 4 * (size_t)Ltot) != hipSuccess ||
            h2d(o_nv, nv.data(), 4 * (size_t)num_instances) != hipSuccess ||
            hipMemsetAsync(d + o_wc, 0, 32, s) != hipSuccess) {   // counter, span (common.h), busy ticks
            rc = hip_fail(hipGetLastError(), "satmi_cdcl_batch_host: staging");
            break;
        }
        CdclArgs A;
        A.inst_clause_begin = (const int32_t *)(d + o_icb);
        A.clause_lit_begin = (const int32_t *)(d + o_clb);
        A.lits = (const int32_t *)(d + o_lits);
        A.inst_nvars = (const int32_t *)(d + o_nv);
        A.num_instances = num_instances;
        A.max_iter = max_iter;
        A.time_limit_ticks = time_limit_s > 0 ? (uint64_t)(time_limit_s * ticks_per_s) : 0;
        A.status = (int32_t *)(d + o_st);
        A.assign_len = (int32_t *)(d + o_al);
        A.assign = (int32_t *)(d + o_as);
        A.assign_stride = assign_stride;
        A.stats = (int64_t *)(d + o_stats);
        A.var_inc = (double *)(d + o_vi);
        A.arena = d + o_arena;
        A.lay = lay;
        A.work_counter = (uint32_t *)(d + o_wc);
        if (lay.lds_bytes)
            hipLaunchKernelGGL(cdcl_kernel<true>, dim3(grid), dim3(64), lay.lds_bytes, s, A);
        else
            hipLaunchKernelGGL(cdcl_kernel<false>, dim3(grid), dim3(64), 0, s, A);
        hipError_t e = hipGetLastError();
        auto d2h = [&](void *dst, size_t off, size_t bytes) {
            if (e == hipSuccess && bytes) e = hipMemcpyAsync(dst, d + off, bytes, hipMemcpyDeviceToHost, s);
        };
        d2h(h_status, o_st, 4 * (size_t)num_instances);
        d2h(h_assign_len, o_al, 4 * (size_t)num_instances);
        d2h(h_assign, o_as, 4 * (size_t)num_instances * assign_stride);
        d2h(h_stats, o_stats, 8 * (size_t)num_instances * SATMI_CDCL_NSTATS);
        d2h(h_var_inc, o_vi, 8 * (size_t)num_instances);
        uint64_t wc[4] = {0, 0, 0, 0};
        d2h(wc, o_wc, sizeof(wc));
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "satmi_cdcl_batch_host: launch / copy back");
        g_cdcl_stats.span_s = (double)(wc[2] - ~wc[1]) / ticks_per_s;
        g_cdcl_stats.busy_wave_s = (double)wc[3] / ticks_per_s;
        g_cdcl_stats.resident_waves = grid;
    } while (0);
    return rc;
}

extern "C" int satmi_cdcl_last_stats(double *span_s, double *busy_wave_s, int *resident_waves) {
    if (span_s) *span_s = g_cdcl_stats.span_s;
    if (busy_wave_s) *busy_wave_s = g_cdcl_stats.busy_wave_s;
    if (resident_waves) *resident_waves = g_cdcl_stats.resident_waves;
    return SATMI_OK;
}
