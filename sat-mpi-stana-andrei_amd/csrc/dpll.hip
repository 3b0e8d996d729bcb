// dpll.hip -- batched DPLL for gfx950: one instance per wavefront.
//
// Replaces dpll_optimized (REF.py:133-214) for batches of CNF formulas.
//
// Formulation (not the reference's list copying, and not a clause re-scan):
//   * The instance is staged once into the wave's LDS slice: literal codes
//     (var<<1 | negative, 16 bit), clause offsets, and per-literal occurrence
//     lists (clause indices) built in LDS by a counting sort.  The search never
//     touches HBM again until it writes the verdict.
//   * The reference's shrinking formula (filtered Python lists) is represented
//     by one 32-bit word per clause, cst[c] = nfree | ntrue << 16: nfree counts
//     the literal occurrences not falsified by an *effective* assignment (the
//     length of the reference's reduced clause), ntrue the occurrences made
//     true (ntrue > 0 <=> the reference dropped the clause).  A clause is a
//     unit clause of the reduced formula iff cst == 1 and is emptied iff
//     nfree == 0.  Unit propagation and pure-literal assignments are effective
//     (they rewrite the formula, REF.py:156-164 / :190-194); in
//     SATMI_MODE_REF a branch assignment is not (REF.py:210-213 never rewrites
//     the formula), in SATMI_MODE_SOUND it is.
//   * Assigning literal l touches only the occurrence lists of l and -l, with
//     LDS atomics on cst; the wave processes the flattened occurrences of a
//     whole range of assignments at once (prefix sum over list lengths, owner
//     lane found by a 6-step shuffle search).  Undo on backtrack is the exact
//     inverse.  cnt[v] = positive | negative << 16 counts v's occurrences in
//     active clauses and is maintained when a clause enters / leaves.
//   * unit_propagate (REF.py:139-165) processes a *snapshot* of unit clauses
//     in clause order.  A snapshot is assigned in parallel (first occurrence of
//     a variable wins, exactly the `if var in a` rule of REF.py:149-152) with a
//     time stamp = its index in the snapshot; a clause emptied by the batch was
//     emptied at the max time stamp of its literals, so the reference's
//     stopping point is the minimum of those, and the assignments after it are
//     undone -- counts match the reference one for one.  Clauses that became
//     unit are flagged in a bitmap; the next snapshot is the flagged clauses
//     still unit, in clause order (ballot/popcount compaction).
//   * Pure literals / branching (REF.py:174-208) read cnt per variable; first
//     occurrences (the dict order of literal_sign / var_counts) are recovered
//     from the occurrence lists only for the pure and the maximal variables.
//   * Recursion is an explicit frame stack + trail in LDS.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <atomic>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.h"
#include "dpll_scan.h"

namespace satmi {

constexpr uint32_t VS_ASSIGNED = 1u, VS_VALUE = 2u, VS_EFF = 4u, VS_FLAGS = 7u;
constexpr int VS_TIME_SHIFT = 3;
// Two storage widths of the same kernel (both exact REF.py semantics):
//  * Narrow: the instance image in the wave's LDS slice; 16-bit literal codes,
//    clause indices and literal positions; cst[c] = nfree | ntrue << 8 | (sum
//    of the free literal codes mod 2^16) << 16 -- when nfree == 1 the high half
//    is the one free literal (clauses <= 255 literals); cnt = pos | neg << 16.
//  * Wide: the image in a per-wave HBM arena (L2 caches the hot part), for
//    formulas beyond one wave's LDS (the reference's own 1000 x 50 and 5000 x 500
//    menu runs, rezultat.txt:248-250 and :488-490); 32-bit codes / indices /
//    positions, cst = nfree | ntrue << 16 | code sum << 32 (clauses <= 65535
//    literals), cnt = pos | neg << 32.
struct Narrow {
    using Idx = uint16_t;
    using Cst = uint32_t;
    using Cnt = uint32_t;
    static constexpr uint32_t PHASE = 0x8000u;   // fvar: the False branch runs
    static constexpr int NT_SHIFT = 8, SUM_SHIFT = 16, CNT_SHIFT = 16;
    static constexpr int MAX_LEN = 255;
};
struct Wide {
    using Idx = uint32_t;
    using Cst = uint64_t;
    using Cnt = uint64_t;
    static constexpr uint32_t PHASE = 0x80000000u;
    static constexpr int NT_SHIFT = 16, SUM_SHIFT = 32, CNT_SHIFT = 32;
    static constexpr int MAX_LEN = 65535;
};
template <typename T> __device__ __forceinline__ typename T::Cst cst_true1() { return (typename T::Cst)1 << T::NT_SHIFT; }
template <typename T> __device__ __forceinline__ uint32_t cst_nfree(typename T::Cst s) {
    return (uint32_t)(s & (((typename T::Cst)1 << T::NT_SHIFT) - 1));
}
template <typename T> __device__ __forceinline__ uint32_t cst_ntrue(typename T::Cst s) {
    return (uint32_t)((s >> T::NT_SHIFT) & (((typename T::Cst)1 << (T::SUM_SHIFT - T::NT_SHIFT)) - 1));
}
// nfree == 1 and ntrue == 0: a unit clause of the reduced formula
template <typename T> __device__ __forceinline__ bool cst_unit(typename T::Cst s) {
    return (s & (((typename T::Cst)1 << T::SUM_SHIFT) - 1)) == 1;
}
template <typename T> __device__ __forceinline__ uint32_t cst_sum(typename T::Cst s) {
    return (uint32_t)(s >> T::SUM_SHIFT);
}
// one occurrence of a positive (negative) literal in a cnt word
template <typename T> __device__ __forceinline__ typename T::Cnt cnt_one(uint32_t code) {
    return (code & 1u) ? ((typename T::Cnt)1 << T::CNT_SHIFT) : (typename T::Cnt)1;
}
template <typename T> __device__ __forceinline__ uint32_t cnt_pos(typename T::Cnt c) {
    return (uint32_t)(c & (((typename T::Cnt)1 << T::CNT_SHIFT) - 1));
}
template <typename T> __device__ __forceinline__ uint32_t cnt_neg(typename T::Cnt c) { return (uint32_t)(c >> T::CNT_SHIFT); }
constexpr uint32_t NO_CLAIM = 0xFFFFFFFFu;

// Diagnostic build only (make diag -> libsatmi_diag.so): per-phase shader-clock
// accounting, written as int64 over the caller's root_lits rows.  The product
// library compiles every stamp away.
#ifdef SATMI_PHASE_STAMPS
struct PhaseClock {
    uint64_t acc[8];
    uint64_t t;
    __device__ void start() {
        for (int i = 0; i < 8; ++i) acc[i] = 0;
        t = __builtin_amdgcn_s_memtime();
    }
    __device__ void mark(int i) {
        const uint64_t x = __builtin_amdgcn_s_memtime();
        acc[i] += x - t;
        t = x;
    }
};
#define PH_MARK(i) ph.mark(i)
#else
struct PhaseClock {
    __device__ void start() {}
    __device__ void mark(int) {}
};
#define PH_MARK(i) ((void)0)
#endif
enum { PH_STAGE = 0, PH_ASSIGN = 1, PH_APPLY = 2, PH_COLLECT = 3, PH_ANALYZE = 4, PH_PURE = 5, PH_BACKTRACK = 6,
       PH_OTHER = 7 };

struct DpllLayout {
    uint32_t lit, coff, occoff, occ, cst, vst, cnt, claim, trail, fvar, ftrail, units, ubits, posbits, mark, bytes;
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

template <typename T>
struct LdsT {
    using Idx = typename T::Idx;
    Idx *lit;                  // [lcap]      literal codes, clause-major (REF.py's clause lists)
    Idx *coff;                 // [mcap+1]    clause offsets into lit
    Idx *occoff;               // [2ncap+3]   occurrence-list offsets per literal code
    Idx *occ;                  // [lcap]      clause index of every occurrence, grouped by literal code
    typename T::Cst *cst;      // [mcap]      nfree | ntrue | free-literal code sum (see Narrow / Wide)
    uint32_t *vst;             // [ncap+1]    assigned / value / effective bits, batch time + 1 above bit 3
    typename T::Cnt *cnt;      // [ncap+1]    occurrences in active clauses: positive | negative
    typename T::Cnt *claim;    // [ncap+1]    first snapshot index claiming the variable (scratch; cursor at staging)
    Idx *trail;                // [ncap+1]    assignment order (literal codes) == dict insertion order
    Idx *fvar;                 // [ncap+1]    decision frames: var | T::PHASE once the False branch runs
    Idx *ftrail;               // [ncap+1]    trail length before the decision
    Idx *units;                // [mcap+1]    current unit-clause snapshot (literal codes)
    uint64_t *ubits;           // [mcap/64]   clauses that became unit in the current batch
    uint64_t *posbits;         // [lcap/64]   pure literals by first position
    int32_t *mark;             // [64]        scratch row (range starts of a flattened apply)
};

// Time stamp of the clause's emptying: the latest batch time among its (all
// false) literals.
template <typename T>
__device__ int emptied_time(const LdsT<T> &S, uint32_t c) {
    int t = -1;
    const int je = S.coff[c + 1];
    for (int j = S.coff[c]; j < je; ++j) t = max(t, (int)(S.vst[S.lit[j] >> 1] >> VS_TIME_SHIFT) - 1);
    return t;
}

// A clause leaves (UNDO: re-enters) the reduced formula: its literals' active
// occurrence counts change.  Slots past the clause end add 0 to cnt[0] (an
// unused word) so the group of four loads and atomics runs without branches.
template <typename T, bool UNDO>
__device__ __forceinline__ void clause_counts(const LdsT<T> &S, uint32_t c) {
    const int jb = S.coff[c], je = S.coff[c + 1];
    for (int j = jb; j < je; j += 4) {
        uint32_t x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] = S.lit[j + u];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const bool in = j + u < je;
            const typename T::Cnt inc = in ? cnt_one<T>(x[u]) : (typename T::Cnt)0;
            const uint32_t v = in ? (x[u] >> 1) : 0u;
            if (UNDO) atomicAdd(&S.cnt[v], inc);
            else atomicSub(&S.cnt[v], inc);
        }
    }
}

// One occurrence of literal `code` (r < n0: in its own list, else in its
// negation's list), as one atomic on the clause word.  Returns true when the
// clause changed satisfied state.
template <typename T, bool UNDO>
__device__ __forceinline__ bool occ_step(const LdsT<T> &S, int r, int n0, int b0, int b1, uint32_t code, int &e_loc) {
    const bool pos = r < n0;
    const uint32_t c = S.occ[pos ? b0 + r : b1 + (r - n0)];
    // own list: a true occurrence more (undo: less); negation's list: a free
    // occurrence less and its code leaves the sum (undo: back)
    using Cst = typename T::Cst;
    const Cst fdelta = (Cst)1 + ((Cst)(code ^ 1u) << T::SUM_SHIFT);
    const Cst delta = pos ? (UNDO ? (Cst)0 - cst_true1<T>() : cst_true1<T>()) : (UNDO ? fdelta : (Cst)0 - fdelta);
    const Cst old = atomicAdd(&S.cst[c], delta);
    const bool trans = pos && cst_ntrue<T>(old) == (UNDO ? 1u : 0u);
    if (trans) clause_counts<T, UNDO>(S, c);
    if (!UNDO && !pos) {
        const uint32_t nf = cst_nfree<T>(old) - 1u;
        if (nf == 0u) {
            e_loc = min(e_loc, emptied_time(S, c));
        } else if (nf == 1u && cst_ntrue<T>(old) == 0u) {
            atomicOr((unsigned long long *)&S.ubits[c >> 6], 1ull << (c & 63));
        }
    }
    return trans;
}

// Apply (UNDO=false) or revert (UNDO=true) the effective assignment of up to 64
// literals held one per lane (`has`), lane order = time order: clauses
// containing the literal gain/lose a true occurrence, clauses containing its
// negation lose/regain a free occurrence.  The occurrences of all lanes are
// flattened over the wave (prefix sum of list lengths; each flat slot finds
// its owner lane by marking range starts and a max-scan).  Returns the change
// in the number of satisfied clauses; on apply, e_loc collects the time stamps
// of emptied clauses and newly-unit clauses are flagged in ubits.
template <typename T, bool UNDO>
__device__ int apply_lanes(const LdsT<T> &S, bool has, uint32_t code, int &e_loc) {
    const int ln = lane_id();
    int b0 = 0, n0 = 0, b1 = 0, len = 0;
    if (has) {
        b0 = S.occoff[code];
        n0 = S.occoff[code + 1] - b0;
        b1 = S.occoff[code ^ 1u];
        len = n0 + (S.occoff[(code ^ 1u) + 1] - b1);
    }
    const uint64_t hm = __ballot(len > 0);
    int dsat = 0;
    if (hm == 0ull) return 0;
    if ((hm & (hm - 1ull)) == 0ull) {   // a single literal: its slots map onto lanes directly
        const int o = __ffsll((unsigned long long)hm) - 1;
        const int on0 = __builtin_amdgcn_readlane(n0, o), ob0 = __builtin_amdgcn_readlane(b0, o);
        const int ob1 = __builtin_amdgcn_readlane(b1, o), olen = __builtin_amdgcn_readlane(len, o);
        const uint32_t ocode = (uint32_t)__builtin_amdgcn_readlane((int)code, o);
        for (int f0 = 0; f0 < olen; f0 += 64) {
            const int f = f0 + ln;
            bool trans = false;
            if (f < olen) trans = occ_step<T, UNDO>(S, f, on0, ob0, ob1, ocode, e_loc);
            dsat += __popcll(__ballot(trans));
        }
    } else {
        const int incl = wave_incl_scan(len);
        const int start = incl - len;
        const int total = lane63(incl);
        int carry = 0;
        for (int f0 = 0; f0 < total; f0 += 64) {
            const int f = f0 + ln;
            S.mark[ln] = -1;
            wave_sync();
            if (len > 0 && start >= f0 && start < f0 + 64) S.mark[start - f0] = ln;
            wave_sync();
            int o = S.mark[ln];
            if (ln == 0) o = max(o, carry);
            o = wave_incl_max(o);
            carry = lane63(o);
            const int r = f - __shfl(start, o, 64);
            const int on0 = __shfl(n0, o, 64);
            const int ob0 = __shfl(b0, o, 64);
            const int ob1 = __shfl(b1, o, 64);
            const uint32_t ocode = (uint32_t)__shfl((int)code, o, 64);
            bool trans = false;
            if (f < total) trans = occ_step<T, UNDO>(S, r, on0, ob0, ob1, ocode, e_loc);
            dsat += __popcll(__ballot(trans));
        }
    }
    wave_sync();
    return UNDO ? -dsat : dsat;
}

// apply_lanes over trail[beg, end) (UNDO: only the effective entries).
template <typename T, bool UNDO>
__device__ int apply_trail(const LdsT<T> &S, int beg, int end) {
    int dsat = 0, e_loc = INT_MAX;
    for (int e0 = beg; e0 < end; e0 += 64) {
        const int e = e0 + lane_id();
        bool has = false;
        uint32_t code = 0;
        if (e < end) {
            code = S.trail[e];
            has = !UNDO || (S.vst[code >> 1] & VS_EFF);
        }
        dsat += apply_lanes<T, UNDO>(S, has, code, e_loc);
    }
    return dsat;
}

template <typename T>
__device__ void clear_ubits(const LdsT<T> &S, int m) {
    for (int w = lane_id(); w < ((m + 63) >> 6); w += 64) S.ubits[w] = 0ull;
    wave_sync();
}

// The next snapshot: clauses flagged in ubits that are still unit, in clause
// order (REF.py:143); cst's high half holds the one free literal's code.
template <typename T>
__device__ int collect_units(const LdsT<T> &S, int m) {
    const int ln = lane_id();
    const int W = (m + 63) >> 6;
    int nu = 0;
    for (int w0 = 0; w0 < W; w0 += 64) {
        const int w = w0 + ln;
        uint64_t bits = 0;
        if (w < W) {
            bits = S.ubits[w];
            S.ubits[w] = 0ull;
        }
        uint64_t keep = 0;
        for (uint64_t b = bits; b; b &= b - 1) {
            const int c = w * 64 + (__ffsll((unsigned long long)b) - 1);
            if (cst_unit<T>(S.cst[c])) keep |= b & (~b + 1);   // nfree == 1, ntrue == 0
        }
        const int kc = __popcll(keep);
        const int incl = wave_incl_scan(kc);
        int pos = nu + incl - kc;
        for (; keep; keep &= keep - 1) {
            const int c = w * 64 + (__ffsll((unsigned long long)keep) - 1);
            S.units[pos++] = (typename T::Idx)cst_sum<T>(S.cst[c]);
        }
        nu += lane63(incl);
    }
    wave_sync();
    return uniform_i32(nu);
}

// unit_propagate (REF.py:139-165) from the snapshot S.units[0, nu).  Returns
// true on conflict.  `trail_len` ends at the exact point the reference stops
// (the assignments it made, including the one that emptied a clause).
template <typename T>
__device__ bool propagate(const LdsT<T> &S, int m, bool has_empty, int &trail_len, int nu, bool decision_round,
                          int64_t &props, int64_t &rounds, int &nsat, PhaseClock &ph) {
    const int ln = lane_id();
    const uint64_t lt = lanemask_lt();
    bool dec = decision_round;
    // every batch that does not stop assigns >= 1 new variable: at most nvars+1 batches
    for (int guard = 0; nu > 0 && guard <= 32768; ++guard) {
        ++rounds;
        const int round_start = trail_len;
        int kmis = INT_MAX, e_min = INT_MAX, first_k = INT_MAX;
        uint32_t code = 0;
        bool first = false;
        for (int k0 = 0; k0 < nu && kmis == INT_MAX && e_min == INT_MAX; k0 += 64) {
            const int k = k0 + ln;
            const bool valid = k < nu;
            code = valid ? (uint32_t)S.units[k] : 0u;
            const uint32_t v = code >> 1;
            const uint32_t s = valid ? S.vst[v] : 0u;
            const bool assigned = (s & VS_ASSIGNED) != 0u;
            // assigned before this snapshot (no time stamp): equal value -> `continue`,
            // different value -> conflict at this unit (REF.py:149-151)
            const bool mis = valid && assigned && (s >> VS_TIME_SHIFT) == 0u && ((s >> 1) & 1u) == (code & 1u);
            kmis = wave_min_i32(mis ? k : INT_MAX);
            // the first occurrence of each unassigned variable before the mismatch
            // is assigned, time-stamped with its snapshot index (REF.py:154)
            const bool claimable = valid && !assigned && k < kmis;
            if (claimable) atomicMin(&S.claim[v], (typename T::Cnt)k);
            wave_sync();
            first = claimable && S.claim[v] == (typename T::Cnt)k;
            wave_sync();
            if (claimable) S.claim[v] = NO_CLAIM;
            const uint64_t mk = __ballot(first);
            if (first) {
                S.trail[trail_len + __popcll(mk & lt)] = (typename T::Idx)code;
                S.vst[v] = VS_ASSIGNED | VS_EFF | ((code & 1u) ? 0u : VS_VALUE) |
                           ((uint32_t)(k + 1) << VS_TIME_SHIFT);
            }
            if (mk && first_k == INT_MAX) first_k = k0 + __ffsll((unsigned long long)mk) - 1;
            trail_len += __popcll(mk);
            wave_sync();
            PH_MARK(PH_ASSIGN);
            // reduce the formula by this part of the batch (REF.py:156-164)
            int e_loc = INT_MAX;
            nsat += apply_lanes<T, false>(S, first, code, e_loc);
            e_min = wave_min_i32(e_loc);
            if (has_empty && mk) e_min = min(e_min, first_k);   // `[]` empties at the first reduction
            PH_MARK(PH_APPLY);
        }
        const int nassign = trail_len - round_start;
        if (e_min != INT_MAX) {
            // the reference stopped at the unit with time stamp e_min: undo the rest
            int keep = 0;
            for (int i0 = round_start; i0 < trail_len; i0 += 64) {
                const int i = i0 + ln;
                bool p = false;
                if (i < trail_len) p = (int)(S.vst[S.trail[i] >> 1] >> VS_TIME_SHIFT) - 1 <= e_min;
                keep += __popcll(__ballot(p));
            }
            const int cut = round_start + keep;
            nsat += apply_trail<T, true>(S, cut, trail_len);
            for (int i = round_start + ln; i < trail_len; i += 64) {
                const uint32_t v = S.trail[i] >> 1;
                S.vst[v] = i < cut ? (S.vst[v] & VS_FLAGS) : 0u;
            }
            trail_len = cut;
            props += keep - (dec ? 1 : 0);
            clear_ubits(S, m);
            return true;
        }
        props += nassign - (dec && nassign > 0 ? 1 : 0);
        dec = false;
        // drop this batch's time stamps
        if (nu <= 64) {
            if (first) S.vst[code >> 1] = VS_ASSIGNED | VS_EFF | ((code & 1u) ? 0u : VS_VALUE);
        } else {
            for (int i = round_start + ln; i < trail_len; i += 64) S.vst[S.trail[i] >> 1] &= VS_FLAGS;
        }
        wave_sync();
        if (kmis != INT_MAX) {
            clear_ubits(S, m);
            return true;
        }
        if (nassign == 0) break;   // `changed` stayed False (REF.py:141-142)
        nu = collect_units(S, m);
        PH_MARK(PH_COLLECT);
    }
    return false;
}

// First occurrence of variable v in the reduced formula (position in lit), the
// key of literal_sign / var_counts' dict order (REF.py:174-179, :198-203).
// Occurrence lists are sorted by clause, so each walk stops at its first
// active clause.  Requires v to occur in an active clause.
template <typename T>
__device__ uint32_t first_position(const LdsT<T> &S, uint32_t v) {
    uint32_t best = 0xFFFFFFFFu;
    for (uint32_t code = v << 1; code <= ((v << 1) | 1u); ++code) {
        const int e = S.occoff[code + 1];
        for (int i = S.occoff[code]; i < e; ++i) {
            const uint32_t c = S.occ[i];
            if (c >= best) break;
            if (cst_ntrue<T>(S.cst[c]) == 0u) {
                best = c;
                break;
            }
        }
    }
    if (best == 0xFFFFFFFFu) return 0xFFFFFFFFu;
    const int je = S.coff[best + 1];
    for (int j = S.coff[best]; j < je; ++j)
        if ((uint32_t)(S.lit[j] >> 1) == v) return (uint32_t)j;
    return 0xFFFFFFFFu;
}

struct AnRes {
    int npure;
    uint32_t best_var;   // 0 = no unassigned variable occurs (REF.py:205)
};

// literal_sign / pure_literals / var_counts (REF.py:174-208).
template <typename T>
__device__ AnRes analyze(const LdsT<T> &S, int n) {
    const int ln = lane_id();
    int npure = 0;
    uint32_t maxc = 0;
    for (int v0 = 1; v0 <= n; v0 += 64) {
        const int v = v0 + ln;
        bool pure = false;
        if (v <= n && !(S.vst[v] & VS_ASSIGNED)) {
            const typename T::Cnt c = S.cnt[v];
            const uint32_t p = cnt_pos<T>(c), q = cnt_neg<T>(c);
            if (p + q) {
                maxc = max(maxc, p + q);
                if (p == 0u || q == 0u) {
                    pure = true;
                    const uint32_t f = first_position(S, (uint32_t)v);
                    atomicOr((unsigned long long *)&S.posbits[f >> 6], 1ull << (f & 63));
                }
            }
        }
        npure += __popcll(__ballot(pure));
    }
    maxc = wave_max_u32(maxc);
    wave_sync();
    if (npure > 0 || maxc == 0) return {npure, 0u};
    // max(var_counts.items(), key=count): the first maximal key in dict order
    uint32_t bestf = 0xFFFFFFFFu;
    for (int v0 = 1; v0 <= n; v0 += 64) {
        const int v = v0 + ln;
        if (v <= n && !(S.vst[v] & VS_ASSIGNED)) {
            const typename T::Cnt c = S.cnt[v];
            if (cnt_pos<T>(c) + cnt_neg<T>(c) == maxc) bestf = min(bestf, first_position(S, (uint32_t)v));
        }
    }
    bestf = wave_min_u32(bestf);
    return {0, uniform_u32(S.lit[bestf] >> 1)};
}

// Append the pure literals to the trail in first-occurrence order (REF.py:187-189).
template <typename T>
__device__ int assign_pures(const LdsT<T> &S, int L, int trail_len) {
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
            const bool positive = cnt_pos<T>(S.cnt[v]) != 0u;
            S.trail[pos++] = (typename T::Idx)((v << 1) | (positive ? 0u : 1u));
            S.vst[v] = VS_ASSIGNED | VS_EFF | (positive ? VS_VALUE : 0u);
        }
        if (w < W) S.posbits[w] = 0ull;
        base += lane63(incl);
    }
    wave_sync();
    return trail_len + uniform_i32(base);
}

template <typename T>
__device__ void store_assignment(const LdsT<T> &S, int trail_len, int32_t *out) {
    for (int i = lane_id(); i < trail_len; i += 64) {
        const uint32_t code = S.trail[i];
        const int v = (int)(code >> 1);
        out[i] = (code & 1u) ? -v : v;
    }
}

// Pop trail[ft, trail_len): revert the effective ones, clear every variable.
template <typename T>
__device__ void unassign_to(const LdsT<T> &S, int ft, int trail_len, int &nsat) {
    nsat += apply_trail<T, true>(S, ft, trail_len);
    for (int i = ft + lane_id(); i < trail_len; i += 64) S.vst[S.trail[i] >> 1] = 0u;
    wave_sync();
}

enum { ST_PROPAGATE = 0, ST_ANALYZE = 1, ST_BACKTRACK = 2, ST_DONE = 3 };

template <typename T>
__device__ void solve_instance(const DpllArgs &A, const LdsT<T> &S, int b) {
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    PhaseClock ph;
    ph.start();
    const int ln = lane_id();
    const uint64_t lt = lanemask_lt();
    const int cb = A.inst_clause_begin[b], ce = A.inst_clause_begin[b + 1];
    const int m = ce - cb;
    const int lb = A.clause_lit_begin[cb], le = A.clause_lit_begin[ce];
    const int L = le - lb;
    const int ib = A.init_begin ? A.init_begin[b] : 0;
    const int nin = A.init_begin ? A.init_begin[b + 1] - ib : 0;
    // variables of the caller's dict may lie beyond the formula's (REF.py:133)
    int nmax = A.inst_nvars[b];
    for (int i = ln; i < nin; i += 64) nmax = max(nmax, abs(A.init_lits[ib + i]));
    const int n = -wave_min_i32(-nmax);
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
        S.lit[i] = (typename T::Idx)((v << 1) | (x < 0 ? 1u : 0u));
    }
    for (int i = ln; i <= m; i += 64) S.coff[i] = (typename T::Idx)(A.clause_lit_begin[cb + i] - lb);
    for (int v = ln; v <= n; v += 64) {
        S.vst[v] = 0u;
        S.cnt[v] = 0u;
        S.claim[v] = 0u;
    }
    for (int w = ln; w < ((m + 63) >> 6); w += 64) S.ubits[w] = 0ull;
    for (int w = ln; w < ((L + 63) >> 6); w += 64) S.posbits[w] = 0ull;
    wave_sync();
    // cst = clause length | code sum; clauses longer than T::MAX_LEN literals do not fit
    bool too_long = false;
    for (int c = ln; c < m; c += 64) {
        const int jb = S.coff[c], je = S.coff[c + 1];
        uint32_t sum = 0;
        for (int j = jb; j < je; ++j) sum += S.lit[j];
        too_long |= (je - jb) > T::MAX_LEN;
        S.cst[c] = (typename T::Cst)(je - jb) | ((typename T::Cst)sum << T::SUM_SHIFT);
    }
    if (__ballot(too_long)) {
        if (ln < SATMI_NCOUNTERS) ctr[ln] = 0;
        if (ln == 0) {
            A.status[b] = SATMI_DPLL_TOO_LARGE;
            if (A.root_len) A.root_len[b] = 0;
        }
        return;
    }
    for (int i = ln; i < L; i += 64) {
        const uint32_t x = S.lit[i];
        atomicAdd(&S.cnt[x >> 1], cnt_one<T>(x));   // all clauses are active
    }
    wave_sync();
    // occurrence-list offsets: exclusive scan over literal codes 0 .. 2n+1
    {
        int base = 0;
        for (int v0 = 0; v0 <= n; v0 += 64) {
            const int v = v0 + ln;
            uint32_t p = 0, q = 0;
            if (v <= n) {
                const typename T::Cnt c = S.cnt[v];
                p = cnt_pos<T>(c);
                q = cnt_neg<T>(c);
            }
            const int tot = (int)(p + q);
            const int incl = wave_incl_scan(tot);
            if (v <= n) {
                const int o = base + incl - tot;
                S.occoff[2 * v] = (typename T::Idx)o;
                S.occoff[2 * v + 1] = (typename T::Idx)(o + (int)p);
            }
            base += lane63(incl);
        }
        if (ln == 0) S.occoff[2 * n + 2] = (typename T::Idx)L;
    }
    wave_sync();
    // scatter occurrences in position (= clause) order so every list is sorted by
    // clause: within a 64-position chunk, equal codes are ranked by lane, the
    // group's first lane advances the code's cursor (claim[] doubles as cursor)
    for (int p0 = 0; p0 < L; p0 += 64) {
        const int p = p0 + ln;
        const bool valid = p < L;
        const uint32_t x = valid ? (uint32_t)S.lit[p] : 0xFFFFFFFFu;
        int rank = 0, grp = 0;
#pragma unroll 8
        for (int l = 0; l < 64; ++l) {
            const uint32_t y = (uint32_t)__builtin_amdgcn_readlane((int)x, l);
            const bool eq = y == x;
            grp += eq ? 1 : 0;
            rank += (eq && l < ln) ? 1 : 0;
        }
        if (valid && rank == 0) atomicAdd(&S.claim[x >> 1], cnt_one<T>(x) * (typename T::Cnt)grp);
        wave_sync();
        if (valid) {
            const typename T::Cnt cur = S.claim[x >> 1];
            const int after = (int)((x & 1u) ? cnt_neg<T>(cur) : cnt_pos<T>(cur));
            // clause of position p: the last c with coff[c] <= p
            int lo = 0, hi = m;
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if ((int)S.coff[mid] <= p) lo = mid;
                else hi = mid;
            }
            S.occ[S.occoff[x] + after - grp + rank] = (typename T::Idx)lo;
        }
        wave_sync();
    }
    for (int v = ln; v <= n; v += 64) S.claim[v] = NO_CLAIM;
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
                        if ((S.trail[t] >> 1) == v) S.trail[t] = (typename T::Idx)code;
                } else {
                    S.trail[tl++] = (typename T::Idx)code;
                }
                S.vst[v] = VS_ASSIGNED | (x > 0 ? VS_VALUE : 0u);
            }
        }
        trail_len = uniform_i32(tl);
        wave_sync();
    }
    // root snapshot: the input's unit clauses in order; does the input hold `[]`?
    bool has_empty = false;
    int nu = 0;
    for (int c0 = 0; c0 < m; c0 += 64) {
        const int c = c0 + ln;
        int len = -1;
        if (c < m) len = S.coff[c + 1] - S.coff[c];
        if (__ballot(len == 0)) has_empty = true;
        const uint64_t mk = __ballot(len == 1);
        if (len == 1) S.units[nu + __popcll(mk & lt)] = S.lit[S.coff[c]];
        nu += __popcll(mk);
    }
    wave_sync();

    PH_MARK(PH_STAGE);
    const bool sound = A.mode == SATMI_MODE_SOUND;
    int64_t nodes = 1, decisions = 0, props = 0, pures = 0, conflicts = 0, sols = 0, rounds = 0;
    int depth = 0, nsat = 0;
    int status = SATMI_DPLL_EXHAUSTED;
    bool decision_round = false, at_root = true;
    int state = ST_PROPAGATE;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();

    while (state != ST_DONE) {
        if (state == ST_PROPAGATE) {
            const bool conflict = propagate(S, m, has_empty, trail_len, nu, decision_round, props, rounds, nsat, ph);
            decision_round = false;
            if (at_root) {
                at_root = false;
                if (A.root_lits) store_assignment(S, trail_len, A.root_lits + (int64_t)b * A.sol_stride);
                if (A.root_len && ln == 0) A.root_len[b] = trail_len;
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
            bool leaf = false;
            AnRes r{0, 0u};
            if (nsat == m) {
                leaf = true;                                  // REF.py:170-171
            } else {
                r = analyze(S, n);
                if (r.npure == 0 && r.best_var == 0) leaf = true;   // REF.py:205-206
            }
            PH_MARK(PH_ANALYZE);
            if (!leaf && r.npure > 0) {                       // REF.py:186-195
                const int before = trail_len;
                trail_len = assign_pures(S, L, trail_len);
                nsat += apply_trail<T, false>(S, before, trail_len);   // a pure literal never empties a clause
                pures += r.npure;
                ++nodes;                                      // recursive call; its unit_propagate is a no-op
                PH_MARK(PH_PURE);
            } else if (!leaf) {                               // REF.py:208-213
                const uint32_t v = r.best_var;
                if (ln == 0) {
                    S.fvar[depth] = (typename T::Idx)v;
                    S.ftrail[depth] = (typename T::Idx)trail_len;
                }
                ++depth;
                ++decisions;
                ++nodes;
                const uint32_t code = v << 1;                 // True first
                if (sound) {
                    if (ln == 0) S.units[0] = (typename T::Idx)code;
                    nu = 1;
                    decision_round = true;
                    state = ST_PROPAGATE;
                } else {
                    if (ln == 0) {
                        S.vst[v] = VS_ASSIGNED | VS_VALUE;
                        S.trail[trail_len] = (typename T::Idx)code;
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
                unassign_to(S, ft, trail_len, nsat);
                trail_len = ft;
                if (!(fv & T::PHASE)) {
                    const uint32_t v = fv;
                    if (ln == 0) S.fvar[top] = (typename T::Idx)(v | T::PHASE);
                    ++decisions;
                    ++nodes;
                    const uint32_t code = (v << 1) | 1u;      // False
                    if (sound) {
                        if (ln == 0) S.units[0] = (typename T::Idx)code;
                        nu = 1;
                        decision_round = true;
                        state = ST_PROPAGATE;
                    } else {
                        if (ln == 0) {
                            S.vst[v] = VS_ASSIGNED;
                            S.trail[trail_len] = (typename T::Idx)code;
                        }
                        ++trail_len;
                        state = ST_ANALYZE;
                    }
                    wave_sync();
                    break;
                }
                --depth;
            }
            PH_MARK(PH_BACKTRACK);
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
        ctr[SATMI_CTR_TICKS] = (int64_t)(__builtin_amdgcn_s_memrealtime() - t_start);
    }
#ifdef SATMI_PHASE_STAMPS
    PH_MARK(PH_OTHER);
    if (A.root_lits && A.sol_stride >= 16 && ln < 8)
        ((int64_t *)(A.root_lits + (int64_t)b * A.sol_stride))[ln] = (int64_t)ph.acc[ln];
#endif
}

template <typename T>
__device__ __forceinline__ LdsT<T> bind_storage(unsigned char *base, const DpllLayout &lay) {
    using Idx = typename T::Idx;
    LdsT<T> S;
    S.lit = (Idx *)(base + lay.lit);
    S.coff = (Idx *)(base + lay.coff);
    S.occoff = (Idx *)(base + lay.occoff);
    S.occ = (Idx *)(base + lay.occ);
    S.cst = (typename T::Cst *)(base + lay.cst);
    S.vst = (uint32_t *)(base + lay.vst);
    S.cnt = (typename T::Cnt *)(base + lay.cnt);
    S.claim = (typename T::Cnt *)(base + lay.claim);
    S.trail = (Idx *)(base + lay.trail);
    S.fvar = (Idx *)(base + lay.fvar);
    S.ftrail = (Idx *)(base + lay.ftrail);
    S.units = (Idx *)(base + lay.units);
    S.ubits = (uint64_t *)(base + lay.ubits);
    S.posbits = (uint64_t *)(base + lay.posbits);
    S.mark = (int32_t *)(base + lay.mark);
    return S;
}

// Persistent grid: every wave pulls instance indices from a global counter until
// the batch is drained (instances differ wildly in search-tree size).
template <typename T>
__device__ __forceinline__ void run_batch(const DpllArgs &A, const LdsT<T> &S) {
    span_begin(A.work_counter);
    for (;;) {
        uint32_t b = 0;
        if (lane_id() == 0) b = atomicAdd(A.work_counter, 1u);
        b = uniform_u32(b);
        if (b >= (uint32_t)A.num_instances) break;
        solve_instance<T>(A, S, (int)b);
        wave_sync();
    }
    span_end(A.work_counter);
}

// Narrow: each wave's image in its slice of the workgroup's LDS.
__global__ void __launch_bounds__(256) dpll_batch_kernel(DpllArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = threadIdx.x >> 6;
    run_batch<Narrow>(A, bind_storage<Narrow>(smem + (size_t)wave * A.lay.bytes, A.lay));
}

// Wide: one-wave workgroups, each wave's image in its own HBM arena of
// A.lay.bytes (the flattened-apply scratch row stays in LDS).
__global__ void __launch_bounds__(64) dpll_wide_kernel(DpllArgs A, unsigned char *arena) {
    __shared__ __attribute__((aligned(16))) int32_t mark_s[64];
    LdsT<Wide> S = bind_storage<Wide>(arena + (size_t)blockIdx.x * (size_t)A.lay.bytes, A.lay);
    S.mark = mark_s;
    run_batch<Wide>(A, S);
}

// ------------------------------------------------------------------ host side
static uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }

static bool make_layout(int max_vars, int max_clauses, int max_lits, DpllLayout *lay) {
    if (max_vars < 0 || max_clauses < 0 || max_lits < 0) return false;
    // 16-bit literal codes, clause indices, literal positions and per-clause counts
    if (max_vars > 32766 || max_clauses > 65534 || max_lits > 65535) return false;
    const uint32_t N = (uint32_t)max_vars + 1, M = (uint32_t)max_clauses + 1, Lc = (uint32_t)max_lits + 1;
    uint32_t o = 0;
    lay->lit = o;     o = align16(o + 2 * (Lc + 4));   // +4: clause_counts reads in groups of four
    lay->coff = o;    o = align16(o + 2 * M);
    lay->occoff = o;  o = align16(o + 2 * (2 * N + 1));
    lay->occ = o;     o = align16(o + 2 * Lc);
    lay->cst = o;     o = align16(o + 4 * M);
    lay->vst = o;     o = align16(o + 4 * N);
    lay->cnt = o;     o = align16(o + 4 * N);
    lay->claim = o;   o = align16(o + 4 * N);
    lay->trail = o;   o = align16(o + 2 * N);
    lay->fvar = o;    o = align16(o + 2 * N);
    lay->ftrail = o;  o = align16(o + 2 * N);
    lay->units = o;   o = align16(o + 2 * M);
    lay->ubits = o;   o = align16(o + 8 * ((M + 63) / 64));
    lay->posbits = o; o = align16(o + 8 * ((Lc + 63) / 64));
    lay->mark = o;    o = align16(o + 4 * 64);
    lay->bytes = o;
    lay->lcap = max_lits;
    lay->mcap = max_clauses;
    lay->ncap = max_vars;
    return o <= 160u * 1024u;
}

// Wide storage (HBM arena per wave): 32-bit codes / indices / positions, 64-bit
// clause and count words.  False when an offset would pass 4 GiB.
static bool make_wide_layout(int max_vars, int max_clauses, int max_lits, DpllLayout *lay) {
    if (max_vars < 0 || max_clauses < 0 || max_lits < 0) return false;
    if (max_vars > (1 << 30) - 2 || max_clauses > (1 << 28) || max_lits > (1 << 30)) return false;
    const uint64_t N = (uint64_t)max_vars + 1, M = (uint64_t)max_clauses + 1, Lc = (uint64_t)max_lits + 1;
    auto a16 = [](uint64_t x) { return (x + 15u) & ~(uint64_t)15u; };
    uint64_t o = 0;
    uint64_t off[15];
    off[0] = o;  o = a16(o + 4 * (Lc + 4));        // lit (+4: clause_counts reads in groups of four)
    off[1] = o;  o = a16(o + 4 * M);               // coff
    off[2] = o;  o = a16(o + 4 * (2 * N + 1));     // occoff
    off[3] = o;  o = a16(o + 4 * Lc);              // occ
    off[4] = o;  o = a16(o + 8 * M);               // cst
    off[5] = o;  o = a16(o + 4 * N);               // vst
    off[6] = o;  o = a16(o + 8 * N);               // cnt
    off[7] = o;  o = a16(o + 8 * N);               // claim
    off[8] = o;  o = a16(o + 4 * N);               // trail
    off[9] = o;  o = a16(o + 4 * N);               // fvar
    off[10] = o; o = a16(o + 4 * N);               // ftrail
    off[11] = o; o = a16(o + 4 * M);               // units
    off[12] = o; o = a16(o + 8 * ((M + 63) / 64)); // ubits
    off[13] = o; o = a16(o + 8 * ((Lc + 63) / 64));// posbits
    off[14] = o; o = a16(o + 4 * 64);              // mark (unused: LDS row)
    o = (o + 255u) & ~(uint64_t)255u;              // arenas start on 256-B boundaries
    if (o >= (1ull << 32)) return false;
    lay->lit = (uint32_t)off[0];
    lay->coff = (uint32_t)off[1];
    lay->occoff = (uint32_t)off[2];
    lay->occ = (uint32_t)off[3];
    lay->cst = (uint32_t)off[4];
    lay->vst = (uint32_t)off[5];
    lay->cnt = (uint32_t)off[6];
    lay->claim = (uint32_t)off[7];
    lay->trail = (uint32_t)off[8];
    lay->fvar = (uint32_t)off[9];
    lay->ftrail = (uint32_t)off[10];
    lay->units = (uint32_t)off[11];
    lay->ubits = (uint32_t)off[12];
    lay->posbits = (uint32_t)off[13];
    lay->mark = (uint32_t)off[14];
    lay->bytes = (uint32_t)o;
    lay->lcap = max_lits;
    lay->mcap = max_clauses;
    lay->ncap = max_vars;
    return true;
}

// Per-device launch state.  Each stream gets its own work counter, so batches
// launched on different streams (a pipelined caller overlapping one batch's
// tail with the next batch) never share a queue; launches on one stream are
// ordered, so reusing that stream's counter is safe.
struct DeviceWork {
    std::unordered_map<hipStream_t, uint32_t *> counters;
    // incremental scan kernel: occurrence-list scratch per stream (grown, never shrunk)
    std::unordered_map<hipStream_t, std::pair<uint16_t *, size_t>> occ;
    // branch splitting: slot pool + donation stacks per stream (grown, never
    // shrunk) and the stream's launch tag for the slot states
    std::unordered_map<hipStream_t, std::pair<void *, size_t>> split;
    std::unordered_map<hipStream_t, uint32_t> split_epoch;
    std::unordered_map<hipStream_t, bool> split_last;   // the stream's last DPLL launch split (stats valid)
    // wide general kernel: per-wave HBM arenas per stream (grown, never shrunk)
    std::unordered_map<hipStream_t, std::pair<void *, size_t>> arena;
    double ticks_per_s = 1e8;
    bool init = false;
};
static std::mutex g_work_mu;
static std::vector<DeviceWork> g_work;
static std::atomic<int> g_kernel_policy{SATMI_KERNEL_AUTO};
static std::atomic<int> g_split_enable{1};
static std::atomic<int> g_split_helpers{SPLIT_HELPERS_PER_CU};
static std::atomic<int> g_split_warmup{SPLIT_WARMUP_NODES};

static int device_work(hipStream_t stream, DeviceWork **out, uint32_t **counter) {
    int dev = 0;
    SATMI_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_work_mu);
    if ((int)g_work.size() <= dev) g_work.resize(dev + 1);
    DeviceWork &w = g_work[dev];
    if (!w.init) {
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) == hipSuccess && khz > 0)
            w.ticks_per_s = (double)khz * 1000.0;
        w.init = true;
    }
    uint32_t *&c = w.counters[stream];
    if (!c) SATMI_HIP(hipMalloc(&c, 256));
    *out = &w;
    *counter = c;
    return SATMI_OK;
}

}  // namespace satmi

using namespace satmi;

extern "C" int satmi_dpll_launch_span(void *stream, uint64_t *d_span) {
    if (!d_span) {
        set_error("satmi_dpll_launch_span: d_span is NULL");
        return SATMI_ERR_ARG;
    }
    DeviceWork *w = nullptr;
    uint32_t *wc = nullptr;
    int rc = device_work((hipStream_t)stream, &w, &wc);
    if (rc) return rc;
    SATMI_HIP(hipMemcpyAsync(d_span, (uint64_t *)wc + 1, 2 * sizeof(uint64_t), hipMemcpyDeviceToDevice,
                             (hipStream_t)stream));
    return SATMI_OK;
}

extern "C" int satmi_wallclock_hz(double *hz) {
    if (!hz) {
        set_error("satmi_wallclock_hz: hz is NULL");
        return SATMI_ERR_ARG;
    }
    DeviceWork *w = nullptr;
    uint32_t *wc = nullptr;
    int rc = device_work(nullptr, &w, &wc);
    if (rc) return rc;
    *hz = w->ticks_per_s;
    return SATMI_OK;
}

// Occurrence-list scratch of the incremental kernel on `stream`: launches on one
// stream are ordered, so a buffer is only replaced after the stream drained.
static uint16_t *occ_scratch(hipStream_t stream, size_t bytes) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_work_mu);
    if ((int)g_work.size() <= dev) g_work.resize(dev + 1);
    auto &slot = g_work[dev].occ[stream];
    if (slot.second >= bytes) return slot.first;
    if (slot.first) {
        if (hipStreamSynchronize(stream) != hipSuccess) return nullptr;
        (void)hipFree(slot.first);
        slot = {nullptr, 0};
    }
    void *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
        set_error("occurrence-list scratch: hipMalloc failed");
        return nullptr;
    }
    slot = {(uint16_t *)p, bytes};
    return slot.first;
}

// Per-wave arenas of the wide general kernel on `stream` (same lifetime rule).
static void *arena_scratch(hipStream_t stream, size_t bytes) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_work_mu);
    if ((int)g_work.size() <= dev) g_work.resize(dev + 1);
    auto &slot = g_work[dev].arena[stream];
    if (slot.second >= bytes) return slot.first;
    if (slot.first) {
        if (hipStreamSynchronize(stream) != hipSuccess) return nullptr;
        (void)hipFree(slot.first);
        slot = {nullptr, 0};
    }
    void *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
        set_error("wide DPLL arenas: hipMalloc failed");
        return nullptr;
    }
    slot = {p, bytes};
    return slot.first;
}

// Branch-splitting scratch on `stream` (same lifetime rule as occ_scratch) and
// the next launch tag of its slot states.
static void *split_scratch(hipStream_t stream, size_t bytes, uint32_t *epoch) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_work_mu);
    if ((int)g_work.size() <= dev) g_work.resize(dev + 1);
    auto &slot = g_work[dev].split[stream];
    uint32_t &ep = g_work[dev].split_epoch[stream];
    if (slot.second < bytes) {
        if (slot.first) {
            if (hipStreamSynchronize(stream) != hipSuccess) return nullptr;
            (void)hipFree(slot.first);
            slot = {nullptr, 0};
        }
        void *p = nullptr;
        if (hipMalloc(&p, bytes) != hipSuccess) {
            set_error("branch-splitting scratch: hipMalloc failed");
            return nullptr;
        }
        // fresh memory: no stale state may carry the next tags
        if (hipMemsetAsync(p, 0, bytes, stream) != hipSuccess) return nullptr;
        slot = {p, bytes};
    }
    ep = (ep + 1u) & 0x0FFFFFFFu;
    if (ep == 0u) ep = 1u;
    *epoch = ep;
    g_work[dev].split_last[stream] = true;
    return slot.first;
}

// A DPLL launch on `stream` is about to be made: until its split_scratch call
// (only launches that split make one) the stream has no split statistics.
static void split_mark_unsplit(hipStream_t stream) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return;
    std::lock_guard<std::mutex> lk(g_work_mu);
    if ((int)g_work.size() <= dev) g_work.resize(dev + 1);
    g_work[dev].split_last[stream] = false;
}

extern "C" int satmi_dpll_split_stats(void *stream, int64_t *out) {
    if (!out) {
        set_error("satmi_dpll_split_stats: out is NULL");
        return SATMI_ERR_ARG;
    }
    for (int i = 0; i < 7; ++i) out[i] = 0;
    int dev = 0;
    SATMI_HIP(hipGetDevice(&dev));
    void *head = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_work_mu);
        if ((int)g_work.size() > dev) {
            auto it = g_work[dev].split.find((hipStream_t)stream);
            auto last = g_work[dev].split_last.find((hipStream_t)stream);
            if (it != g_work[dev].split.end() && last != g_work[dev].split_last.end() && last->second)
                head = it->second.first;
        }
    }
    if (!head) return SATMI_OK;   // the stream's last launch did not split: all zero (done = 0)
    unsigned char h[SPLIT_HEAD_BYTES];
    SATMI_HIP(hipStreamSynchronize((hipStream_t)stream));
    SATMI_HIP(hipMemcpy(h, head, sizeof(h), hipMemcpyDeviceToHost));
    dpll_split_decode(h, out);
    return SATMI_OK;
}

extern "C" int satmi_dpll_split_busy(void *stream, int64_t *busy_ticks) {
    if (!busy_ticks) {
        set_error("satmi_dpll_split_busy: busy_ticks is NULL");
        return SATMI_ERR_ARG;
    }
    *busy_ticks = 0;
    int dev = 0;
    SATMI_HIP(hipGetDevice(&dev));
    void *head = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_work_mu);
        if ((int)g_work.size() > dev) {
            auto it = g_work[dev].split.find((hipStream_t)stream);
            auto last = g_work[dev].split_last.find((hipStream_t)stream);
            if (it != g_work[dev].split.end() && last != g_work[dev].split_last.end() && last->second)
                head = it->second.first;
        }
    }
    if (!head) return SATMI_OK;   // the stream's last launch did not split
    unsigned char h[SPLIT_HEAD_BYTES];
    SATMI_HIP(hipStreamSynchronize((hipStream_t)stream));
    SATMI_HIP(hipMemcpy(h, head, sizeof(h), hipMemcpyDeviceToHost));
    *busy_ticks = dpll_split_busy(h);
    return SATMI_OK;
}

extern "C" int satmi_dpll_set_split(int enable, int helpers_per_cu) {
    if (helpers_per_cu < 0 || helpers_per_cu > 32) {
        set_error("satmi_dpll_set_split: helpers_per_cu must be in [0, 32]");
        return SATMI_ERR_ARG;
    }
    if (enable < 0 || enable > 2) {
        set_error("satmi_dpll_set_split: enable must be 0 (off), 1 (auto) or 2 (always)");
        return SATMI_ERR_ARG;
    }
    g_split_enable.store(enable);
    g_split_helpers.store(helpers_per_cu ? helpers_per_cu : SPLIT_HELPERS_PER_CU);
    return SATMI_OK;
}

extern "C" int satmi_dpll_set_split_warmup(int nodes) {
    g_split_warmup.store(nodes < 0 ? SPLIT_WARMUP_NODES : nodes);
    return SATMI_OK;
}

extern "C" int satmi_dpll_set_kernel(int policy) {
    if (policy != SATMI_KERNEL_AUTO && policy != SATMI_KERNEL_GENERAL && policy != SATMI_KERNEL_SCAN &&
        policy != SATMI_KERNEL_INC && policy != SATMI_KERNEL_WIDE) {
        set_error("satmi_dpll_set_kernel: unknown policy");
        return SATMI_ERR_ARG;
    }
    g_kernel_policy.store(policy);
    return SATMI_OK;
}

extern "C" uint64_t satmi_dpll_scan_lds_bytes(int max_vars, int max_clauses, int max_lits, int max_clause_len) {
    uint32_t bytes = 0;
    if (!dpll_scan_eligible(max_vars, max_clauses, max_lits, max_clause_len, false, &bytes)) return 0;
    return bytes;
}

extern "C" int satmi_dpll_plan(int max_vars, int max_clauses, int max_lits, int max_clause_len, int mode,
                               int has_init, int *kernel, uint64_t *lds_bytes_per_wave, int *waves_per_cu) {
    if (!kernel || !lds_bytes_per_wave || !waves_per_cu) {
        set_error("satmi_dpll_plan: null output");
        return SATMI_ERR_ARG;
    }
    const int policy = g_kernel_policy.load();
    uint32_t sb = 0;
    const bool inc = policy != SATMI_KERNEL_SCAN;
    if (mode == SATMI_MODE_SOUND && !has_init && policy != SATMI_KERNEL_GENERAL &&
        dpll_scan_eligible(max_vars, max_clauses, max_lits, max_clause_len, inc, &sb)) {
        *kernel = inc ? SATMI_KERNEL_INC : SATMI_KERNEL_SCAN;
        const int rc = dpll_scan_resident(max_vars, max_clauses, max_clause_len, inc, waves_per_cu, &sb);
        *lds_bytes_per_wave = sb;
        return rc;
    }
    DpllLayout lay;
    if (policy == SATMI_KERNEL_WIDE || !make_layout(max_vars, max_clauses, max_lits, &lay)) {
        if (!make_wide_layout(max_vars, max_clauses, max_lits, &lay)) {
            set_error("satmi_dpll_plan: instance too large for the wide (HBM arena) layout");
            return SATMI_ERR_TOO_LARGE;
        }
        *kernel = SATMI_KERNEL_WIDE;
        *lds_bytes_per_wave = 256;   // the arena is in HBM; LDS holds one scratch row
        *waves_per_cu = 32;
        return SATMI_OK;
    }
    *kernel = SATMI_KERNEL_GENERAL;
    *lds_bytes_per_wave = lay.bytes;
    int best = 0;
    for (int wpg : {4, 2, 1}) {
        const int wgs = std::min(16, (int)((160u * 1024u) / (lay.bytes * (uint32_t)wpg)));
        if (wgs >= 1) best = std::max(best, std::min(32, wgs * wpg));
    }
    *waves_per_cu = best;
    return SATMI_OK;
}

extern "C" uint64_t satmi_dpll_lds_bytes(int max_vars, int max_clauses, int max_lits) {
    DpllLayout lay;
    if (!make_layout(max_vars, max_clauses, max_lits, &lay)) return 0;
    return lay.bytes;
}

extern "C" int satmi_dpll_batch_device(int num_instances, const int32_t *d_inst_clause_begin,
                                       const int32_t *d_clause_lit_begin, const int32_t *d_lits,
                                       const int32_t *d_inst_nvars, int max_vars, int max_clauses,
                                       int max_lits, int max_clause_len, const int32_t *d_init_begin,
                                       const int32_t *d_init_lits,
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
    // SOUND mode without a caller assignment: the clause-scan kernel
    // (dpll_scan.hip) when the batch shape fits it, unless policy says otherwise
    const int policy = g_kernel_policy.load();
    const bool inc = policy != SATMI_KERNEL_SCAN;
    const bool scan_ok = mode == SATMI_MODE_SOUND && !d_init_begin && policy != SATMI_KERNEL_GENERAL &&
                         dpll_scan_eligible(max_vars, max_clauses, max_lits, max_clause_len, inc, nullptr);
    if ((policy == SATMI_KERNEL_SCAN || policy == SATMI_KERNEL_INC) && !scan_ok) {
        set_error("satmi_dpll_batch_device: SATMI_KERNEL_SCAN/INC policy but the batch is not eligible (SOUND "
                  "mode, no caller assignment, clause lengths 1..5, <= 2047 variables)");
        return SATMI_ERR_ARG;
    }
    if (scan_ok) {
        DeviceWork *w = nullptr;
        uint32_t *wc = nullptr;
        int rc = device_work((hipStream_t)stream, &w, &wc);
        if (rc) return rc;
        int dev = 0, cus = 256;
        SATMI_HIP(hipGetDevice(&dev));
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        ScanLaunch Lc;
        Lc.num_instances = num_instances;
        Lc.inst_clause_begin = d_inst_clause_begin;
        Lc.clause_lit_begin = d_clause_lit_begin;
        Lc.lits = d_lits;
        Lc.inst_nvars = d_inst_nvars;
        Lc.max_vars = max_vars;
        Lc.max_clauses = max_clauses;
        Lc.max_lits = max_lits;
        Lc.max_clause_len = max_clause_len;
        Lc.max_solutions = max_solutions;
        Lc.node_limit = node_limit;
        Lc.time_limit_ticks = time_limit_s > 0 ? (uint64_t)(time_limit_s * w->ticks_per_s) : 0;
        Lc.sol_cap = sol_cap;
        Lc.sol_stride = sol_stride;
        Lc.status = d_status;
        Lc.counters = d_counters;
        Lc.sol_len = d_sol_len;
        Lc.sol_lits = d_sol_lits;
        Lc.root_len = d_root_len;
        Lc.root_lits = d_root_lits;
        Lc.work_counter = wc;
        Lc.num_cus = cus;
        Lc.stream = (hipStream_t)stream;
        Lc.inc = inc;
        Lc.occ_alloc = [stream](size_t bytes) { return occ_scratch((hipStream_t)stream, bytes); };
        // branch splitting reproduces the sequential search exactly only when
        // the search stops at its first model and nothing else cuts it short
        const int sm = g_split_enable.load();
        Lc.split = sm && max_solutions == 1 && node_limit <= 0 && time_limit_s <= 0;
        Lc.split_always = sm == 2;
        Lc.split_helpers_per_cu = g_split_helpers.load();
        Lc.split_warmup = g_split_warmup.load();
        Lc.split_alloc = [stream](size_t bytes, uint32_t *epoch) {
            return split_scratch((hipStream_t)stream, bytes, epoch);
        };
        SATMI_HIP(hipMemsetAsync(wc, 0, 24, Lc.stream));   // counter + launch span (common.h)
        split_mark_unsplit(Lc.stream);
        return dpll_scan_launch(Lc);
    }
    DpllLayout lay;
    const bool wide = policy == SATMI_KERNEL_WIDE || !make_layout(max_vars, max_clauses, max_lits, &lay);
    if (wide && !make_wide_layout(max_vars, max_clauses, max_lits, &lay)) {
        set_error("satmi_dpll_batch_device: instance too large (wide layout: vars < 2^30, clauses <= 2^28, "
                  "literals <= 2^30, < 4 GiB per wave)");
        return SATMI_ERR_TOO_LARGE;
    }
    DeviceWork *w = nullptr;
    uint32_t *wc = nullptr;
    int rc = device_work((hipStream_t)stream, &w, &wc);
    if (rc) return rc;
    split_mark_unsplit((hipStream_t)stream);   // this launch does not split: its stats are all zero
    if (wide) {
        // one-wave workgroups, each with an HBM arena; resident waves bounded by
        // 32 per CU and by half the free device memory
        int dev = 0, cus = 256;
        SATMI_HIP(hipGetDevice(&dev));
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        size_t free_b = 0, total_b = 0;
        SATMI_HIP(hipMemGetInfo(&free_b, &total_b));
        const size_t per = lay.bytes;
        const size_t by_mem = std::max<size_t>(1, (free_b / 2) / per);
        const int grid = (int)std::min<size_t>({(size_t)num_instances, (size_t)cus * 32, by_mem});
        unsigned char *arena = (unsigned char *)arena_scratch((hipStream_t)stream, (size_t)grid * per);
        if (!arena) return SATMI_ERR_NOMEM;
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
        A.work_counter = wc;
        A.lay = lay;
        hipStream_t s = (hipStream_t)stream;
        SATMI_HIP(hipMemsetAsync(wc, 0, 24, s));   // counter + launch span (common.h)
        hipLaunchKernelGGL(dpll_wide_kernel, dim3(grid), dim3(64), 0, s, A, arena);
        SATMI_HIP(hipGetLastError());
        return SATMI_OK;
    }
    // Occupancy is set by LDS: pick the workgroup shape that keeps the most
    // waves resident (<= 32 waves and, conservatively, <= 16 workgroups per CU).
    int waves_per_wg = 1, wg_per_cu = 1, best_waves = 0;
    for (int wpg : {4, 2, 1}) {
        const int wgs = std::min(16, (int)((160u * 1024u) / (lay.bytes * (uint32_t)wpg)));
        const int waves = std::min(32, wgs * wpg);
        if (wgs >= 1 && waves > best_waves) {
            best_waves = waves;
            waves_per_wg = wpg;
            wg_per_cu = std::max(1, std::min(wgs, 32 / wpg));
        }
    }
    const uint32_t wg_lds = lay.bytes * (uint32_t)waves_per_wg;
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
    A.work_counter = wc;
    A.lay = lay;

    hipStream_t s = (hipStream_t)stream;
    SATMI_HIP(hipMemsetAsync(wc, 0, 24, s));   // counter + launch span (common.h)
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
    int max_vars = 0, max_clauses = 0, max_lits = 0, max_len = 0, min_len = INT_MAX;
    for (int c = 0; c < C; ++c) {
        const int len = h_clause_lit_begin[c + 1] - h_clause_lit_begin[c];
        max_len = std::max(max_len, len);
        min_len = std::min(min_len, len);
    }
    // the scan kernel needs every clause non-empty: report 0 (unknown) otherwise
    const int max_clause_len = (C > 0 && min_len >= 1) ? max_len : 0;
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
            max_clause_len, h_init_begin ? (const int32_t *)(d + o_ib) : nullptr,
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
