// dpll_scan.hip -- batched DPLL for gfx950, SOUND mode: the clause-scan kernel.
//
// Same procedure and counters as dpll_batch_kernel (dpll.hip) in
// SATMI_MODE_SOUND -- dpll_optimized (REF.py:133-214) with each branch literal
// applied as a unit clause -- in a formulation built for the CDNA4 issue model
// instead of for minimal work:
//
//   * The only mutable state of the formula is one byte per literal code,
//     lv[code] (free / true / false, see LV_*); four codes per LDS dword.  No clause state:
//     the reference's reduced formula (its filtered Python lists) is
//     *re-derived* by scanning the packed clauses, 64 clauses per wave step.
//     A clause is one LDS word (<= 3 literal codes of 10 bits, or <= 5 of 12
//     bits); the SUM of its literals' state bytes is the reduced clause:
//     satisfied or not and its length (length 1: the free slot is the unit).
//   * unit_propagate (REF.py:139-165): a scan collects the unit clauses in
//     clause order (ballot + popcount compaction) -- exactly REF.py:143's
//     snapshot.  The snapshot is assigned at once, the first occurrence of a
//     variable winning (epoch-tagged LDS atomicMax stamps written by the scan
//     itself: the `if var in a` rule of REF.py:149-152).  The next scan builds
//     the next snapshot and sees emptied clauses; an emptied clause was emptied by the
//     latest-stamped of its literals, so the reference's stopping unit is the
//     minimum of those stamps, and the assignments stamped after it are
//     dropped -- counters match the reference one for one.
//   * Backtracking clears the state bytes of the popped trail entries and
//     nothing else: there is no clause state to undo.
//   * Pure literals / branching (REF.py:174-208): one scan adds every free
//     occurrence of an active clause into per-variable counters and keeps the
//     first position (the dict order of literal_sign / var_counts).
//
// A scan step is K independent LDS gathers and K-1 adds per lane, so the
// kernel is VALU/LDS-issue bound with short dependency chains, and the
// per-wave LDS image is small (n=100, m=426: 4.8 KB, 32 waves per CU).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <type_traits>

#include "common.h"
#include "dpll_scan.h"

// minimum waves per SIMD the register allocation must allow (launch bounds)
#ifndef SATMI_SCAN_WAVES_PER_SIMD
#define SATMI_SCAN_WAVES_PER_SIMD 8
#endif

namespace satmi {
namespace {

// Diagnostic build only (make diag): per-phase shader-clock accounting, written
// as int64[8] over the caller's root_lits row (tools/dpll_probe.py --diag).
#ifdef SATMI_PHASE_STAMPS
struct PhaseClock {
    uint64_t acc[8];
    uint64_t cnt[16];   // path counts (written after the clocks)
    uint64_t t;
    __device__ void start() {
        for (int i = 0; i < 8; ++i) acc[i] = 0;
        for (int i = 0; i < 16; ++i) cnt[i] = 0;
        t = __builtin_amdgcn_s_memtime();
    }
    __device__ void count(int i, uint64_t v = 1) { cnt[i] += v; }
    __device__ void mark(int i) {
        const uint64_t x = __builtin_amdgcn_s_memtime();
        acc[i] += x - t;
        t = x;
    }
};
#else
struct PhaseClock {
    __device__ void start() {}
    __device__ void mark(int) {}
    __device__ void count(int, uint64_t = 1) {}
};
#endif
enum { PH_STAGE = 0, PH_ASSIGN = 1, PH_UNITS = 2, PH_CONFLICT = 3, PH_COUNTS = 4, PH_CHOOSE = 5, PH_PURE = 6,
       PH_OTHER = 7 };

constexpr uint32_t NONE32 = 0xFFFFFFFFu;


// Literal state byte lv[code] (code = v << 1 | negative): free 1, true 8,
// false 0.  The sum of a clause's bytes: bits 0-2 = free occurrences (REF.py's
// len(c)), bits 3-7 = 8 x true occurrences (!= 0: the reference dropped the
// clause); a unit clause's literal is its one free slot.  Code 0 (variable 0,
// positive) pads short clauses and is pinned false; code 1 is pinned true and
// fills the dummy clauses that round the clause array up to whole 64-clause
// chunks.  One byte per code (not a word) packs 4 codes per LDS dword: a
// gather of 32 random codes of n=100 touches at most 2 dwords per bank.
constexpr uint32_t LV_TRUE = 8u, LV_FALSE = 0u, LV_FREE = 1u;
constexpr uint32_t CODE_PAD = 0u, CODE_DUMMY = 1u;
__device__ __forceinline__ bool sum_true(uint32_t s) { return (s & 0xF8u) != 0u; }
__device__ __forceinline__ bool sum_open(uint32_t s) { return s < 8u; }
__device__ __forceinline__ uint32_t sum_nfree(uint32_t s) { return s & 7u; }

template <int K>
struct Pack;
template <>
struct Pack<3> {
    using W = uint32_t;
    static constexpr int BITS = 10;
    static constexpr int MAXV = 511;
    static constexpr int UNROLL = 7;
};
template <>
struct Pack<5> {
    using W = uint64_t;
    static constexpr int BITS = 12;
    static constexpr int MAXV = 2047;
    static constexpr int UNROLL = 2;
};

// Clause slots of an instance of m clauses: whole 64-clause chunks (padding a
// partial unroll group with dummy chunks was measured slower -- the kernel is
// LDS-throughput bound, not latency bound).
__host__ __device__ __forceinline__ int padded_clauses(int m) { return (m + 63) & ~63; }

template <int K>
__device__ __forceinline__ uint32_t field(typename Pack<K>::W w, int j) {
    return (uint32_t)(w >> (Pack<K>::BITS * j)) & ((1u << Pack<K>::BITS) - 1u);
}

struct ScanLayout {
    uint32_t cls, lv, ts, cnt, first, trail, fvar, ftrail, scratch, occ_off, bm, bytes;
    int32_t mcap, ncap, nw;   // nw: 32-clause words of the unit bitmap (incremental kernel)
};

struct ScanArgs {
    const int32_t *inst_clause_begin, *clause_lit_begin, *lits, *inst_nvars;
    int32_t num_instances, sol_cap, sol_stride;
    int64_t max_solutions, node_limit;
    uint64_t time_limit_ticks;
    int32_t *status;
    int64_t *counters;
    int32_t *sol_len, *sol_lits, *root_len, *root_lits;
    uint32_t *work_counter;
    uint16_t *occ;      // per-wave HBM/L2 scratch, occ_cap entries each: the incremental kernel's
    int32_t occ_cap;    // occurrence lists [0, occ_lists), then the snapshot entries past snap_lds
    ScanLayout lay;
    // branch splitting (see "Splitting the tail" below); nullptr: off.  Its
    // geometry lives in device memory, not in kernel arguments: the node loop
    // is SGPR-bound, and only this pointer stays live across it.
    struct SplitCfg *split;
    // (last: the fields above keep their kernel-argument offsets -- the node
    // loop's SGPR allocation is sensitive to them)
    int32_t occ_lists;
    uint32_t snap_lds;   // snapshot entries in LDS (16-bit codes; see snap_put)
};

// C: the type of a literal code / variable / trail position in the trail,
// decision frames and snapshot -- uint8_t for the 256-B size class (n <= 127),
// which halves those arrays, else uint16_t.
template <int K, typename C>
struct SLds {
    static constexpr uint32_t PHASE_BIT = 1u << (8 * sizeof(C) - 1);   // fvar: the False branch runs
    typename Pack<K>::W *cls;   // [mcap rounded up to 64]  packed literal codes per clause
    uint8_t *lv;                // [2(ncap+1)]  literal state bytes
    uint32_t *ts;               // [ncap+1]  snapshot index of the assignment in the running batch
    uint32_t *cnt;              // [2(ncap+1)]  free occurrences in active clauses, per literal code
    uint32_t *first;            // [ncap+1]  flags / first positions of choose()'s scans (the fixed
                                //           kernel: the ts array, see dpll_fixed_kernel)
    C *trail;                   // [ncap+1]  assignment order (literal codes) == dict insertion order
    C *fvar;                    // [ncap+1]  decision frames: var | PHASE_BIT once False runs
    C *ftrail;                  // [ncap+1]  trail length before the decision
    C *snap;                    // scratch:  unit-clause snapshot (propagation), entries [0, scap)
    uint32_t *plist;            // scratch:  pure literals (analysis), aliases snap: their first positions,
                                //           or (plist_vars) their variables as C, whose positions are
                                //           S.first[v] - 1
    C *snapg;                   // global:   snapshot entries [scap, m] (16-bit codes only)
    uint32_t scap;
    // incremental kernel only
    uint16_t *occ_off;          // [2(ncap+1)+1]  start of each literal code's occurrence list in `occ`
    uint2 *bm;                  // [nw]  unit bitmap of the round: .x one bit per clause (32 clauses
                                //       per word), .y units before the word once the round is scanned
    const uint16_t *occ;        // global: clause indices holding each literal code (distinct per clause)
};

// literal `code` becomes true: one 2-byte store sets both literals of its variable
__device__ __forceinline__ void lv_assign(uint8_t *lv, uint32_t code) {
    // two byte stores (LDS issue) instead of one 16-bit store of a selected value (VALU issue)
    lv[code] = (uint8_t)LV_TRUE;
    lv[code ^ 1u] = (uint8_t)LV_FALSE;
}
__device__ __forceinline__ void lv_clear(uint8_t *lv, uint32_t v) {
    *(uint16_t *)(lv + 2 * v) = (uint16_t)(LV_FREE | (LV_FREE << 8));
}
__device__ __forceinline__ bool var_free(const uint8_t *lv, uint32_t v) { return (lv[2 * v] & 1u) != 0u; }

// The hot LDS accesses by kind: the product forms, or (attribution builds,
// never the product) each issued twice -- see dpll_scan_access.h.
#include "dpll_scan_access.h"

// Per-literal-code counters (the counting pass, the occurrence-list build).
// One word per code, except for 3-literal clauses with 16-bit codes (n = 128 ..
// 511): the two codes of a variable share a word, code 2v in the low half (a
// count is at most the instance's literal count, which the scan kernel bounds
// by 65,535: dpll_scan_eligible, run_queue), which halves the array --
// uf250 fits 15 searches per CU instead of 13 (+10 %).  (5-SAT n=200 gains no
// residency from it and pays the packing's shifts: one word per code there.)
// The pure-literal list holds variables (16 bits) instead of positions (32)
// for 3-literal clauses with 16-bit codes: with the snapshot's LDS part at 256
// entries it halves the wave's scratch, and uf250 fits 16 searches per CU
// instead of 15 (+10 % node-capped, profiles/r06/uf250_occupancy_ab.txt).
// (5-SAT n=200 stays at 4 per CU whatever the scratch: positions there.)
template <int K, typename C>
constexpr bool plist_vars() { return sizeof(C) == 2 && K == 3; }
template <int K, typename C>
constexpr bool cnt_packed() {
#ifdef SATMI_CNT_PACK_ALL   // A/B variant: byte codes (the bench kernel) packed too
    return K == 3;
#else
    return sizeof(C) == 2 && K == 3;
#endif
}
template <int K, typename C>
__device__ __forceinline__ void cnt_inc(const SLds<K, C> &S, uint32_t code, uint32_t inc) {
    if constexpr (!cnt_packed<K, C>()) atomicAdd(&S.cnt[code], inc);
    else atomicAdd(&S.cnt[code >> 1], inc << ((code & 1u) << 4));
}
template <int K, typename C>
__device__ __forceinline__ uint32_t cnt_fetch_inc(const SLds<K, C> &S, uint32_t code) {   // the count before
    if constexpr (!cnt_packed<K, C>()) {
        return atomicAdd(&S.cnt[code], 1u);
    } else {
        const uint32_t sh = (code & 1u) << 4;
        return (atomicAdd(&S.cnt[code >> 1], 1u << sh) >> sh) & 0xFFFFu;
    }
}
template <int K, typename C>
__device__ __forceinline__ uint32_t cnt_get(const SLds<K, C> &S, uint32_t code) {
    if constexpr (!cnt_packed<K, C>()) return S.cnt[code];
    else return (S.cnt[code >> 1] >> ((code & 1u) << 4)) & 0xFFFFu;
}
template <int K, typename C>
__device__ __forceinline__ uint2 cnt_pair(const SLds<K, C> &S, uint32_t v) {   // codes 2v, 2v + 1
    if constexpr (!cnt_packed<K, C>()) {
        return ((const uint2 *)S.cnt)[v];
    } else {
        const uint32_t w = S.cnt[v];
        return make_uint2(w & 0xFFFFu, w >> 16);
    }
}
template <int K, typename C>
__device__ __forceinline__ void cnt_clear_var(const SLds<K, C> &S, uint32_t v) {
    if constexpr (!cnt_packed<K, C>()) ((uint2 *)S.cnt)[v] = make_uint2(0u, 0u);
    else S.cnt[v] = 0u;
}


// Apply f(c, w, x) to every clause c (w its packed word, x[j] the state byte of
// its slot j), one 64-clause chunk per lane step; the loads of U chunks are
// issued before any is used.  mpad is a multiple of 64 (dummy clauses are
// always satisfied).
template <int K, int U, typename C, typename F>
__device__ __forceinline__ void chunk_group(const SLds<K, C> &S, int c0, F &&f) {
    using W = typename Pack<K>::W;
    const int ln = lane_id();
    W w[U];
    uint32_t x[U][K];
#pragma unroll
    for (int u = 0; u < U; ++u) w[u] = S.cls[c0 + 64 * u + ln];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < K; ++j) x[u][j] = lv_get(S, field<K>(w[u], j));
#pragma unroll
    for (int u = 0; u < U; ++u) f(c0 + 64 * u + ln, w[u], x[u]);
}

// Groups of U chunks, then (U > 4) groups of 4, then single chunks: n=100's 7
// chunks are one group of 7, n=50's 4 chunks one group of 4.
template <int K, int U, typename C, typename F>
__device__ __forceinline__ void for_chunks(const SLds<K, C> &S, int mpad, F &&f) {
    using W = typename Pack<K>::W;
    const int ln = lane_id();
    int c0 = 0;
    for (; c0 + 64 * U <= mpad; c0 += 64 * U) chunk_group<K, U>(S, c0, f);
    if constexpr (U > 4)
        for (; c0 + 64 * 4 <= mpad; c0 += 64 * 4) chunk_group<K, 4>(S, c0, f);
    for (; c0 < mpad; c0 += 64) {
        const W w = S.cls[c0 + ln];
        uint32_t x[K];
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = lv_get(S, field<K>(w, j));
        f(c0 + ln, w, x);
    }
}

template <int K>
__device__ __forceinline__ uint32_t clause_sum(const uint32_t (&x)[K]) {
    uint32_t s = x[0];
#pragma unroll
    for (int j = 1; j < K; ++j) s += x[j];
    return s;
}

// The literal of a unit clause: its one free slot.  (A unit clause has no
// true slot, so each state byte is 0 or 1: for K = 3 the free slot's field
// offset is 10 x[1] + 20 x[2], one extract.)
template <int K>
__device__ __forceinline__ uint32_t unit_code(typename Pack<K>::W w, const uint32_t (&x)[K]) {
    if constexpr (K == 3) {
        return __builtin_amdgcn_ubfe((uint32_t)w, x[1] * (uint32_t)Pack<3>::BITS + x[2] * (2u * Pack<3>::BITS),
                                     Pack<3>::BITS);
    } else {
        uint32_t code = field<K>(w, 0);
#pragma unroll
        for (int j = 1; j < K; ++j)
            if (x[j] & 1u) code = field<K>(w, j);
        return code;
    }
}

// Snapshot stamps ts[v]: epoch << 16 | (0xFFFF - k) for the variable of
// snapshot entry k.  Every snapshot gets a fresh epoch, so stamps never need
// clearing: an older epoch is smaller, and atomicMax keeps the first entry of
// a variable (the smallest k) within the current one.
constexpr uint32_t EPOCH_LIMIT = 0xFFFFu - 4096u;   // > rounds of one propagate call (<= n+1 <= 2048)
__device__ __forceinline__ uint32_t stamp(uint32_t ep, uint32_t k) { return ((ep << 16) | 0xFFFFu) - k; }   // k <= 0xFFFF
__device__ __forceinline__ uint32_t stamp_index(uint32_t st) { return 0xFFFFu - (st & 0xFFFFu); }

// Snapshot entry k.  With byte codes (n <= 127) the whole snapshot is in LDS;
// with 16-bit codes the first `scap` entries are (a few hundred: a round finds
// tens of units), the rest of a larger snapshot goes to the wave's HBM scratch,
// so the LDS does not hold m entries that are almost never used (5-SAT n=200:
// 8.4 KB of 47 KB per wave, the difference between 3 and 4 waves per CU).
template <int K, typename C>
__device__ __forceinline__ void snap_put(const SLds<K, C> &S, uint32_t k, uint32_t code) {
    if constexpr (sizeof(C) == 1) {
        S.snap[k] = (C)code;
    } else {
        if (k < S.scap) S.snap[k] = (C)code;
        else S.snapg[k - S.scap] = (C)code;
    }
}
template <int K, typename C>
__device__ __forceinline__ uint32_t snap_get(const SLds<K, C> &S, uint32_t k) {
    if constexpr (sizeof(C) == 1) return S.snap[k];
    else return k < S.scap ? (uint32_t)S.snap[k] : (uint32_t)S.snapg[k - S.scap];
}
// before a snapshot of nu entries is read back: the HBM part written by other
// lanes of this wave is complete (the occurrence lists' recipe)
template <int K, typename C>
__device__ __forceinline__ void snap_ready(const SLds<K, C> &S, int nu) {
    if constexpr (sizeof(C) == 2)
        if ((uint32_t)nu > S.scap) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
}

// Scan for unit_propagate: the unit-clause snapshot (REF.py:143), in clause
// order, into S.snap, each entry's variable stamped with epoch `ep` (the first
// occurrence of a variable keeps the smallest index: REF.py:149-152's
// `if var in a`).  *empty_at: INT_MAX if no clause is empty, else the snapshot
// index (within the batch of epoch `bep` just assigned) whose assignment
// emptied a clause first -- an emptied clause was emptied by the
// latest-stamped of its literals (REF.py:161-162), found in the same pass.
template <int K, typename C>
__device__ int scan_units(const SLds<K, C> &S, int mpad, uint32_t ep, uint32_t bep, int *empty_at) {
    using W = typename Pack<K>::W;
    const uint64_t lt = lanemask_lt();
    int nu = 0;
    int e = INT_MAX;
    for_chunks<K, Pack<K>::UNROLL>(S, mpad, [&](int c, W, const uint32_t(&x)[K]) {
        const uint32_t s = clause_sum<K>(x);
        const bool open = !sum_true(s);
        const uint32_t nf = sum_nfree(s);
        if (open && nf == 0u) {   // rare: only in a conflicting round
            const W w = S.cls[c];
            int t = -1;
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const uint32_t code = field<K>(w, j);
                const uint32_t st = code > CODE_DUMMY ? S.ts[code >> 1] : 0u;
                if ((st >> 16) == bep) t = max(t, (int)stamp_index(st));
            }
            e = min(e, t);
        }
        const bool unit = open && nf == 1u;
        const uint64_t mk = __ballot(unit);
        if (unit) {
            const uint32_t k = (uint32_t)nu + (uint32_t)__popcll(mk & lt);
            const uint32_t code = unit_code<K>(S.cls[c], x);   // re-read: keeps U words out of VGPRs
            snap_put(S, k, code);
            ts_stamp(S, code >> 1, stamp(ep, k));
        }
        nu += __popcll(mk);
    });
    wave_sync();
    *empty_at = __ballot(e != INT_MAX) ? wave_min_i32(e) : INT_MAX;
    return nu;
}

// Incremental form of scan_units for every round after the first: the next
// snapshot can only hold clauses that lost a literal in the batch just
// assigned, trail[rs, tl) -- every unit of the previous snapshot is now
// satisfied (or the round ended in a conflict), and no other clause changed.
// So only the clauses on the occurrence lists of the batch's negated literals
// are read (64 per wave step, gathered from the HBM/L2-resident lists).  Unit
// clauses set their bit in a clause bitmap; the bitmap's prefix popcounts give
// each unit its snapshot index, i.e. REF.py:143's clause order, with a clause
// reached twice counted once.  Emptied clauses are found among the same
// touched clauses (an emptied clause lost its last literal in this batch).
// Same results as scan_units, bit for bit.
// Emptied-clause search of one touched clause (REF.py:161-162): the snapshot
// index in batch epoch `bep` of its latest-stamped literal, -1 if none.
template <int K, typename C>
__device__ __forceinline__ int emptier(const SLds<K, C> &S, typename Pack<K>::W w, uint32_t bep) {
    int tt = -1;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const uint32_t code = field<K>(w, j);
        const uint32_t ts = S.ts[code >> 1];   // predicated: padding codes read variable 0's word
        const uint32_t st = code > CODE_DUMMY ? ts : 0u;
        tt = (st >> 16) == bep ? max(tt, (int)stamp_index(st)) : tt;
    }
    return tt;
}

// A round whose touched clauses fit one wave step ranks at most two unit
// clauses by register comparisons; more go through the clause bitmap, which
// measured faster than ranking 3-8 units by readlane loops
// (profiles/r04/steps/dpll_fast_units_threshold_ab.txt).
constexpr int FAST_UNITS = 2;
constexpr int FAST_BATCH = 16;

template <int K, typename C>
__device__ int inc_units(const SLds<K, C> &S, int nw, int rs, int tl, uint32_t ep, uint32_t bep, int *empty_at,
                         int *pre, PhaseClock &ph) {
    using W = typename Pack<K>::W;
    const int ln = lane_id();
    ph.count(0);
    ph.count(7, (uint64_t)(tl - rs));
    // fast path: a batch of at most FAST_BATCH literals (lanes 0..15; larger
    // batches are rare and take the general path below)
    if (__builtin_expect(tl - rs <= FAST_BATCH, 1)) {
        // lane b: the b-th batch literal's negation and its occurrence list
        // predicated (no exec-mask branch): lanes past the batch read entry rs
        const bool inb = ln < tl - rs;
        const uint32_t x = (uint32_t)S.trail[inb ? rs + ln : rs] ^ 1u;
        const int o0 = S.occ_off[x], o1 = S.occ_off[x + 1];
        const int ob = inb ? o0 : 0, len = inb ? o1 - o0 : 0;
        // the batch sits in lanes 0..15: the row scan covers it
        const int incl = row_incl_scan(len);
        const int excl = incl - len;
        const int delta = ob - excl;
        const int total = __builtin_amdgcn_readlane(incl, 15);
        if (__builtin_expect(total <= 64, 1)) {
            ph.count(1);
            // one touched clause per lane
            int d = __builtin_amdgcn_readlane(delta, 0);
            if (tl - rs > 1)   // one batch literal: lane 0's list is the whole range
            for (int b = 1; b < tl - rs; ++b) {
                const int eb = __builtin_amdgcn_readlane(excl, b);
                const int db = __builtin_amdgcn_readlane(delta, b);
                d = ln >= eb ? db : d;
            }
            const bool valid = ln < total;
            const uint32_t c = S.occ[(uint32_t)(valid ? d + ln : 0)];   // 32-bit offset from the wave's base
            const W w = cls_at(S, c);
            uint32_t x[K];
#pragma unroll
            for (int j = 0; j < K; ++j) x[j] = lv_get(S, field<K>(w, j));
            const uint32_t sv = valid ? clause_sum<K>(x) : 0xFFu;
            const bool empty = sv == 0u;
            if (__builtin_expect(__ballot(empty) != 0ull, 0)) {
                ph.count(2);
                const int et = emptier<K>(S, w, bep);   // every lane: no exec-mask branch
                const int e = empty ? et : INT_MAX;
                *empty_at = wave_min_i32(e);
                return 0;
            }
            *empty_at = INT_MAX;
            const bool unit = sv == 1u;
            const uint64_t um = __ballot(unit);
            const int nun = __popcll(um);
            ph.count(4, (uint64_t)nun);
            ph.count(nun == 0 ? 10 : nun == 1 ? 11 : nun == 2 ? 12 : nun <= 8 ? 13 : 6, nun <= 8 ? 1 : 0);
            if (__builtin_expect(nun <= FAST_UNITS, 1)) {
                ph.count(3);
                // a clause reached from two batch literals is one snapshot entry
                uint64_t dm = um;
                int rank = 0;
                // The next batch is assigned right here -- REF.py:146-155 on a
                // snapshot of at most two entries: both are assigned unless they
                // name one variable (the first wins) -- so the next round skips
                // the snapshot's write-back and its stamp pass.
                const uint32_t code = unit_code<K>(w, x);
                bool keep = unit;
                int nkeep = nun;
                if (nun == 2) {   // lanes u0 < u1
                    const int u0 = __builtin_ctzll(um), u1 = 63 - __builtin_clzll(um);
                    const uint32_t c0 = (uint32_t)__builtin_amdgcn_readlane((int)c, u0);
                    const uint32_t c1 = (uint32_t)__builtin_amdgcn_readlane((int)c, u1);
                    const uint32_t v0 = (uint32_t)__builtin_amdgcn_readlane((int)code, u0) >> 1;
                    const uint32_t v1 = (uint32_t)__builtin_amdgcn_readlane((int)code, u1) >> 1;
                    dm = c0 == c1 ? 1ull << u0 : um;   // a duplicate keeps lane u0 only
                    rank = ln == u0 ? (c1 < c0 ? 1 : 0) : (c0 < c1 ? 1 : 0);
                    const bool one = (c0 == c1) | (v0 == v1);   // one entry is assigned: the first in clause order
                    keep = unit & (!one | (rank == 0));
                    nkeep = one ? 1 : 2;
                }
                if (keep) {
                    S.trail[tl + rank] = (C)code;
                    lv_assign(S.lv, code);
                    S.ts[code >> 1] = stamp(ep, (uint32_t)rank);
                }
                wave_sync();
                *pre = nkeep;
                return __popcll(dm);
            }
            // more units than the register ranking takes: the touched clauses
            // are already in the lanes (one step), so they are placed in clause
            // order through the bitmap right here, not scanned again below (a
            // clause reached from two batch literals sets one bit; its lanes
            // write the same snapshot entry and stamp)
            if (unit) atomicOr(&S.bm[c >> 5].x, 1u << (c & 31u));
            wave_sync();
            int nu = 0;
            if (nw <= 64) {   // up to 2,048 clauses: one prefix scan
                const uint32_t bits = ln < nw ? S.bm[ln].x : 0u;
                const int pc = __popc(bits);
                const int in = wave_incl_scan(pc);
                if (ln < nw) S.bm[ln].y = (uint32_t)(in - pc);
                nu = lane63(in);
            } else
            for (int w0 = 0; w0 < nw; w0 += 64) {
                const int wi = w0 + ln;
                const uint32_t bits = wi < nw ? S.bm[wi].x : 0u;
                const int pc = __popc(bits);
                const int in = wave_incl_scan(pc);
                if (wi < nw) S.bm[wi].y = (uint32_t)(nu + in - pc);
                nu += lane63(in);
            }
            wave_sync();
            if (unit) {
                const uint2 pb = S.bm[c >> 5];
                const uint32_t k = pb.y + (uint32_t)__popc(pb.x & ((1u << (c & 31u)) - 1u));
                const uint32_t code = unit_code<K>(w, x);
                snap_put(S, k, code);
                ts_stamp(S, code >> 1, stamp(ep, k));
                // clean bitmap for the next round: only the words units set (a
                // wave's LDS operations run in order, so every lane of the word
                // has read it above)
                S.bm[c >> 5].x = 0u;
            }
            wave_sync();
            ph.count(6);
            return nu;
        }
    }
    ph.count(5);
    ph.count(tl - rs > FAST_BATCH ? 8 : 9);
    int e = INT_MAX;
    int passes = 0;
    bool unit = false;          // this lane found a unit clause (valid when one pass covered all touched clauses)
    uint32_t uc = 0, ucode = 0;
    for (int i0 = rs; i0 < tl; i0 += 64) {
        // lane b: the b-th batch literal's negation and its occurrence list
        const int i = i0 + ln;
        int ob = 0, len = 0;
        if (i < tl) {
            const uint32_t x = (uint32_t)S.trail[i] ^ 1u;
            ob = S.occ_off[x];
            len = (int)S.occ_off[x + 1] - ob;
        }
        const int incl = wave_incl_scan(len);
        const int excl = incl - len;
        const int delta = ob - excl;   // touched index t of list b reads occ[delta_b + t]
        const int total = lane63(incl);
        const int nb = min(64, tl - i0);
        for (int t0 = 0; t0 < total; t0 += 64) {
            const int t = t0 + ln;
            int d = 0;
            for (int b = 0; b < nb; ++b) {   // segments are in order: the last that starts at or before t owns it
                const int eb = __builtin_amdgcn_readlane(excl, b);
                const int db = __builtin_amdgcn_readlane(delta, b);
                d = t >= eb ? db : d;
            }
            ++passes;
            if (t < total) {
                const uint32_t c = S.occ[d + t];
                const W w = cls_at(S, c);
                uint32_t x[K];
#pragma unroll
                for (int j = 0; j < K; ++j) x[j] = lv_get(S, field<K>(w, j));
                const uint32_t s = clause_sum<K>(x);
                if (!sum_true(s)) {
                    const uint32_t nf = sum_nfree(s);
                    if (nf == 0u) {   // emptied in this batch: by its latest-stamped literal
                        e = min(e, emptier<K>(S, w, bep));
                    } else if (nf == 1u) {
                        atomicOr(&S.bm[c >> 5].x, 1u << (c & 31u));
                        unit = true;
                        uc = c;
                        ucode = unit_code<K>(w, x);
                    }
                }
            }
        }
    }
    wave_sync();
    const int emp = __ballot(e != INT_MAX) ? wave_min_i32(e) : INT_MAX;
    *empty_at = emp;
    if (emp != INT_MAX) {   // conflict: the snapshot is not needed, only a clean bitmap
        for (int w = ln; w < nw; w += 64) S.bm[w].x = 0u;
        wave_sync();
        return 0;
    }
    // prefix popcounts of the bitmap
    int nu = 0;
    for (int w0 = 0; w0 < nw; w0 += 64) {
        const int w = w0 + ln;
        const uint32_t bits = w < nw ? S.bm[w].x : 0u;
        const int pc = __popc(bits);
        const int in = wave_incl_scan(pc);
        if (w < nw) S.bm[w].y = (uint32_t)(nu + in - pc);
        nu += lane63(in);
    }
    wave_sync();
    if (passes <= 1) {
        // one pass held every touched clause: each unit lane places its clause
        if (unit) {
            const uint2 p = S.bm[uc >> 5];
            const uint32_t k = p.y + (uint32_t)__popc(p.x & ((1u << (uc & 31u)) - 1u));
            snap_put(S, k, ucode);
            ts_stamp(S, ucode >> 1, stamp(ep, k));
        }
    } else {
        // long batch: walk the bitmap word by word, re-deriving each unit literal
        for (int w = ln; w < nw; w += 64) {
            const uint2 p = S.bm[w];
            uint32_t bits = p.x, k = p.y;
            while (bits) {
                const uint32_t c = ((uint32_t)w << 5) | (uint32_t)__builtin_ctz(bits);
                bits &= bits - 1u;
                const W wd = S.cls[c];
                uint32_t x[K];
#pragma unroll
                for (int j = 0; j < K; ++j) x[j] = lv_get(S, field<K>(wd, j));
                const uint32_t code = unit_code<K>(wd, x);
                snap_put(S, k, code);
                ts_stamp(S, code >> 1, stamp(ep, k));
                ++k;
            }
        }
    }
    wave_sync();
    for (int w = ln; w < nw; w += 64) S.bm[w].x = 0u;   // clean bitmap for the next round
    return nu;
}

// The epoch of a decision snapshot.  No stamp is live between propagate calls,
// so this is where the 16-bit epoch wraps: all stamps are reset to epoch 0.
template <int K, typename C>
__device__ uint32_t next_decision_epoch(const SLds<K, C> &S, int n, uint32_t ep) {
    if (ep < EPOCH_LIMIT) return ep + 1;
    for (int v = lane_id(); v <= n; v += 64) S.ts[v] = 0u;
    wave_sync();
    return 1;
}

// unit_propagate (REF.py:139-165) from the snapshot S.snap[0, nu), stamped
// with epoch `ep` (the last epoch used; each scan takes the next).  Returns
// true on conflict; `tl` ends where the reference stops (the assignments it
// made, including the one that emptied a clause).  `dec`: the first batch is
// the decision literal, which REF.py's counters do not count as a propagation.
template <int K, bool INC, typename C>
__device__ bool propagate(const SLds<K, C> &S, int mpad, int &tl, int nu, bool dec, uint32_t &ep, uint32_t &props,
                          uint32_t &rounds, PhaseClock &ph) {
    const int ln = lane_id();
    int e = INT_MAX;   // set: the round that emptied a clause (handled after the loop)
    int rs = tl;
    // the decision literal (the first batch's first entry, always assigned or
    // kept) is not a propagation in REF.py's counters: taken off once here
    props -= dec ? 1u : 0u;
    ph.count(14);
    int pre = -1;   // >= 0: the unit scan assigned the next batch itself (this many entries)
    while (nu > 0) {
        ++rounds;
        rs = tl;
        const uint32_t bep = ep;   // the batch's epoch
        if (pre >= 0) {
            tl += pre;
        } else {
        int k0 = 0;
        snap_ready(S, nu);
        do {   // nu > 0: at least one step
            ph.count(15);
            const int k = k0 + ln;
            // lanes past nu read entry 0 (its variable is stamped with index 0
            // != k: never first).  Stale entries past nu are not safe to read:
            // an epoch can repeat across rounds, and so can (stamp, index).
            const uint32_t code = snap_get(S, (uint32_t)(k < nu ? k : 0));
            const uint32_t v = code >> 1;
            // (one compare: its ballot folds into the v_cmp)
            const bool first = ts_first(S, v) == stamp(bep, (uint32_t)k);
            const uint64_t mk = __ballot(first);
            if (first) {   // trail slot: tl + the first entries on lower lanes (k order)
                S.trail[__builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32),
                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)mk, (uint32_t)tl))] = (C)code;
                lv_assign(S.lv, code);
            }
            dup_assign_store(S, first, code);
            tl += __popcll(mk);
            k0 += 64;
        } while (k0 < nu);
        wave_sync();
        }
        ph.mark(PH_ASSIGN);
        const int nassign = tl - rs;
        pre = -1;
        const int nu_next = INC ? inc_units<K>(S, (mpad + 31) >> 5, rs, tl, ++ep, bep, &e, &pre, ph)
                                : scan_units<K>(S, mpad, ++ep, bep, &e);
        ph.mark(PH_UNITS);
        if (__builtin_expect(e != INT_MAX, 0)) break;
        props += nassign;   // >= 1: a snapshot's first entry is always assigned (`changed`, REF.py:141-142)
        nu = nu_next;
    }
    if (e == INT_MAX) return false;
    // the reference stopped at snapshot index e of the last batch, trail[rs,
    // tl): keep the prefix stamped <= e (the batch is in stamp order)
    int keep = 0;
    for (int i0 = rs; i0 < tl; i0 += 64) {
        const int i = i0 + ln;
        const bool p = i < tl && (int)stamp_index(S.ts[S.trail[i] >> 1]) <= e;
        keep += __popcll(__ballot(p));
    }
    const int cut = rs + keep;
    for (int i = cut + lane_id_here(); i < tl; i += 64) lv_clear(S.lv, S.trail[i] >> 1);
    wave_sync();
    tl = cut;
    props += keep;   // >= 1: the batch's first entry (stamp index 0) is kept
    ph.mark(PH_CONFLICT);
    return true;
}

// literal_sign / var_counts scan (REF.py:174-179, :198-203): every free
// occurrence in an active clause is counted per literal code.  Returns whether
// any clause is active (none: REF.py:170-171).  In an active clause a slot's
// state byte is 1 (free) or 0 (false; a true slot would make the clause
// inactive), which is the slot's count increment as it is: the atomic runs
// for every slot with no branch and no arithmetic (padding adds 0 to code
// 0, never read).  The dict order
// (first positions) is not tracked here: only the branch candidates and the
// pure literals need it, and choose() finds those afterwards (a per-slot
// atomicMin of the first position here cost 21 LDS atomics per node, most of
// the kernel's bank-conflict cycles).
template <int K, typename C>
__device__ int scan_counts(const SLds<K, C> &S, int mpad) {
    using W = typename Pack<K>::W;
    uint64_t any = 0;   // only "no active clause" matters: OR the ballots (one scalar op per chunk)
    for_chunks<K, Pack<K>::UNROLL>(S, mpad, [&](int, W w, const uint32_t(&x)[K]) {
        const bool act = sum_open(clause_sum<K>(x));
        any |= __ballot(act);
        if (act) {
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const uint32_t code = field<K>(w, j);
                cnt_inc(S, code, x[j]);
                dup_count(S, code);
            }
        }
    });
    wave_sync();
    return any != 0ull;
}

// Positions in the reduced formula: c << 3 | slot, in REF.py's iteration
// order (clauses in order, literals in order), over the free literals of the
// active clauses.  S.first[v] != 0 flags variable v for the two scans below.
//
// The first flagged position (chunks in order, the scan stops at the first
// chunk with a hit): the first flagged key in dict order.
template <int K, typename C>
__device__ uint32_t first_flagged(const SLds<K, C> &S, int mpad) {
    using W = typename Pack<K>::W;
    const int ln = lane_id();
    for (int c0 = 0; c0 < mpad; c0 += 64) {
        const int c = c0 + ln;
        const W w = S.cls[c];
        uint32_t x[K], f[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            x[j] = lv_get(S, field<K>(w, j));
            f[j] = S.first[field<K>(w, j) >> 1];
        }
        const bool act = !sum_true(clause_sum<K>(x));
        uint32_t pos = NONE32;
#pragma unroll
        for (int j = K - 1; j >= 0; --j)
            pos = (act & ((x[j] & 1u) != 0u) & (f[j] != 0u)) ? (((uint32_t)c << 3) | (uint32_t)j) : pos;
        const uint64_t hit = __ballot(pos != NONE32);
        if (hit) return (uint32_t)__builtin_amdgcn_readlane((int)pos, __builtin_ctzll(hit));
    }
    return NONE32;   // unreachable: a flagged variable occurs free in an active clause
}

// First positions of the `npure` flagged (pure) variables: S.first[v] = its
// first position + 1 (flag NONE32 before; 0 = not pure).  Chunks in order
// until every pure variable has been met once.
template <int K, typename C>
__device__ void first_of_pures(const SLds<K, C> &S, int mpad, int npure) {
    using W = typename Pack<K>::W;
    const int ln = lane_id();
    int found = 0;
    for (int c0 = 0; c0 < mpad && found < npure; c0 += 64) {
        const int c = c0 + ln;
        const W w = S.cls[c];
        uint32_t x[K], f[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            x[j] = lv_get(S, field<K>(w, j));
            f[j] = S.first[field<K>(w, j) >> 1];
        }
        const bool act = !sum_true(clause_sum<K>(x));
#pragma unroll
        for (int j = 0; j < K; ++j) {
            bool met = false;
            if (act & ((x[j] & 1u) != 0u) & (f[j] != 0u))
                met = atomicMin(&S.first[field<K>(w, j) >> 1], (((uint32_t)c << 3) | (uint32_t)j) + 1u) == NONE32;
            found += __popcll(__ballot(met));
        }
    }
    wave_sync();
}

struct Choice {
    int npure;
    uint32_t best_var;   // 0 = no unassigned variable occurs (REF.py:205)
};

// pure_literals (REF.py:181-184) into plist (first positions), else the
// branching variable: max(var_counts.items(), key=count), the first maximal
// key in dict order (REF.py:208).  Clears cnt for the next scan.  The
// variables are read twice -- the largest count and the pure count, then the
// flags of the position scans -- and a position scan runs only when the
// order matters: several variables share the largest count (the first of
// them in dict order wins), or there are pure literals (their order is the
// assignment's dict order).
template <int K, typename C>
__device__ Choice choose(const SLds<K, C> &S, int n, int mpad) {
    const int ln = lane_id_here();   // per call: lane-invariant addresses hoisted out of the node loop spill
    const uint64_t lt = lanemask_lt();
    int npure = 0;
    uint32_t lmax = 0;
    // predicated (no exec-mask branches): lanes past n read variable n's words
    auto count_step = [&](int v0) {
        const int v = v0 + ln;
        const uint32_t vc = (uint32_t)min(v, n);
        const bool live = (v <= n) & var_free(S.lv, vc);
        const uint2 c = cnt_pair(S, vc);   // the counts of codes 2v, 2v + 1
        const uint32_t p = c.x, q = c.y;
        lmax = live ? max(lmax, p + q) : lmax;
        npure += __popcll(__ballot(live & ((p + q) != 0u) & ((p == 0u) | (q == 0u))));
    };
    if constexpr (sizeof(C) == 1) {   // byte trail codes: n <= 127, two steps at most, no loop
        if (n >= 1) count_step(1);
        if (n >= 65) count_step(65);
    } else {
        for (int v0 = 1; v0 <= n; v0 += 64) count_step(v0);
    }
    const uint32_t maxc = wave_max_u32(lmax);
    int ncand = 0;
    uint32_t cvar = 0;   // the first candidate by variable index (the winner when it is the only one)
    // flags for the position scans (lanes past n flag variable 0: never flagged), counts cleared
    auto flag_step = [&](int v0) {
        const int v = v0 + ln;
        const uint32_t vc = (uint32_t)min(v, n);
        const bool live = (v <= n) & var_free(S.lv, vc);
        const uint2 c = cnt_pair(S, vc);
        const uint32_t p = c.x, q = c.y;
        const bool pure = live & ((p + q) != 0u) & ((p == 0u) | (q == 0u));
        const bool cand = live & (p + q == maxc);
        const uint64_t cm = __ballot(cand);
        cvar = (ncand == 0 && cm) ? (uint32_t)v0 + (uint32_t)__builtin_ctzll(cm) : cvar;
        ncand += __popcll(cm);
        const uint32_t vw = v <= n ? vc : 0u;
        S.first[vw] = npure ? (pure ? NONE32 : 0u) : (cand ? 1u : 0u);
        cnt_clear_var(S, vw);   // cleared for the next scan
    };
    if constexpr (sizeof(C) == 1) {
        if (n >= 1) flag_step(1);
        if (n >= 65) flag_step(65);
    } else {
        for (int v0 = 1; v0 <= n; v0 += 64) flag_step(v0);
    }
    cnt_clear_var(S, 0u);   // variable 0: the padding slots' counts (never read)
    S.first[0] = 0u;
    wave_sync();
    uint32_t best = 0;
    if (npure > 0) {
        first_of_pures<K>(S, mpad, npure);
        // plist in variable order; assign_pures ranks the entries by position
        int k = 0;
        auto collect = [&](int v0) {
            const int v = v0 + ln;
            const uint32_t f = v <= n ? S.first[v] : 0u;
            const bool pure = f != 0u;
            const uint64_t mk = __ballot(pure);
            if constexpr (!plist_vars<K, C>()) {
                if (pure) S.plist[k + __popcll(mk & lt)] = f - 1u;
            } else {
                if (pure) ((C *)S.plist)[k + __popcll(mk & lt)] = (C)v;
            }
            k += __popcll(mk);
        };
        if constexpr (sizeof(C) == 1) {
            if (n >= 1) collect(1);
            if (n >= 65) collect(65);
        } else {
            for (int v0 = 1; v0 <= n; v0 += 64) collect(v0);
        }
        wave_sync();
    } else if (maxc > 0) {
        if (ncand == 1) {
            best = cvar;
        } else {
            const uint32_t bestf = first_flagged<K>(S, mpad);
            best = uniform_u32(field<K>(S.cls[bestf >> 3], (int)(bestf & 7u)) >> 1);
        }
    }
    return {npure, best};
}

// Append the pure literals in first-occurrence order (REF.py:187-189); the
// literal at a pure variable's first position carries its (only) sign.
template <int K, typename C>
__device__ int assign_pures(const SLds<K, C> &S, int npure, int tl) {
    const int ln = lane_id();
    // entry j's first position
    const auto pos = [&](int j) -> uint32_t {
        if constexpr (!plist_vars<K, C>()) return S.plist[j];
        else return S.first[((const C *)S.plist)[j]] - 1u;
    };
    for (int i0 = 0; i0 < npure; i0 += 64) {
        const int i = i0 + ln;
        const uint32_t my = i < npure ? pos(i) : NONE32;
        int rank = 0;
        for (int j = 0; j < npure; ++j) rank += pos(j) < my ? 1 : 0;
        if (i < npure) {
            const uint32_t code = field<K>(S.cls[my >> 3], (int)(my & 7u));
            S.trail[tl + rank] = (C)code;
            lv_assign(S.lv, code);
        }
    }
    wave_sync();
    return tl + npure;
}

template <int K, typename C>
__device__ void store_assignment(const SLds<K, C> &S, int tl, int32_t *out) {
    for (int i = lane_id(); i < tl; i += 64) {
        const uint32_t code = S.trail[i];
        const int v = (int)(code >> 1);
        out[i] = (code & 1u) ? -v : v;
    }
}

enum { ST_PROPAGATE = 0, ST_ANALYZE = 1, ST_BACKTRACK = 2, ST_DONE = 3 };

// Incremental kernel: occurrence lists of the staged clauses, S.occ[S.occ_off[x] ..
// S.occ_off[x+1]) = the clauses holding literal code x (each clause once, in no
// particular order -- the unit bitmap restores clause order).  cnt is borrowed
// as the per-code counter / fill cursor and left zeroed.
template <int K, typename C>
__device__ void build_occurrences(const SLds<K, C> &S, uint16_t *occ, int m, int n) {
    using W = typename Pack<K>::W;
    const int ln = lane_id();
    // distinct slots of a clause: a repeated code counts once
    auto each_slot = [&](auto &&f) {
        for (int c = ln; c < m; c += 64) {
            const W w = S.cls[c];
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const uint32_t code = field<K>(w, j);
                bool dup = code <= CODE_DUMMY;
#pragma unroll
                for (int i = 0; i < j; ++i) dup |= field<K>(w, i) == code;
                if (!dup) f(c, code);
            }
        }
    };
    each_slot([&](int, uint32_t code) { cnt_inc(S, code, 1u); });
    wave_sync();
    int carry = 0;
    for (int x0 = 0; x0 < 2 * (n + 1); x0 += 64) {
        const int x = x0 + ln;
        const int cx = x < 2 * (n + 1) ? (int)cnt_get(S, (uint32_t)x) : 0;
        const int in = wave_incl_scan(cx);
        if (x < 2 * (n + 1)) {
            S.occ_off[x] = (uint16_t)(carry + in - cx);
            if constexpr (!cnt_packed<K, C>()) S.cnt[x] = 0u;
            else if (!(x & 1)) S.cnt[x >> 1] = 0u;   // (both codes of the variable were read)
        }
        carry += lane63(in);
    }
    if (ln == 0) S.occ_off[2 * (n + 1)] = (uint16_t)carry;
    wave_sync();
    each_slot([&](int c, uint32_t code) {
        const uint32_t old = cnt_fetch_inc(S, code);
        occ[S.occ_off[code] + old] = (uint16_t)c;
    });
    wave_sync();
    if constexpr (!cnt_packed<K, C>())
        for (int x = ln; x < 2 * (n + 1); x += 64) S.cnt[x] = 0u;
    else
        for (int v = ln; v <= n; v += 64) S.cnt[v] = 0u;
    // the lists are read back by this wave only: complete the stores first
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    wave_sync();
}

// Per-instance counters between flushes (see solve_instance).
struct Ctr32 {
    uint32_t nodes = 0, decisions = 0, props = 0, pures = 0, conflicts = 0, rounds = 0;
};
constexpr uint32_t FLUSH_NODES = 1u << 20;   // props per flush <= 2^20 x n < 2^32
constexpr uint32_t TIME_CHECK_NODES = 1024;

// Global words shared between the waves of one launch go through agent-scope
// atomics (written through to memory, never cached stale in another XCD's L2).
#define SATMI_RLX_AGENT __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT
template <typename T>
__device__ __forceinline__ T ld_agent(T *p) { return __hip_atomic_load(p, SATMI_RLX_AGENT); }
template <typename T>
__device__ __forceinline__ void st_agent(T *p, T v) { __hip_atomic_store(p, v, SATMI_RLX_AGENT); }
template <typename T>
__device__ __forceinline__ T add_agent(T *p, T v) { return __hip_atomic_fetch_add(p, v, SATMI_RLX_AGENT); }
template <typename T>
__device__ __forceinline__ T cas_agent(T *p, T expect, T v) {
    __hip_atomic_compare_exchange_strong(p, &expect, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return expect;   // the value found
}

// Add the 32-bit counters into the int64 row (an instance's, or a split
// slot's; the first flush stores), zero them, and return the row's node total
// so far.  Write-through stores: a slot's row is read by another wave.
__device__ uint64_t flush_counters(int64_t *ctr, Ctr32 &c, bool &flushed) {
    uint64_t total = 0;
    if (lane_id() == 0) {
        const uint32_t v[6] = {c.nodes, c.decisions, c.props, c.pures, c.conflicts, c.rounds};
        const int k[6] = {SATMI_CTR_NODES, SATMI_CTR_DECISIONS, SATMI_CTR_UNIT_PROPS, SATMI_CTR_PURE,
                          SATMI_CTR_CONFLICTS, SATMI_CTR_ROUNDS};
        if (!flushed) {
            for (int i = 0; i < 6; ++i) st_agent(&ctr[k[i]], (int64_t)v[i]);
            total = c.nodes;
        } else {
            total = (uint64_t)add_agent(&ctr[SATMI_CTR_NODES], (int64_t)c.nodes) + c.nodes;
            for (int i = 1; i < 6; ++i) add_agent(&ctr[k[i]], (int64_t)v[i]);
        }
    }
    flushed = true;
    c = Ctr32{};
    return (uint64_t)uniform_u32((uint32_t)total) | ((uint64_t)uniform_u32((uint32_t)(total >> 32)) << 32);
}

// ---- Splitting the tail of a launch.
// Search trees differ by orders of magnitude, so a launch ends with a few
// long searches and idle waves.  A wave whose instance queue has drained asks
// for work (SplitCtl::want); a searching wave that sees a request donates the
// False branch of its shallowest open decision: the trail prefix before that
// decision and the branch literal go into a slot, the frame is marked DONATED,
// and an idle wave (the helper) re-stages the instance, assigns the prefix and
// searches that subtree exactly as the donor would have -- same counters,
// same model.  When the donor's backtracking reaches the donated frame it
// takes the helper's result instead of searching: UNSAT adds the helper's
// counters and backtracking continues, SAT ends the search with the helper's
// model.  A donation still unclaimed at that point is reclaimed and searched
// locally; a donor that finds a model first cancels its outstanding
// donations, whose work the sequential search never did (they add nothing).
// So the split search reports exactly the sequential one.  Used only where
// that holds: SOUND mode, stop at the first model, no node or time limit.
//
// Hand-off instead of a wait (r06): a donor whose backtracking reaches a
// donated frame that a helper is still searching does not wait for it.  It
// writes the rest of its search -- its identity (root instance or task slot),
// its decision frames above the donated one and its live donation stack --
// into the slot as a continuation, marks the slot HANDED, and is free for
// other work.  The helper, on finishing the subtree, finds its slot HANDED
// instead of publishing it, and continues the donor's search itself in its own
// LDS: same instance (clauses and occurrence lists already staged), same trail
// prefix (the subtree started from the donor's trail before the donated
// decision), the donor's frames and donation stack restored, its result taken
// exactly as the donor would have taken it (UNSAT: backtracking goes on; SAT:
// the model is the search's).  No wave ever waits on another, so a search split
// many ways no longer leaves donors idle on chains of joins.
//
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility): payload written
// through (agent atomic stores), `s_waitcnt vmcnt(0)`, then the state flag by
// an agent atomic; the reader polls the flag relaxed, then one agent acquire
// and plain loads.  Flags and payload live on separate 128-B lines.
// Head of the splitting scratch, rewritten before each launch (the slot pool
// follows at SPLIT_POOL_OFF, then the per-wave donation stacks).  One 128-B
// line per access pattern: the queue line is polled by the helpers, the
// request line read by every searching wave every SPLIT_CHECK_NODES nodes --
// kept apart so that polling never queues the searches' reads.
struct SplitCfg {
    uint32_t pub;              // line 0: slots allocated
    uint32_t taken;            //         slots ticketed by helpers
    uint32_t pad0[30];
    int32_t want;              // line 1: open requests of idle helpers
    uint32_t pad1[31];
    uint32_t done;             // line 2: root instances finished
    int32_t helpers;           //         waves that registered as helpers
    uint32_t claims, reclaims; //         statistics: subtrees run by helpers, taken back by donors
    unsigned long long handoffs;     //   continuations handed to helpers (see "Hand-off")
    unsigned long long busy;         //   wave ticks spent searching (every wave of the launch)
    uint32_t pad2[24];
    int32_t slot_cap, slot_bytes, dstack_cap;   // line 3: geometry (read only)
    uint32_t epoch;            // launch tag of the slot states (the pool is not cleared between launches)
    int32_t max_helpers;       // waves beyond this count exit when the queue drains (their CU slots go
                               // to the next launch on another stream)
    uint32_t warm;             // nodes of a search before it may donate
    int32_t cont_off;          // slot offset of the continuation: frames fvar[], ftrail[] (cont_fb bytes
    int32_t cont_fb;           // each), then the donation stack (int32)
    uint32_t pad3[24];
};
constexpr int SPLIT_POOL_OFF = 512;
static_assert(sizeof(SplitCfg) == SPLIT_POOL_OFF, "SplitCfg layout");
// A donation check every SPLIT_CHECK_NODES nodes, run from the node loop's
// existing event test (next_event), so the split form's loop carries no
// per-decision counter: what it keeps live is only read at the checks.  (r06:
// 16 -> 64 nodes, the N=8 shard +1.5 %, the split form at full size +0.5 %:
// each check is two dependent agent-scope loads; 256 measured the same as 64.)
#ifndef SATMI_SPLIT_CHECK_NODES
#define SATMI_SPLIT_CHECK_NODES 64u
#endif
constexpr uint32_t SPLIT_CHECK_NODES = SATMI_SPLIT_CHECK_NODES;
constexpr int SPLIT_MAX_PER_WAVE = 8;   // split a launch only up to this many instances per resident wave (r06: every
                                         // rank's shard at N=8 / 4 / 2, profiles/r06/slices.json)
// Kernels come in two forms: SPLIT = false has no branch-splitting code at all
// (its register cost -- SGPR spills in the node loop -- was measured at ~4 % of
// the full-size rate), SPLIT = true can split.  The host launches the split
// form only for launches with few instances per resident wave.
enum : uint32_t { SL_PENDING = 1, SL_RUNNING = 2, SL_DONE = 3, SL_RECLAIMED = 4, SL_HANDED = 5 };
struct SlotFlags {     // line 0 of a slot
    uint32_t state;    // split_epoch << 4 | SL_*
    uint32_t cancel;   // the donor no longer needs the result
};
struct SlotHdr {       // line 1 (payload)
    int32_t inst, tl0, dec_code, status, model_len;
    int32_t cont_task, cont_depth, cont_nd;   // a handed-over continuation: identity (-1: the root
                                              // search of `inst`), its frames and live donations
    int64_t ctr[SATMI_NCOUNTERS];
};
constexpr int SLOT_HDR_OFF = 128, SLOT_TRAIL_OFF = 256;
// a slot: flags line, payload line, the trail (prefix in, model out), then the
// continuation area (frames fvar / ftrail, the donation stack)
__host__ __device__ __forceinline__ int slot_frames_bytes(int ncap, int cb) { return ((ncap + 1) * cb + 127) & ~127; }
__host__ __device__ __forceinline__ int slot_cont_off(int ncap, int cb) {
    return SLOT_TRAIL_OFF + slot_frames_bytes(ncap, cb);
}
__host__ __device__ __forceinline__ int slot_bytes_for(int ncap, int cb) {
    return slot_cont_off(ncap, cb) + 2 * slot_frames_bytes(ncap, cb) + ((4 * (ncap + 1) + 127) & ~127);
}

struct SlotRef {
    SlotFlags *f;
    SlotHdr *h;
    uint32_t *trail;   // trail codes (C), as 32-bit words
};
__device__ __forceinline__ SlotRef slot_ref(const ScanArgs &A, int s) {
    unsigned char *p = (unsigned char *)A.split + SPLIT_POOL_OFF + (size_t)s * (size_t)A.split->slot_bytes;
    return {(SlotFlags *)p, (SlotHdr *)(p + SLOT_HDR_OFF), (uint32_t *)(p + SLOT_TRAIL_OFF)};
}
__device__ __forceinline__ uint32_t slot_state(const ScanArgs &A, uint32_t st) { return A.split->epoch << 4 | st; }
// wave w's donation stack
__device__ __forceinline__ int32_t *split_dstack(const SplitCfg *cfg, size_t w) {
    unsigned char *p = (unsigned char *)cfg + SPLIT_POOL_OFF + (size_t)cfg->slot_cap * (size_t)cfg->slot_bytes;
    return (int32_t *)p + w * (size_t)cfg->dstack_cap;
}

// After this wave's payload stores: drain them, then raise the flag.
__device__ __forceinline__ void publish_state(uint32_t *flag, uint32_t v) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane_id() == 0) st_agent(flag, v);
}
__device__ __forceinline__ void acquire_agent() {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Write `nbytes` of the wave's LDS trail (or any 4-B aligned LDS array) to a
// slot's trail, written through.
__device__ __forceinline__ void put_words(uint32_t *dst, const void *lds, int nbytes) {
    const uint32_t *src = (const uint32_t *)lds;
    for (int i = lane_id_here(); 4 * i < nbytes; i += 64) st_agent(&dst[i], src[i]);
}

// Nodes (counted from the last flush, at which the instance had `total`) after
// which the node loop stops for its rare checks.
__device__ uint32_t next_event_after(const ScanArgs &A, uint64_t total) {
    uint64_t ev = A.time_limit_ticks ? TIME_CHECK_NODES : FLUSH_NODES;
    if (A.node_limit > 0) ev = min(ev, (uint64_t)A.node_limit + 1u - total);   // total <= node_limit here
    return (uint32_t)ev;
}

// Donate the False branch of the shallowest open decision frame (see
// "Splitting the tail") if an idle wave asked for work.  `nd` entries of the
// wave's donation stack `dst` are live; frames donated later are deeper, so
// backtracking meets them in stack order.
template <int K, typename C>
__device__ void try_donate(const ScanArgs &A, const SLds<K, C> &S, int depth, int b, int32_t *dst, int &nd) {
    constexpr uint32_t PHASE = SLds<K, C>::PHASE_BIT, DON = SLds<K, C>::PHASE_BIT;
    const int ln = lane_id_here();
    int old = 0;
    if (ln == 0) old = add_agent(&A.split->want, -1);
    if (uniform_i32(old) <= 0) {
        if (ln == 0) add_agent(&A.split->want, 1);
        return;
    }
    int j = -1;
    for (int d0 = 0; d0 < depth; d0 += 64) {
        const int d = d0 + ln;
        const bool open = d < depth && !((uint32_t)S.fvar[d] & PHASE) && !((uint32_t)S.ftrail[d] & DON);
        const uint64_t mk = __ballot(open);
        if (mk) {
            j = d0 + __builtin_ctzll(mk);
            break;
        }
    }
    int s = -1;
    if (j >= 0 && nd < A.split->dstack_cap) {
        uint32_t x = 0;
        if (ln == 0) x = add_agent(&A.split->pub, 1u);
        x = uniform_u32(x);
        if (x < (uint32_t)A.split->slot_cap) s = (int)x;
    }
    if (s < 0) {
        if (ln == 0) add_agent(&A.split->want, 1);
        return;
    }
    const SlotRef r = slot_ref(A, s);
    const uint32_t fv = uniform_u32(S.fvar[j]);
    const int ft = uniform_i32(S.ftrail[j]);
    put_words(r.trail, S.trail, ft * (int)sizeof(C));
    if (ln == 0) {
        st_agent(&r.h->inst, b);
        st_agent(&r.h->tl0, ft);
        st_agent(&r.h->dec_code, (int32_t)((fv << 1) | 1u));   // the False branch
        st_agent(&r.f->cancel, 0u);
        S.ftrail[j] = (C)((uint32_t)ft | DON);
        dst[nd] = s;
    }
    publish_state(&r.f->state, slot_state(A, SL_PENDING));
    ++nd;
    wave_sync();
}

// Cancel the donations dst[0, nd): an unclaimed one is reclaimed (never run),
// a running one told to stop.
__device__ void cancel_donations(const ScanArgs &A, const int32_t *dst, int nd) {
    if (lane_id_here() != 0) return;
    for (int i = 0; i < nd; ++i) {
        const SlotRef r = slot_ref(A, dst[i]);
        if (cas_agent(&r.f->state, slot_state(A, SL_PENDING), slot_state(A, SL_RECLAIMED)) !=
            slot_state(A, SL_PENDING))
            st_agent(&r.f->cancel, 1u);
    }
}

enum { TAKE_LOCAL = 0, TAKE_UNSAT = 1, TAKE_SAT = 2, TAKE_CANCELLED = 3, TAKE_HANDED = 4 };

// The donor's backtracking reached donated slot s (frames [0, top) below it,
// donations dst[0, nd) still live): reclaim it if no helper took it
// (TAKE_LOCAL: search the branch here); take the helper's result if it has
// finished (its payload readable after the acquire); else hand the rest of
// this search to the helper (TAKE_HANDED: the caller ends without publishing
// -- see "Hand-off").  A search whose own task was cancelled passes the
// cancellation on and returns TAKE_CANCELLED.  Before a hand-off the donor's
// counters and busy ticks go into its row (the helper adds to the same row).
template <int K, typename C>
__device__ int take_donation(const ScanArgs &A, const SLds<K, C> &S, int s, int top, const int32_t *dst, int nd,
                             int task, int64_t *ctr, Ctr32 &c, bool &flushed, uint64_t &t_start) {
    const SlotRef r = slot_ref(A, s);
    const int ln = lane_id_here();
    uint32_t prev = 0;
    if (ln == 0) prev = cas_agent(&r.f->state, slot_state(A, SL_PENDING), slot_state(A, SL_RECLAIMED));
    if (uniform_u32(prev) == slot_state(A, SL_PENDING)) {
        if (ln == 0) add_agent(&A.split->reclaims, 1u);
        return TAKE_LOCAL;
    }
    if (uniform_u32(ld_agent(&r.f->state)) != slot_state(A, SL_DONE)) {
        if (task >= 0 && uniform_u32(ld_agent(&slot_ref(A, task).f->cancel))) {
            if (ln == 0) st_agent(&r.f->cancel, 1u);
            return TAKE_CANCELLED;
        }
        flush_counters(ctr, c, flushed);
        // this wave's busy time so far into the row before the hand-off can be
        // adopted (after it, the helper may publish the row at any moment)
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (ln == 0) add_agent(&ctr[SATMI_CTR_TICKS], (int64_t)(now - t_start));
        t_start = now;   // (if the helper published first, the search goes on here from now)
        unsigned char *cont = (unsigned char *)r.f + A.split->cont_off;
        const int fb = A.split->cont_fb;
        put_words((uint32_t *)cont, S.fvar, top * (int)sizeof(C));
        put_words((uint32_t *)(cont + fb), S.ftrail, top * (int)sizeof(C));
        int32_t *cd = (int32_t *)(cont + 2 * fb);
        for (int i = ln; i < nd; i += 64) st_agent(&cd[i], dst[i]);
        if (ln == 0) {
            st_agent(&r.h->cont_task, task);
            st_agent(&r.h->cont_depth, top);
            st_agent(&r.h->cont_nd, nd);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (ln == 0) prev = cas_agent(&r.f->state, slot_state(A, SL_RUNNING), slot_state(A, SL_HANDED));
        if (uniform_u32(prev) == slot_state(A, SL_RUNNING)) {
            if (ln == 0) add_agent(&A.split->handoffs, 1ull);
            return TAKE_HANDED;
        }
        // (the helper published meanwhile: take its result)
    }
    acquire_agent();
    return uniform_i32(r.h->status) == SATMI_DPLL_STOPPED ? TAKE_SAT : TAKE_UNSAT;
}

// Add a finished slot's counters into the row `ctr` (own counters flushed
// first); the helper's busy ticks go into the row's tick count.
__device__ void merge_counters(int64_t *ctr, Ctr32 &c, bool &flushed, const SlotHdr *h) {
    flush_counters(ctr, c, flushed);
    if (lane_id_here() == 0) {
        const int k[7] = {SATMI_CTR_NODES, SATMI_CTR_DECISIONS, SATMI_CTR_UNIT_PROPS, SATMI_CTR_PURE,
                          SATMI_CTR_CONFLICTS, SATMI_CTR_ROUNDS, SATMI_CTR_TICKS};
        for (int i = 0; i < 7; ++i) add_agent(&ctr[k[i]], h->ctr[k[i]]);
    }
}

// A model (ml trail codes at `src`, a slot's trail) as the first model of
// search identity `task` of instance b: into that task's slot, or (task < 0)
// the instance's first solution row.
template <typename C>
__device__ void deliver_model(const ScanArgs &A, int b, int task, const uint32_t *src, int ml) {
    const int lh = lane_id_here();
    if (task >= 0) {
        const SlotRef me = slot_ref(A, task);
        for (int i = lh; 4 * i < ml * (int)sizeof(C); i += 64) st_agent(&me.trail[i], src[i]);
        if (lh == 0) st_agent(&me.h->model_len, ml);
    } else if (A.sol_cap > 0) {
        const C *mt = (const C *)src;
        int32_t *out = A.sol_lits + (int64_t)b * A.sol_cap * A.sol_stride;
        for (int i = lh; i < ml; i += 64) {
            const uint32_t code = mt[i];
            out[i] = (code & 1u) ? -(int)(code >> 1) : (int)(code >> 1);
        }
        if (lh == 0) A.sol_len[(int64_t)b * A.sol_cap] = ml;
    }
}

constexpr int STATUS_HANDED = -1;   // (internal) the search was handed to a helper: nothing to publish

// Search instance b from its root (task < 0: results into the instance's
// rows), or the donated subtree of split slot `task` (results into the slot).
// dst: this wave's donation stack.  Returns whether a root search of the
// launch finished here (its own, or a donor's handed over to this wave).
template <int K, bool INC, typename C, bool SPLIT>
__device__ bool solve_instance(const ScanArgs &A, const SLds<K, C> &S, int b, int task, int32_t *dst) {
    SplitCfg *const SPL = SPLIT ? A.split : nullptr;
    using W = typename Pack<K>::W;
    constexpr uint32_t DON = SLds<K, C>::PHASE_BIT;   // ftrail: the frame's False branch was donated
    uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    const int ln = lane_id();
    PhaseClock ph;
    ph.start();
    const int cb = A.inst_clause_begin[b], ce = A.inst_clause_begin[b + 1];
    const int m = ce - cb;
    const int mpad = padded_clauses(m);
    const int L = A.clause_lit_begin[ce] - A.clause_lit_begin[cb];
    const int n = A.inst_nvars[b];
    bool is_task = SPLIT && task >= 0;   // the unsplit form has no donated tasks
    int64_t *ctr = is_task ? slot_ref(A, task).h->ctr : A.counters + (int64_t)b * SATMI_NCOUNTERS;
    bool bad = m > A.lay.mcap || n > A.lay.ncap || n < 0 || L > 65535 || (INC && L > (sizeof(C) == 1 ? A.occ_cap : A.occ_lists));
    if (!bad) {
        // ---- stage: pack each clause's literal codes into one word
        for (int c = ln; c < mpad; c += 64) {
            W w = (W)CODE_DUMMY;
            if (c < m) {
                const int j0 = A.clause_lit_begin[cb + c], j1 = A.clause_lit_begin[cb + c + 1];
                const int len = j1 - j0;
                w = 0;
                if (len < 1 || len > K) {
                    bad = true;
                } else {
                    for (int j = 0; j < len; ++j) {
                        const int x = A.lits[j0 + j];
                        const uint32_t v = (uint32_t)(x < 0 ? -x : x);
                        if (v == 0u || v > (uint32_t)n) bad = true;
                        w |= (W)((v << 1) | (x < 0 ? 1u : 0u)) << (Pack<K>::BITS * j);
                    }
                }
            }
            S.cls[c] = w;
        }
        for (int v = ln; v <= n; v += 64) {
            if (v == 0) {
                S.lv[CODE_PAD] = LV_FALSE;
                S.lv[CODE_DUMMY] = LV_TRUE;
            } else {
                lv_clear(S.lv, (uint32_t)v);
            }
            S.ts[v] = 0u;   // (the fixed kernel's `first` flags alias ts: set by choose() before use)
            cnt_clear_var(S, (uint32_t)v);
        }
    }
    if (__ballot(bad)) {
        if (ln < SATMI_NCOUNTERS) ctr[ln] = 0;
        if (ln == 0) {
            A.status[b] = SATMI_DPLL_TOO_LARGE;
            if (A.root_len) A.root_len[b] = 0;
        }
        return !is_task;
    }
    wave_sync();
    if constexpr (INC) build_occurrences<K>(S, const_cast<uint16_t *>(S.occ), m, n);
    ph.mark(PH_STAGE);

    // Counters since the last flush, 32-bit (few live registers in the node
    // loop); flush_counters() adds them into the instance's int64 row.  The
    // node loop compares one counter against next_event: the node limit, the
    // next time check or the next flush, whichever comes first.
    Ctr32 c;
    c.nodes = 1;
    int64_t sols = 0;
    bool flushed = false;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t next_flush = next_event_after(A, 0);
    uint32_t next_event = SPL ? min(next_flush, SPLIT_CHECK_NODES) : next_flush;
    int depth = 0, tl = 0;
    int status = SATMI_DPLL_EXHAUSTED;
    int state;
    uint32_t ep = 1;
    int nu = 0;
    bool dec_round = false;
    int nd = 0;                    // live entries of the donation stack
    // the row's tick count collects helpers' busy time minus time spent waiting
    // on them; the wave's own elapsed time is added at the end
    if (SPL && ln == 0) st_agent(&ctr[SATMI_CTR_TICKS], (int64_t)0);
    if (!is_task) {
        // root snapshot: the input's unit clauses in order (no clause is empty yet)
        int root_empty = INT_MAX;   // no clause is empty before any assignment
        nu = scan_units<K>(S, mpad, ep, 0u, &root_empty);
        ph.mark(PH_UNITS);
        const bool conflict = propagate<K, INC, C>(S, mpad, tl, nu, false, ep, c.props, c.rounds, ph);
        if (A.root_lits) store_assignment<K>(S, tl, A.root_lits + (int64_t)b * A.sol_stride);
        if (A.root_len && ln == 0) A.root_len[b] = tl;
        c.conflicts += conflict ? 1u : 0u;
        state = conflict ? ST_DONE : ST_ANALYZE;   // a root conflict has nothing to backtrack to
    } else {
        // donated subtree: the donor's trail before its decision, then the
        // False branch as the donor's backtracking would start it
        const SlotRef me = slot_ref(A, task);
        const int tl0 = uniform_i32(me.h->tl0);
        const uint32_t dcode = uniform_u32((uint32_t)me.h->dec_code);
        const C *pt = (const C *)me.trail;
        for (int i = ln; i < tl0; i += 64) {
            const uint32_t code = pt[i];
            S.trail[i] = (C)code;
            lv_assign(S.lv, code);
        }
        tl = tl0;
        wave_sync();
        if (ln == 0) {
            S.snap[0] = (C)dcode;
            S.ts[dcode >> 1] = stamp(ep, 0u);
        }
        c.decisions = 1;
        nu = 1;
        dec_round = true;
        state = ST_PROPAGATE;
        wave_sync();
    }

    for (;;) {   // (split form) a continuation handed to this wave runs the search loop again
    while (state != ST_DONE) {
        if (state == ST_PROPAGATE) {
            const bool conflict = propagate<K, INC, C>(S, mpad, tl, nu, dec_round, ep, c.props, c.rounds, ph);
            dec_round = false;
            if (conflict) {
                ++c.conflicts;
                state = ST_BACKTRACK;
            } else {
                state = ST_ANALYZE;
            }
        }
        // no event test between propagation and analysis: the node count
        // only moves in the analysis, so the test after it sees the same
        if (state == ST_ANALYZE) {
            bool leaf = false;
            Choice r{0, 0u};
            ph.mark(PH_OTHER);
            const int nact = scan_counts<K>(S, mpad);
            ph.mark(PH_COUNTS);
            if (nact == 0) {
                leaf = true;                                   // REF.py:170-171
            } else {
                r = choose<K>(S, n, mpad);
                if (r.npure == 0 && r.best_var == 0u) leaf = true;   // REF.py:205-206
            }
            ph.mark(PH_CHOOSE);
            if (!leaf && r.npure > 0) {                        // REF.py:186-195
                tl = assign_pures<K>(S, r.npure, tl);
                ph.mark(PH_PURE);
                c.pures += (uint32_t)r.npure;
                ++c.nodes;                                     // recursive call; its unit_propagate is a no-op
            } else if (!leaf) {                                // REF.py:208-213, as formula + [[var]]
                const uint32_t v = r.best_var;
                ep = next_decision_epoch<K>(S, n, ep);
                if (ln == 0) {
                    S.fvar[depth] = (C)v;
                    S.ftrail[depth] = (C)tl;
                    S.snap[0] = (C)(v << 1);                   // True first
                    S.ts[v] = stamp(ep, 0u);
                }
                ++depth;
                ++c.decisions;
                ++c.nodes;
                nu = 1;
                dec_round = true;
                state = ST_PROPAGATE;
                wave_sync();
            } else {
                if (is_task) {
                    const SlotRef me = slot_ref(A, task);
                    put_words(me.trail, S.trail, tl * (int)sizeof(C));   // the model, as trail codes
                    if (lane_id_here() == 0) st_agent(&me.h->model_len, tl);
                } else if (sols < A.sol_cap) {
                    store_assignment<K>(S, tl, A.sol_lits + ((int64_t)b * A.sol_cap + sols) * A.sol_stride);
                    if (ln == 0) A.sol_len[(int64_t)b * A.sol_cap + sols] = tl;
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
        if (!SPLIT && state == ST_BACKTRACK) {
            // unwind the finished frames (both branches run) with one scalar
            // read each, then clear the trail above the open frame once
            state = ST_DONE;
            int top = depth - 1;
            while (top >= 0 && (uniform_u32(S.fvar[top]) & SLds<K, C>::PHASE_BIT)) --top;
            depth = top + 1;
            if (top >= 0) {
                const uint32_t fv = uniform_u32(S.fvar[top]);
                const int ft = (int)uniform_u32(S.ftrail[top]);
                for (int i = ft + lane_id_here(); i < tl; i += 64) lv_clear(S.lv, S.trail[i] >> 1);
                tl = ft;
                ep = next_decision_epoch<K>(S, n, ep);
                if (ln == 0) {
                    S.fvar[top] = (C)(fv | SLds<K, C>::PHASE_BIT);
                    S.snap[0] = (C)((fv << 1) | 1u);           // False
                    S.ts[fv] = stamp(ep, 0u);
                }
                ++c.decisions;
                ++c.nodes;
                nu = 1;
                dec_round = true;
                state = ST_PROPAGATE;
                wave_sync();
            }
        }
        if (SPLIT && state == ST_BACKTRACK) {
            state = ST_DONE;
            for (;;) {
                // unwind the finished frames with one scalar read each
                while (depth > 0 && (uniform_u32(S.fvar[depth - 1]) & SLds<K, C>::PHASE_BIT)) --depth;
                if (depth == 0) break;
                const int top = depth - 1;
                const uint32_t fv = uniform_u32(S.fvar[top]);   // its False branch has not run here
                const uint32_t ftw = uniform_u32(S.ftrail[top]);
                const int ft = (int)(ftw & ~DON);
                for (int i = ft + lane_id_here(); i < tl; i += 64) lv_clear(S.lv, S.trail[i] >> 1);
                tl = ft;
                wave_sync();
                if (ftw & DON) {
                    // the False branch was donated: take its result
                    --nd;
                    const int s = uniform_i32(dst[nd]);
                    if (lane_id_here() == 0) S.ftrail[top] = (C)ft;
                    const int got = take_donation<K>(A, S, s, top, dst, nd, is_task ? task : -1, ctr, c, flushed,
                                                     t_start);
                    if (got == TAKE_HANDED) {   // the helper continues this search (see "Hand-off")
                        status = STATUS_HANDED;
                        break;
                    }
                    if (got == TAKE_CANCELLED) {
                        status = SATMI_DPLL_TIMEOUT;
                        break;
                    }
                    if (got != TAKE_LOCAL) {
                        const SlotRef r = slot_ref(A, s);
                        merge_counters(ctr, c, flushed, r.h);
                        if (got == TAKE_UNSAT) {
                            --depth;
                            continue;
                        }
                        // SAT: the helper's model is the search's first model
                        deliver_model<C>(A, b, is_task ? task : -1, r.trail, uniform_i32(r.h->model_len));
                        sols = 1;
                        status = SATMI_DPLL_STOPPED;
                        break;
                    }
                }
                ep = next_decision_epoch<K>(S, n, ep);
                if (ln == 0) {
                    S.fvar[top] = (C)(fv | SLds<K, C>::PHASE_BIT);
                    S.snap[0] = (C)((fv << 1) | 1u);               // False
                    S.ts[fv] = stamp(ep, 0u);
                }
                ++c.decisions;
                ++c.nodes;
                nu = 1;
                dec_round = true;
                state = ST_PROPAGATE;
                wave_sync();
                break;
            }
        }
        if (__builtin_expect(c.nodes >= next_event, 0) && state != ST_DONE) {
            if (SPL) {
                // between nodes every decision frame below depth is complete,
                // so the shallowest open one can be donated here
                if (is_task && uniform_u32(ld_agent(&slot_ref(A, task).f->cancel))) {
                    status = SATMI_DPLL_TIMEOUT;               // abandoned: the donor found its model first
                    state = ST_DONE;
                    continue;
                }
                // warm: this search's nodes so far (c counts since the last flush, and a
                // flush comes only after far more nodes than any warm-up)
                if ((flushed || c.nodes >= SPL->warm) && uniform_i32(ld_agent(&SPL->want)) > 0)
                    try_donate<K>(A, S, depth, b, dst, nd);
            }
            if (!SPL || c.nodes >= next_flush) {
                const uint64_t total = flush_counters(ctr, c, flushed);
                if (A.node_limit > 0 && total > (uint64_t)A.node_limit) {
                    status = SATMI_DPLL_NODE_LIMIT;
                    state = ST_DONE;
                } else if (A.time_limit_ticks && __builtin_amdgcn_s_memrealtime() - t0 > A.time_limit_ticks) {
                    status = SATMI_DPLL_TIMEOUT;
                    state = ST_DONE;
                } else {
                    next_flush = next_event_after(A, total);
                }
            }
            next_event = SPL ? min(next_flush, c.nodes + SPLIT_CHECK_NODES) : next_flush;
        }
    }
#ifdef SATMI_PHASE_STAMPS
    ph.mark(PH_OTHER);
    if (!is_task && A.root_lits && A.sol_stride >= 48 && ln < 24)
        ((int64_t *)(A.root_lits + (int64_t)b * A.sol_stride))[ln] = (int64_t)(ln < 8 ? ph.acc[ln] : ph.cnt[ln - 8]);
#endif
    if (SPLIT && status == STATUS_HANDED) return false;   // counters and ticks are in the row already
    if (SPLIT && nd > 0) cancel_donations(A, dst, nd);   // a model (or a cancellation) came first
    flush_counters(ctr, c, flushed);
    const int64_t ticks = (int64_t)(__builtin_amdgcn_s_memrealtime() - t_start);
    if (!is_task) {
        if (ln == 0) {
            A.status[b] = status;
            ctr[SATMI_CTR_SOLUTIONS] = sols;
            if (SPL) add_agent(&ctr[SATMI_CTR_TICKS], ticks);
            else ctr[SATMI_CTR_TICKS] = ticks;
        }
        return true;
    }
    if constexpr (SPLIT) {
        const SlotRef me = slot_ref(A, task);
        if (ln == 0) {
            st_agent(&me.h->status, status);
            st_agent(&ctr[SATMI_CTR_SOLUTIONS], sols);
            add_agent(&ctr[SATMI_CTR_TICKS], ticks);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint32_t prev = 0;
        if (ln == 0) prev = cas_agent(&me.f->state, slot_state(A, SL_RUNNING), slot_state(A, SL_DONE));
        if (uniform_u32(prev) != slot_state(A, SL_HANDED)) return false;   // published
        // The donor handed the rest of its search to this wave: take this
        // subtree's result as the donor would have, then go on as the donor
        // (same instance, same trail prefix [0, tl0); see "Hand-off").
        acquire_agent();
        const int ctask = uniform_i32(me.h->cont_task), cdepth = uniform_i32(me.h->cont_depth);
        const int cnd = uniform_i32(me.h->cont_nd), tl0 = uniform_i32(me.h->tl0);
        int64_t *nctr = ctask >= 0 ? slot_ref(A, ctask).h->ctr : A.counters + (int64_t)b * SATMI_NCOUNTERS;
        if (ln == 0) {   // this subtree's row (complete) into the donor's
            const int k[7] = {SATMI_CTR_NODES, SATMI_CTR_DECISIONS, SATMI_CTR_UNIT_PROPS, SATMI_CTR_PURE,
                              SATMI_CTR_CONFLICTS, SATMI_CTR_ROUNDS, SATMI_CTR_TICKS};
            for (int i = 0; i < 7; ++i) add_agent(&nctr[k[i]], ld_agent(&ctr[k[i]]));
        }
        uint32_t *cont = (uint32_t *)((unsigned char *)me.f + A.split->cont_off);
        const int fw = A.split->cont_fb / 4;
        for (int i = lane_id_here(); 4 * i < cdepth * (int)sizeof(C); i += 64) {
            ((uint32_t *)S.fvar)[i] = ld_agent(&cont[i]);
            ((uint32_t *)S.ftrail)[i] = ld_agent(&cont[fw + i]);
        }
        for (int i = lane_id_here(); i < cnd; i += 64) st_agent(&dst[i], (int32_t)ld_agent(&cont[2 * fw + i]));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        acquire_agent();   // (the donation stack is read back with plain loads)
        const int mine = status;
        task = ctask;
        is_task = ctask >= 0;
        ctr = nctr;
        flushed = true;
        depth = cdepth;
        nd = cnd;
        sols = 0;
        t_start = __builtin_amdgcn_s_memrealtime();
        next_flush = next_event_after(A, 0);
        next_event = min(next_flush, c.nodes + SPLIT_CHECK_NODES);
        if (mine == SATMI_DPLL_STOPPED) {
            // this subtree's model (in this slot's trail) is the donor's first model
            deliver_model<C>(A, b, is_task ? task : -1, me.trail, uniform_i32(me.h->model_len));
            sols = 1;
            status = SATMI_DPLL_STOPPED;
            state = ST_DONE;
        } else if (mine != SATMI_DPLL_EXHAUSTED) {   // cancelled
            status = mine;
            state = ST_DONE;
        } else {   // UNSAT: the donor's backtracking goes on from its trail before the donated decision
            for (int i = tl0 + lane_id_here(); i < tl; i += 64) lv_clear(S.lv, S.trail[i] >> 1);
            tl = tl0;
            status = SATMI_DPLL_EXHAUSTED;
            state = ST_BACKTRACK;
        }
        wave_sync();
        continue;
    }
    return false;
    }
}

// The launch's split header (counters zeroed, geometry set) from `cfg`.
__global__ void __launch_bounds__(64) split_init_kernel(SplitCfg *dst, SplitCfg cfg) {
    static_assert(sizeof(SplitCfg) % 4 == 0, "SplitCfg words");
    const uint32_t *src = (const uint32_t *)&cfg;
    for (int i = threadIdx.x; i < (int)(sizeof(SplitCfg) / 4); i += 64) ((uint32_t *)dst)[i] = src[i];
}

// An idle wave's next donated subtree: {instance, slot}, or y < 0 once every
// instance of the launch has finished.  Not inlined: its polling addresses
// would otherwise be hoisted into registers held across the node loop.
__device__ __forceinline__ int2 next_donation(SplitCfg *cfg, int num_instances) {
    const int ln = lane_id();
    for (uint32_t polls = 0;; ++polls) {
        if ((polls & 7u) == 0u && uniform_u32(ld_agent(&cfg->done)) >= (uint32_t)num_instances)
            return make_int2(-1, -1);
        // pub and taken in one load: the queue line is the only one a helper polls
        const unsigned long long q = ld_agent((unsigned long long *)&cfg->pub);
        const uint32_t p = min(uniform_u32((uint32_t)q), (uint32_t)cfg->slot_cap);
        const uint32_t t = uniform_u32((uint32_t)(q >> 32));
        if (t >= p) {
            __builtin_amdgcn_s_sleep(127);   // ~8k cycles between polls
            continue;
        }
        uint32_t got = 0;
        if (ln == 0) got = cas_agent(&cfg->taken, t, t + 1u);
        if (uniform_u32(got) != t) continue;
        unsigned char *slot = (unsigned char *)cfg + SPLIT_POOL_OFF + (size_t)t * (size_t)cfg->slot_bytes;
        SlotFlags *f = (SlotFlags *)slot;
        const uint32_t pending = cfg->epoch << 4 | SL_PENDING;
        // the donor raises the flag right after allocating the slot
        while ((uniform_u32(ld_agent(&f->state)) >> 4) != cfg->epoch) __builtin_amdgcn_s_sleep(2);
        uint32_t prev = 0;
        if (ln == 0) prev = cas_agent(&f->state, pending, (cfg->epoch << 4) | SL_RUNNING);
        if (uniform_u32(prev) != pending) {   // reclaimed by its donor
            if (ln == 0) add_agent(&cfg->want, 1);
            continue;
        }
        if (ln == 0) add_agent(&cfg->claims, 1u);
        acquire_agent();
        return make_int2(uniform_i32(((SlotHdr *)(slot + SLOT_HDR_OFF))->inst), (int)t);
    }
}

// One wave's share of a launch: instances from the queue, then (splitting on)
// donated subtrees until every instance of the launch has finished.  One call
// site of solve_instance (one inlined copy: register pressure).
template <int K, bool INC, typename C, bool SPLIT>
__device__ void run_queue(const ScanArgs &A, const SLds<K, C> &S, int32_t *dst) {
    SplitCfg *const SPL = SPLIT ? A.split : nullptr;
    const int ln = lane_id();
    bool draining = false;   // the instance queue is empty: take donated subtrees
    uint64_t busy = 0;       // (split form) this wave's ticks inside searches
    for (;;) {
        int b = -1, task = -1;
        if (!draining) {
            uint32_t x = 0;
            if (ln == 0) x = atomicAdd(A.work_counter, 1u);
            x = uniform_u32(x);
            if (x < (uint32_t)A.num_instances) {
                b = (int)x;
            } else {
                if (!SPL) break;
                // a bounded set of helpers stays; the rest free their slots
                int h = 0;
                if (ln == 0) h = add_agent(&SPL->helpers, 1);
                if (uniform_i32(h) >= SPL->max_helpers) break;
                draining = true;
                if (ln == 0) add_agent(&SPL->want, 1);
            }
        }
        if (draining) {
            const int2 w = next_donation(SPL, A.num_instances);
            if (w.y < 0) break;
            b = w.x;
            task = w.y;
        }
        // wave-uniform (a divergent-looking b costs 64-bit VGPR address math)
        const uint64_t tb = SPLIT ? __builtin_amdgcn_s_memrealtime() : 0;
        const bool root_done = solve_instance<K, INC, C, SPLIT>(A, S, uniform_i32(b), uniform_i32(task), dst);
        if (SPLIT) busy += __builtin_amdgcn_s_memrealtime() - tb;
        if (SPL && ln == 0) {
            if (root_done) add_agent((int32_t *)&SPL->done, 1);   // (own, or a donor's handed over)
            if (draining) add_agent(&SPL->want, 1);                // a helper asks for its next subtree
        }
        wave_sync();
    }
    if (SPL && ln == 0) add_agent(&SPL->busy, (unsigned long long)busy);
}

// Persistent grid: waves pull instance indices from a global counter until the
// batch is drained (search-tree sizes differ by orders of magnitude).
// LVS > 0: one-wave workgroups whose literal states live in a static LDS array
// of LVS bytes -- its address is fixed at code generation, so a gather
// addresses lv[code] with the code register and an immediate offset (no
// per-wave base add per literal).  LVS = 0: multi-wave workgroups, the waves
// taking consecutive images of the dynamic LDS, lv included.
template <int K, int LVS, bool INC, bool SPLIT>
__global__ void __launch_bounds__(LVS ? 64 : 256, SATMI_SCAN_WAVES_PER_SIMD) dpll_scan_kernel(ScanArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    using C = std::conditional_t<LVS == 256, uint8_t, uint16_t>;
    const int wave = (int)(threadIdx.x >> 6);
    unsigned char *base = LVS ? smem : smem + (size_t)wave * A.lay.bytes;
    SLds<K, C> S;
    S.cls = (typename Pack<K>::W *)(base + A.lay.cls);
    if constexpr (LVS > 0) {
        __shared__ __attribute__((aligned(16))) uint8_t lv_static[LVS];
        S.lv = lv_static;
    } else {
        S.lv = (uint8_t *)(base + A.lay.lv);
    }
    S.ts = (uint32_t *)(base + A.lay.ts);
    S.cnt = (uint32_t *)(base + A.lay.cnt);
    S.first = (uint32_t *)(base + A.lay.first);
    S.trail = (C *)(base + A.lay.trail);
    S.fvar = (C *)(base + A.lay.fvar);
    S.ftrail = (C *)(base + A.lay.ftrail);
    S.snap = (C *)(base + A.lay.scratch);
    S.plist = (uint32_t *)(base + A.lay.scratch);
    S.scap = A.snap_lds;
    uint16_t *const wreg = A.occ ? A.occ + ((size_t)blockIdx.x * (blockDim.x >> 6) + (size_t)wave) * (size_t)A.occ_cap
                                 : nullptr;
    S.snapg = (C *)(wreg ? wreg + A.occ_lists : nullptr);
    if constexpr (INC) {
        S.occ_off = (uint16_t *)(base + A.lay.occ_off);
        S.bm = (uint2 *)(base + A.lay.bm);
        S.occ = wreg;
        for (int w = lane_id(); w < A.lay.nw; w += 64) S.bm[w].x = 0u;
        wave_sync();
    }
    span_begin(A.work_counter);
    const size_t wave_gid = (size_t)blockIdx.x * (blockDim.x >> 6) + (size_t)wave;
    run_queue<K, INC, C, SPLIT>(A, S, SPLIT ? split_dstack(A.split, wave_gid) : nullptr);
    span_end(A.work_counter);
}

// The bench shape class (K = 3, n <= 127, m <= FIXM): the incremental kernel
// with every per-wave array static, so all LDS addresses are link-time
// constants -- an access is `ds_* vindex offset:imm`, with no base register
// to keep live or add (the runtime-layout kernel spends an SGPR and a VALU
// add per access).  5,108 B of LDS per wave at FIXM = 448: 32 waves per CU.
constexpr int FIX_NCAP = 127;
template <int FIXM, bool SPLIT>
__global__ void __launch_bounds__(64, SATMI_SCAN_WAVES_PER_SIMD) dpll_fixed_kernel(ScanArgs A) {
    static_assert(FIXM % 64 == 0, "whole 64-clause chunks");
    __shared__ __attribute__((aligned(16))) uint32_t cls_s[FIXM];
    __shared__ __attribute__((aligned(16))) uint8_t lv_s[2 * (FIX_NCAP + 1)];
    // cnt: one word per literal code; choose()'s `first` flags live in ts (a
    // flag is < 0x10000 here -- m <= FIXM positions -- so it never matches a
    // stamp of an epoch >= 1, nor outranks one in atomicMax)
    __shared__ __attribute__((aligned(16))) uint32_t ts_s[FIX_NCAP + 1], cnt_s[2 * (FIX_NCAP + 1)];
    __shared__ __attribute__((aligned(16))) uint8_t trail_s[FIX_NCAP + 1], fvar_s[FIX_NCAP + 1],
        ftrail_s[FIX_NCAP + 1];
    // snapshot (<= FIXM + 1 byte codes) / pure-literal positions (<= 128 words)
    __shared__ __attribute__((aligned(16))) uint32_t scratch_s[(FIXM + 4) / 4 > FIX_NCAP + 1 ? (FIXM + 4) / 4
                                                                                             : FIX_NCAP + 1];
    __shared__ __attribute__((aligned(16))) uint16_t occ_off_s[2 * (FIX_NCAP + 1) + 2];
    __shared__ __attribute__((aligned(16))) uint2 bm_s[FIXM / 32];
    SLds<3, uint8_t> S;
    S.cls = cls_s;
    S.lv = lv_s;
    S.ts = ts_s;
    S.cnt = cnt_s;
    S.first = ts_s;
    S.trail = trail_s;
    S.fvar = fvar_s;
    S.ftrail = ftrail_s;
    S.snap = (uint8_t *)scratch_s;
    S.plist = scratch_s;
    S.snapg = nullptr;   // byte codes: the whole snapshot in LDS
    S.scap = FIXM + 4;
    S.occ_off = occ_off_s;
    S.bm = bm_s;
    S.occ = A.occ + (size_t)blockIdx.x * (size_t)A.occ_cap;
    for (int w = lane_id(); w < FIXM / 32; w += 64) S.bm[w].x = 0u;
    wave_sync();
    span_begin(A.work_counter);
    run_queue<3, true, uint8_t, SPLIT>(A, S, SPLIT ? split_dstack(A.split, blockIdx.x) : nullptr);
    span_end(A.work_counter);
}
constexpr int FIX_MCAP = 448;   // configs[1] (n=50, m=213) and configs[2] (n=100, m=426)
constexpr uint32_t FIX_LDS_BYTES = 4 * FIX_MCAP + 2 * (FIX_NCAP + 1) + 3 * 4 * (FIX_NCAP + 1) + 3 * (FIX_NCAP + 1) +
                                   4 * (FIX_NCAP + 1) + 2 * (2 * (FIX_NCAP + 1) + 2) + 8 * (FIX_MCAP / 32);

// Static literal-state size class of the one-wave kernel: 2(n+1) bytes rounded
// up to 256 (n <= 127) or to the packing's variable limit.
int lv_static_class(int K, int max_vars) {
    const int need = 2 * (max_vars + 1);
    if (K == 3) return need <= 256 ? 256 : need <= 512 ? 512 : 2 * (Pack<3>::MAXV + 1);
    return need <= 512 ? 512 : 2 * (Pack<5>::MAXV + 1);   // 5-SAT n <= 255: 3.5 KB less per wave
}

uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }

// snapshot entries kept in LDS: all with byte codes, at most 512 with 16-bit
// codes (the rest in HBM: snap_put); M = clauses + 1
// snapshot entries in LDS: all (byte codes), else the first 256 for 3-literal
// clauses (see plist_vars) and 512 for longer ones (rounds find tens of
// units; a larger snapshot's tail goes to the wave's HBM scratch)
uint32_t snap_lds_entries(int K, uint32_t cb, uint32_t M) { return cb == 1 ? M : std::min(M, K == 3 ? 256u : 512u); }

int pick_k(int max_vars, int max_clause_len) {
    if (max_clause_len < 1 || max_clause_len > 5) return 0;
    if (max_clause_len <= 3 && max_vars <= Pack<3>::MAXV) return 3;
    if (max_vars <= Pack<5>::MAXV) return 5;
    return 0;
}

// cb: bytes of a trail / frame / snapshot entry (1 for the 256-B size class, see SLds)
bool make_layout(int K, int max_vars, int max_clauses, bool with_lv, bool inc, uint32_t cb, ScanLayout *lay) {
    if (max_vars < 0 || max_clauses < 0 || max_clauses > 65534) return false;
    const uint32_t N = (uint32_t)max_vars + 1, M = (uint32_t)max_clauses + 1;
    const uint32_t Mpad = (uint32_t)padded_clauses(max_clauses);
    const uint32_t NW = (Mpad + 31u) / 32u;
    uint32_t o = 0;
    lay->lv = o;      o = align16(o + (with_lv ? 2 * N : 0u));   // one-wave kernel: static LDS instead
    lay->cls = o;     o = align16(o + (K == 3 ? 4u : 8u) * Mpad);
    lay->ts = o;      o = align16(o + 4 * N);
    lay->cnt = o;     o = align16(o + (cb == 2 && K == 3 ? 4 : 8) * N);   // see cnt_packed
    // choose()'s flags alias the stamps when every first position + 1, (c << 3 |
    // slot) + 1, stays <= 0x10000: below any stamp of an epoch >= 1 (as in
    // dpll_fixed_kernel); larger formulas keep a separate array
    if (max_clauses <= 8191) lay->first = lay->ts;
    else { lay->first = o; o = align16(o + 4 * N); }
    lay->trail = o;   o = align16(o + cb * N);
    lay->fvar = o;    o = align16(o + cb * N);
    lay->ftrail = o;  o = align16(o + cb * N);
    // the snapshot, or the pure literals (positions, 4 B; variables, cb B: plist_vars)
    lay->scratch = o; o = align16(o + std::max(cb * snap_lds_entries(K, cb, M), (cb == 2 && K == 3 ? cb : 4u) * N));
    lay->occ_off = o; o = align16(o + (inc ? 2 * (2 * N + 1) : 0u));
    lay->bm = o;      o = align16(o + (inc ? 8 * NW : 0u));
    lay->bytes = o;
    lay->mcap = max_clauses;
    lay->ncap = max_vars;
    lay->nw = (int32_t)NW;
    return o <= 160u * 1024u;
}

template <bool INC>
const void *scan_fn(int K, int lvs) {   // occupancy queries: the split form (the larger register budget)
    if (K == 3) {
        if (lvs == 256) return (const void *)dpll_scan_kernel<3, 256, INC, true>;
        if (lvs == 512) return (const void *)dpll_scan_kernel<3, 512, INC, true>;
        if (lvs == 1024) return (const void *)dpll_scan_kernel<3, 1024, INC, true>;
        return (const void *)dpll_scan_kernel<3, 0, INC, true>;
    }
    if (lvs == 512) return (const void *)dpll_scan_kernel<5, 512, INC, true>;
    return lvs ? (const void *)dpll_scan_kernel<5, 4096, INC, true> : (const void *)dpll_scan_kernel<5, 0, INC, true>;
}
const void *scan_fn(int K, int lvs, bool inc) { return inc ? scan_fn<true>(K, lvs) : scan_fn<false>(K, lvs); }

struct ScanPlan {
    int waves_per_wg = 1, wg_per_cu = 1, lvs = 0;
    bool fixed = false;   // dpll_fixed_kernel<FIX_MCAP> (static layout)
    ScanLayout lay;
};

bool fixed_class(int K, int max_vars, int max_clauses, bool inc) {
    return inc && K == 3 && max_vars <= FIX_NCAP && max_clauses <= FIX_MCAP;
}

// Launch shape: the workgroup size that keeps the most waves resident under
// LDS (<= 32 waves per CU) and the kernel's register budget
// (hipOccupancyMaxActiveBlocksPerMultiprocessor); one-wave workgroups (the
// cheaper gather addressing) whenever they reach the same residency.
int scan_plan(int K, int max_vars, int max_clauses, bool inc, ScanPlan *P) {
    if (fixed_class(K, max_vars, max_clauses, inc)) {
        const void *fn = (const void *)dpll_fixed_kernel<FIX_MCAP, true>;
        int occ = 0, wgs = 32;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, 64, 0) == hipSuccess && occ > 0)
            wgs = std::min(wgs, occ);
        P->fixed = true;
        P->waves_per_wg = 1;
        P->wg_per_cu = wgs;
        P->lvs = 0;
        P->lay = ScanLayout{};
        P->lay.mcap = FIX_MCAP;
        P->lay.ncap = FIX_NCAP;
        P->lay.nw = FIX_MCAP / 32;
        P->lay.bytes = 0;
        return SATMI_OK;
    }
    int best = 0;
    for (int wpg : {1, 4, 2}) {
        const int lvs = wpg == 1 ? lv_static_class(K, max_vars) : 0;
        ScanLayout lay;
        if (!make_layout(K, max_vars, max_clauses, lvs == 0, inc, lvs == 256 ? 1u : 2u, &lay)) continue;
        const void *fn = scan_fn(K, lvs, inc);
        const uint32_t wg_lds = lay.bytes * (uint32_t)wpg;
        const uint32_t wg_all = wg_lds + (uint32_t)lvs;
        if (wg_all > 160u * 1024u) continue;
        int wgs = std::min(32 / wpg, (int)((160u * 1024u) / wg_all));
        if (wg_lds > 64u * 1024u)
            SATMI_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)wg_lds));
        int occ = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, 64 * wpg, wg_lds) == hipSuccess && occ > 0)
            wgs = std::min(wgs, occ);
        const int waves = std::min(32, wgs * wpg);
        if (waves > best) {
            best = waves;
            P->waves_per_wg = wpg;
            P->wg_per_cu = std::max(1, std::min(wgs, 32 / wpg));
            P->lvs = lvs;
            P->lay = lay;
        }
    }
    if (!best) {
        set_error("dpll_scan: no resident workgroup shape");
        return SATMI_ERR_TOO_LARGE;
    }
    return SATMI_OK;
}

template <bool INC, bool SPLIT>
void launch_kernel(int K, int lvs, dim3 g, dim3 blk, uint32_t wg_lds, hipStream_t s, const ScanArgs &A) {
    if (K == 3 && lvs == 256)
        hipLaunchKernelGGL((dpll_scan_kernel<3, 256, INC, SPLIT>), g, blk, wg_lds, s, A);
    else if (K == 3 && lvs == 512)
        hipLaunchKernelGGL((dpll_scan_kernel<3, 512, INC, SPLIT>), g, blk, wg_lds, s, A);
    else if (K == 3 && lvs == 1024)
        hipLaunchKernelGGL((dpll_scan_kernel<3, 1024, INC, SPLIT>), g, blk, wg_lds, s, A);
    else if (K == 3)
        hipLaunchKernelGGL((dpll_scan_kernel<3, 0, INC, SPLIT>), g, blk, wg_lds, s, A);
    else if (lvs == 512)
        hipLaunchKernelGGL((dpll_scan_kernel<5, 512, INC, SPLIT>), g, blk, wg_lds, s, A);
    else if (lvs)
        hipLaunchKernelGGL((dpll_scan_kernel<5, 4096, INC, SPLIT>), g, blk, wg_lds, s, A);
    else
        hipLaunchKernelGGL((dpll_scan_kernel<5, 0, INC, SPLIT>), g, blk, wg_lds, s, A);
}

}  // namespace

int64_t dpll_split_busy(const void *head) { return (int64_t)((const SplitCfg *)head)->busy; }

void dpll_split_decode(const void *head, int64_t out[7]) {
    static_assert(SPLIT_HEAD_BYTES == SPLIT_POOL_OFF, "split head");
    const SplitCfg *c = (const SplitCfg *)head;
    out[0] = c->pub;
    out[1] = c->taken;
    out[2] = c->claims;
    out[3] = c->reclaims;
    out[4] = c->helpers;
    out[5] = (int64_t)c->handoffs;
    out[6] = c->done;
}

bool dpll_scan_eligible(int max_vars, int max_clauses, int max_lits, int max_clause_len, bool inc,
                        uint32_t *lds_bytes) {
    const int K = pick_k(max_vars, max_clause_len);
    if (!K || max_lits > 65535) return false;
    ScanLayout lay;
    if (!make_layout(K, max_vars, max_clauses, true, inc, 2u, &lay)) return false;
    if (lds_bytes) *lds_bytes = lay.bytes;
    return true;
}

int dpll_scan_resident(int max_vars, int max_clauses, int max_clause_len, bool inc, int *waves_per_cu,
                       uint32_t *lds_per_wave) {
    const int K = pick_k(max_vars, max_clause_len);
    if (!K) return SATMI_ERR_ARG;
    ScanPlan P;
    const int rc = scan_plan(K, max_vars, max_clauses, inc, &P);
    if (rc) return rc;
    *waves_per_cu = P.waves_per_wg * P.wg_per_cu;
    if (lds_per_wave) *lds_per_wave = P.fixed ? FIX_LDS_BYTES : P.lay.bytes + (uint32_t)P.lvs;
    return SATMI_OK;
}

int dpll_scan_launch(const ScanLaunch &L) {
    const int K = pick_k(L.max_vars, L.max_clause_len);
    ScanPlan P;
    if (!K || !dpll_scan_eligible(L.max_vars, L.max_clauses, L.max_lits, L.max_clause_len, L.inc, nullptr)) {
        set_error("dpll_scan_launch: batch shape not eligible for the scan kernel");
        return SATMI_ERR_ARG;
    }
    const int prc = scan_plan(K, L.max_vars, L.max_clauses, L.inc, &P);
    if (prc) return prc;
    const ScanLayout &lay = P.lay;
    const int waves_per_wg = P.waves_per_wg;
    const uint32_t wg_lds = lay.bytes * (uint32_t)waves_per_wg;
    const int need = (L.num_instances + waves_per_wg - 1) / waves_per_wg;
    int grid = std::max(1, std::min(need, L.num_cus * P.wg_per_cu));

    ScanArgs A;
    A.inst_clause_begin = L.inst_clause_begin;
    A.clause_lit_begin = L.clause_lit_begin;
    A.lits = L.lits;
    A.inst_nvars = L.inst_nvars;
    A.num_instances = L.num_instances;
    A.sol_cap = L.sol_cap;
    A.sol_stride = L.sol_stride;
    A.max_solutions = L.max_solutions;
    A.node_limit = L.node_limit;
    A.time_limit_ticks = L.time_limit_ticks;
    A.status = L.status;
    A.counters = L.counters;
    A.sol_len = L.sol_len;
    A.sol_lits = L.sol_lits;
    A.root_len = L.root_len;
    A.root_lits = L.root_lits;
    A.work_counter = L.work_counter;
    A.occ = nullptr;
    A.occ_cap = 0;
    A.occ_lists = 0;
    A.snap_lds = P.fixed ? 0u : snap_lds_entries(K, P.lvs == 256 ? 1u : 2u, (uint32_t)lay.mcap + 1u);
    A.lay = lay;
    A.split = nullptr;
    // split only where the launch's tail matters: at most SPLIT_MAX_PER_WAVE
    // instances per resident wave (at 32 per wave the tail is a few percent and
    // the two-stream pipeline hides it; the split form's register cost is not;
    // at 16 -- the N=2 shard -- the unsplit form still ran 2.5 % faster, while
    // at 4 -- the N=8 shard -- one hard search in one rank's slice made that
    // rank 34 % slower than the others unsplit and the split form evened them),
    // but at least one per resident wave (a launch that leaves CU slots empty
    // from the start -- configs[1]: 4,096 short searches -- loses 7 % to the
    // split form and gains nothing: the other stream's launch fills those slots)
    const int64_t waves = (int64_t)grid * waves_per_wg;
    const bool few = L.split_always || ((int64_t)L.num_instances <= (int64_t)SPLIT_MAX_PER_WAVE * waves &&
                                        (int64_t)L.num_instances >= (int64_t)L.num_cus * P.wg_per_cu * waves_per_wg);
    if (L.split && L.split_alloc && few) {
        // slot pool: trail codes of the launch's entry width; one donation-stack
        // entry per decision frame per resident wave
        SplitCfg cfg{};
        const int ncap = P.fixed ? FIX_NCAP : lay.ncap;
        const int cbytes = (P.fixed || P.lvs == 256) ? 1 : 2;
        cfg.slot_bytes = slot_bytes_for(ncap, cbytes);
        cfg.cont_off = slot_cont_off(ncap, cbytes);
        cfg.cont_fb = slot_frames_bytes(ncap, cbytes);
        // slots are never reused within a launch: room for the donations of a
        // long split search (uf250 solved, 512 searches, 10 helpers per CU:
        // 2.6 * 10^5 per launch; a pool of 768 MB -- 2.9 * 10^5 uf250 slots --
        // ran dry at 16 helpers per CU and the helpers idled: 50.7 -> 9.4
        // instances/s).  2 GiB per stream of the 288 GB.
        cfg.slot_cap = (int)std::min<size_t>(1u << 21, ((size_t)2048 << 20) / (size_t)cfg.slot_bytes);
        cfg.dstack_cap = ncap + 1;
        cfg.max_helpers = L.num_cus * L.split_helpers_per_cu;
        cfg.warm = (uint32_t)std::max(L.split_warmup, 0);
        // a batch smaller than the resident slots (split always: configs[4]
        // solved to the end) gets its helpers from the start: waves beyond the
        // instances find the queue empty and register as helpers at once, so
        // the hard searches' subtrees spread over idle CU slots instead of
        // waiting for the easy instances to finish
        const int64_t with_helpers = ((int64_t)L.num_instances + cfg.max_helpers + waves_per_wg - 1) / waves_per_wg;
        grid = (int)std::max<int64_t>(grid, std::min<int64_t>(with_helpers, (int64_t)L.num_cus * P.wg_per_cu));
        const size_t pool = (size_t)cfg.slot_cap * (size_t)cfg.slot_bytes;
        const size_t stacks = (size_t)grid * (size_t)waves_per_wg * (size_t)cfg.dstack_cap * sizeof(int32_t);
        uint32_t epoch = 0;
        void *p = L.split_alloc(SPLIT_POOL_OFF + pool + stacks, &epoch);
        if (!p) {
            set_error("dpll_scan_launch: no scratch for branch splitting");
            return SATMI_ERR_NOMEM;
        }
        cfg.epoch = epoch & 0x0FFFFFFFu;
        // written by a one-wave kernel on the launch's stream, the header by
        // value in its arguments: a copy from this pageable host struct would
        // make the runtime stage it synchronously, and the host then waits for
        // the stream's earlier work before it can queue the next launch -- the
        // two-stream overlap of the bench's steps was lost that way (split
        // form at full size: launch +1 %, step rate -5 %)
        hipLaunchKernelGGL(split_init_kernel, dim3(1), dim3(64), 0, L.stream, (SplitCfg *)p, cfg);
        A.split = (SplitCfg *)p;
    }
    // per resident wave: occurrence lists (max_lits entries, rounded to 128 B),
    // then the snapshot entries LDS does not hold (<= one per clause)
    if (L.inc) A.occ_lists = (std::max(L.max_lits, 1) + 63) & ~63;
    const int snap_ovf = (!P.fixed && (uint32_t)lay.mcap + 1u > A.snap_lds) ? ((lay.mcap + 1 - (int)A.snap_lds) + 63) & ~63 : 0;
    A.occ_cap = A.occ_lists + snap_ovf;
    if (A.occ_cap > 0) {
        const size_t bytes = (size_t)grid * (size_t)waves_per_wg * (size_t)A.occ_cap * sizeof(uint16_t);
        A.occ = L.occ_alloc ? L.occ_alloc(bytes) : nullptr;
        if (!A.occ) {
            set_error("dpll_scan_launch: no per-wave scratch (occurrence lists / snapshot)");
            return SATMI_ERR_NOMEM;
        }
    }
    const dim3 g(grid), blk(64 * waves_per_wg);
    const bool sp = A.split != nullptr;
    if (P.fixed && sp) hipLaunchKernelGGL((dpll_fixed_kernel<FIX_MCAP, true>), g, blk, 0, L.stream, A);
    else if (P.fixed) hipLaunchKernelGGL((dpll_fixed_kernel<FIX_MCAP, false>), g, blk, 0, L.stream, A);
    else if (L.inc && sp) launch_kernel<true, true>(K, P.lvs, g, blk, wg_lds, L.stream, A);
    else if (L.inc) launch_kernel<true, false>(K, P.lvs, g, blk, wg_lds, L.stream, A);
    else if (sp) launch_kernel<false, true>(K, P.lvs, g, blk, wg_lds, L.stream, A);
    else launch_kernel<false, false>(K, P.lvs, g, blk, wg_lds, L.stream, A);
    SATMI_HIP(hipGetLastError());
    return SATMI_OK;
}

}  // namespace satmi
