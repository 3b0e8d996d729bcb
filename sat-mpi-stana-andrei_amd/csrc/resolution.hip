// resolution.hip -- resolution saturation (REF.py:63-95) on gfx950.
//
// The reference keeps Python sets of literals and, every pass, resolves every
// pair (i < j) of its clause list on every clashing literal, skips tautologies,
// returns False on an empty resolvent and adds the resolvents it has not seen;
// True when a pass adds nothing.  Each pass's new-clause *set* does not depend
// on iteration order, so the GPU formulation is free to pick its own:
//
//   * a clause is a key of K = 2W uint64 words: positive / negative literal
//     bitsets over the formula's dense variable index (encode_keys_kernel);
//   * pair kernel (a workgroup per clause j, its key in registers, 256 keys i
//     per step): clash = (Pi & Nj) | (Ni & Pj).
//     Two or more clashing variables make every resolvent a tautology (the
//     other clash survives in both signs); with exactly one, the resolvent is
//     (Pi|Pj, Ni|Nj) minus that variable, a tautology iff its two halves meet,
//     empty iff both are zero.  Candidates are appended with one atomic per
//     wavefront (ballot + popcount);
//   * hash dedup: one open-addressing table per pass over every clause key
//     (the reference's `seen`); every candidate claims its key's slot run
//     with a 64-bit CAS, and the claimers -- the pass's new clauses -- are
//     compacted (flag scan) and appended to the clause array;
//   * a pass runs in chunks of about PAIR_CHUNK pairs: candidates of a chunk
//     (a buffer of the chunk's worst case), their claims, the winners
//     appended -- memory is bounded by the chunk and the new clauses, not by
//     the pass's candidates -- and the deadline is checked between chunks, so
//     a long pass ends as a timeout (REF.py:417-437);
//   * semi-naive passes: pairs whose newer clause was added in the previous pass
//     (all pairs in pass 1) -- every older pair was resolved in an earlier pass
//     and its resolvents are already in `seen`, so the new set is identical.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstddef>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "common.h"
#include "prims.h"

namespace satmi {

// dense variable index per variable id (-1: absent), keys[c*K ..] from CSR literals
__global__ void encode_keys_kernel(int nclauses, const int32_t *off, const int32_t *lits, const int32_t *var2dense,
                                   int W, uint64_t *keys) {
    const int K = 2 * W;
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < nclauses; c += gridDim.x * blockDim.x) {
        uint64_t *k = keys + (int64_t)c * K;
        for (int w = 0; w < K; ++w) k[w] = 0ull;
        for (int j = off[c]; j < off[c + 1]; ++j) {
            const int x = lits[j];
            const int d = var2dense[x < 0 ? -x : x];
            k[(x < 0 ? W : 0) + (d >> 6)] |= 1ull << (d & 63);
        }
    }
}

__device__ __forceinline__ int64_t tri(int64_t j) { return j * (j - 1) / 2; }   // pairs (i<j') with j' < j

// The resolvent of keys a and b on their single clashing variable
// (word cw, bit cbit): (Pa|Pb, Na|Nb) minus that variable.
template <typename KB>
__device__ __forceinline__ void resolvent(const uint64_t *a, KB &&B, int W, int cw, uint64_t cbit, uint64_t *r) {
    for (int w = 0; w < W; ++w) {
        uint64_t rp = a[w] | B(w), rn = a[W + w] | B(W + w);
        if (w == cw) {
            rp &= ~cbit;
            rn &= ~cbit;
        }
        r[w] = rp;
        r[W + w] = rn;
    }
}

// Classify pair (a, b): 1 = candidate resolvent (clash word / bit out), 0 =
// no resolvent or a tautology, 2 = the empty resolvent.
template <int WT, typename KB>
__device__ __forceinline__ int classify(const uint64_t *a, KB &&B, int W, int *cw, uint64_t *cbit) {
    int nclash = 0;
#pragma unroll
    for (int w0 = 0; w0 < (WT ? WT : 1); ++w0) {
        for (int w = w0; w < W; w += (WT ? WT : 1)) {
            const uint64_t c = (a[w] & B(W + w)) | (a[W + w] & B(w));
            if (c) {
                nclash += __popcll(c);
                *cw = w;
                *cbit = c & (~c + 1ull);
            }
        }
    }
    if (nclash != 1) return 0;   // no clash, or >= 2: every resolvent is a tautology
    bool taut = false, empty = true;
    for (int w = 0; w < W; ++w) {
        uint64_t rp = a[w] | B(w), rn = a[W + w] | B(W + w);
        if (w == *cw) {
            rp &= ~*cbit;
            rn &= ~*cbit;
        }
        taut |= (rp & rn) != 0ull;
        empty &= (rp | rn) == 0ull;
    }
    return taut ? 0 : (empty ? 2 : 1);
}

// Pairs (i, j), i < j, for j in [j_begin, j_end): one workgroup per clause j
// (grid-stride), 256 i's per step -- key j stays in registers (WT = W words
// per sign known at compile time; WT = 0 reads it from memory), keys i stream
// coalesced.  The candidates' i indices collect in an LDS buffer and are
// flushed with ONE append atomic per buffer (a single global counter takes
// under ~90 atomics per microsecond chip-wide: one per wavefront step was the
// kernel's bound); slot k (from *count, started at `slot_base`) goes to
// cand[k - slot_base] when it fits in cand_cap -- a sweep that overflows is
// re-run with a larger buffer.
constexpr int PAIR_BUF = 2048;
template <int WT>
__global__ void __launch_bounds__(256) res_pairs_kernel(const uint64_t *keys, int Wrt, int64_t j_begin, int64_t j_end,
                                                        unsigned long long *count, int *empty_found,
                                                        uint64_t *cand, int64_t cand_cap, int64_t slot_base) {
    __shared__ int32_t ibuf[PAIR_BUF];
    __shared__ int nbuf;
    __shared__ unsigned long long base_sh;
    const int W = WT ? WT : Wrt;
    const int K = 2 * W;
    const int ln = lane_id();
    if (threadIdx.x == 0) nbuf = 0;
    __syncthreads();
    for (int64_t j = j_begin + blockIdx.x; j < j_end; j += gridDim.x) {
        const uint64_t *b = keys + j * K;
        uint64_t bj[WT ? 2 * WT : 1];
        if constexpr (WT > 0) {
#pragma unroll
            for (int w = 0; w < 2 * WT; ++w) bj[w] = b[w];
        }
        const auto B = [&](int w) { return WT ? bj[WT ? w : 0] : b[w]; };
        const auto flush = [&]() {
            // block-uniform: called between __syncthreads with nbuf settled
            const int n = nbuf;
            if (threadIdx.x == 0) base_sh = atomicAdd(count, (unsigned long long)n);
            __syncthreads();
            const int64_t base = (int64_t)base_sh - slot_base;
            for (int t = threadIdx.x; t < n; t += blockDim.x) {
                const int64_t slot = base + t;
                if (slot < 0 || slot >= cand_cap) continue;
                const uint64_t *a = keys + (int64_t)ibuf[t] * K;
                int cw = 0;
                uint64_t cbit = 0;
                (void)classify<WT>(a, B, W, &cw, &cbit);
                resolvent(a, B, W, cw, cbit, cand + slot * K);
            }
            __syncthreads();
            if (threadIdx.x == 0) nbuf = 0;
            __syncthreads();
        };
        for (int64_t i0 = 0; i0 < j; i0 += blockDim.x) {
            const int64_t i = i0 + threadIdx.x;
            int cls = 0, cw = 0;
            uint64_t cbit = 0;
            if (i < j) cls = classify<WT>(keys + i * K, B, W, &cw, &cbit);
            if (cls == 2) *empty_found = 1;   // REF.py:84-85
            const uint64_t m = __ballot(cls == 1);
            if (m) {
                int pos = 0;
                if (ln == 0) pos = atomicAdd(&nbuf, __popcll(m));
                pos = uniform_i32(pos) + __popcll(m & lanemask_lt());
                if (cls == 1) ibuf[pos] = (int32_t)i;
            }
            // block-uniform flush decision: every wave reads the settled count
            // before any wave can append again (a second barrier), and the
            // last step of j flushes whatever is buffered
            __syncthreads();
            const int nb = nbuf;
            __syncthreads();
            const bool last = i0 + (int64_t)blockDim.x >= j;
            if (nb > (last ? 0 : PAIR_BUF - (int)blockDim.x)) flush();
        }
    }
}

// ---- dedup by hashing: one open-addressing table per pass over every clause
// key (the reference's `seen`, REF.py:65/94) and every candidate.  A candidate
// is new iff it is the first to claim its key's slot run: neither an old
// clause nor an earlier-claiming equal candidate holds the key.  Which of
// several equal candidates wins is left to the hardware; the *set* of new
// keys -- all REF.py's pass depends on -- is not.  Expected O(1) probes per
// key at load factor <= 1/2, against the O(n log^2 n) of a comparison sort.
constexpr uint64_t HT_EMPTY = ~0ull;
constexpr uint64_t CAND_BIT = 1ull << 62;   // table value: candidate (append slot) vs clause index

struct KeySrc {
    const uint64_t *clauses, *cand;
    int64_t base;   // append slot of cand[0]
    int K;
    __device__ __forceinline__ const uint64_t *at(uint64_t v) const {
        return (v & CAND_BIT) ? cand + ((int64_t)(v & ~CAND_BIT) - base) * K : clauses + (int64_t)v * K;
    }
};

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t key_hash(const uint64_t *x, int K) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (int w = 0; w < K; ++w) h = mix64(h ^ x[w]) + (uint64_t)w;
    return h;
}

__device__ __forceinline__ bool key_eq(const uint64_t *a, const uint64_t *b, int K) {
    for (int w = 0; w < K; ++w)
        if (a[w] != b[w]) return false;
    return true;
}

// Claim a slot for value v (key x): the slot if x was absent, else -1.
__device__ int64_t ht_insert(uint64_t *table, uint64_t mask, const KeySrc &S, uint64_t v, const uint64_t *x) {
    uint64_t s = key_hash(x, S.K) & mask;
    for (;;) {
        uint64_t cur = __hip_atomic_load(table + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == HT_EMPTY) {
            cur = atomicCAS((unsigned long long *)(table + s), (unsigned long long)HT_EMPTY, (unsigned long long)v);
            if (cur == HT_EMPTY) return (int64_t)s;
        }
        if (key_eq(S.at(cur), x, S.K)) return -1;
        s = (s + 1) & mask;
    }
}

// clauses [c0, c1) into the table (an input clause equal to an earlier one stays out)
__global__ void ht_clauses_kernel(uint64_t *table, uint64_t mask, KeySrc S, int64_t c0, int64_t c1) {
    for (int64_t c = c0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < c1; c += (int64_t)gridDim.x * blockDim.x)
        (void)ht_insert(table, mask, S, (uint64_t)c, S.clauses + c * S.K);
}

// flag[t] = candidate t claimed its key (new in this pass), slot[t] its table slot
__global__ void ht_cand_kernel(uint64_t *table, uint64_t mask, KeySrc S, int64_t n, int64_t *flag, int64_t *slot) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t sl = ht_insert(table, mask, S, CAND_BIT | (uint64_t)(S.base + t), S.cand + t * S.K);
        flag[t] = sl >= 0 ? 1 : 0;
        slot[t] = sl;
    }
}

// Packed table (at most 31 variables): a key (P, N) is one word P | N << 32 and
// the table holds the keys themselves, so a probe compares in register -- no
// second random read of the occupant's key -- and nothing is re-pointed at
// append time.  Bit 31 of P and N is never set, so no key equals HT_EMPTY.
__device__ __forceinline__ uint64_t pack_key(const uint64_t *x) { return x[0] | (x[1] << 32); }

// 1 if key k claimed a slot (absent before), 0 if it was present
__device__ __forceinline__ int ht_insert_packed(uint64_t *table, uint64_t mask, uint64_t k) {
    uint64_t s = mix64(k) & mask;
    for (;;) {
        uint64_t cur = __hip_atomic_load(table + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == HT_EMPTY) {
            cur = atomicCAS((unsigned long long *)(table + s), (unsigned long long)HT_EMPTY, (unsigned long long)k);
            if (cur == HT_EMPTY) return 1;
        }
        if (cur == k) return 0;
        s = (s + 1) & mask;
    }
}

__global__ void ht_clauses_packed_kernel(uint64_t *table, uint64_t mask, const uint64_t *clauses, int64_t c0,
                                         int64_t c1) {
    for (int64_t c = c0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < c1; c += (int64_t)gridDim.x * blockDim.x)
        (void)ht_insert_packed(table, mask, pack_key(clauses + 2 * c));
}

__global__ void ht_cand_packed_kernel(uint64_t *table, uint64_t mask, const uint64_t *cand, int64_t n,
                                      int64_t *flag) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
        flag[t] = ht_insert_packed(table, mask, pack_key(cand + 2 * t));
    }
}

// clauses.extend(new): the claimed candidates become clauses first .. first +
// count, in append order; their table entries are re-pointed at the clause
// array (the candidate buffer is reused by the next chunk)
__global__ void res_append_kernel(const uint64_t *cand, const int64_t *flag, const int64_t *pos, const int64_t *slot,
                                  int64_t n, int K, uint64_t *clauses, int64_t first, uint64_t *table) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
        if (!flag[t]) continue;
        const int64_t c = first + pos[t];
        for (int w = 0; w < K; ++w) clauses[c * K + w] = cand[t * K + w];
        if (table) __hip_atomic_store(table + slot[t], (uint64_t)c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---- packed keys (at most 31 variables): one fused pass.  Every clause is
// one word P | N << 32, the dedup table holds the keys themselves and lives
// for the whole saturation (it IS the reference's `seen`, REF.py:65/94), so a
// pair's resolvent is classified and claimed in registers: no candidate
// buffer, no flags, no compaction.  A claim (the key was absent) appends the
// key after the clause list -- the pass's new-clause set is exactly the keys
// claimed, whatever the order the hardware claims them in.  A pass's sizes live
// on the device (ResState); the host enqueues passes without waiting.
struct ResState {
    int64_t ncl, jlo;             // clauses; first clause added by the previous pass
    unsigned long long count;     // claims of the last pass
    int64_t passes;
    int64_t pairs, candidates;    // whole saturation
    int64_t stripe_max;           // the last pass's largest stripe count (sizes a regrown stage)
    uint64_t tk_pass, pass_ticks; // the running pass kernel's start tick; pass kernel ticks summed
    uint64_t tk_last;             // the last pass kernel's ticks (added by finish_pass unless the pass overflowed)
    uint64_t clk_cyc, clk_ticks;  // sampled pass-kernel blocks: shader cycles (s_memtime) and device-clock
                                  // ticks (s_memrealtime) summed -- the live shader clock is their ratio
    uint64_t t0;                  // s_memrealtime at the start
    int32_t done, result, empty, timeout, overflow;
    int32_t spill;                // the pass's new keys outgrew the stage: counted, not stored
};

struct ResArgs {
    ResState *st;
    uint64_t *keys;      // packed clause keys, clause c at keys[c]
    int64_t key_cap;
    uint64_t *table;     // HT_EMPTY or a key, in buckets of RES_BUCKET slots
    uint64_t tmask;      // bucket mask
    int64_t *pass_new;   // device copy of the per-pass counts
    int pass_cap;
    int64_t max_passes, clause_limit;
    uint64_t limit_ticks;
    int64_t slot_base;   // test knob (satmi_resolution_debug_slot_base)
    // A pass's new keys are appended to RES_STRIPES staging regions (stripe =
    // block index mod RES_STRIPES, each with its own counter): one hot counter
    // serialises its atomics (~60 ns each under contention), so the appends are
    // spread over many, and res_gather_kernel packs the regions after the pass.
    uint64_t *stage;
    int64_t stage_region;            // keys per stripe region
    unsigned long long *stripes;     // [RES_STRIPES] append counts (from slot_base), [RES_STRIPES] candidates
};
constexpr int RES_STRIPES = 64;
// words after the stripes' 2 x RES_STRIPES counters, each group on its own 128-B line
constexpr int RES_CLK = 2 * RES_STRIPES;         // [RES_CLK], [RES_CLK + 1]: sampled shader cycles, device ticks
constexpr int RES_GDONE = 2 * RES_STRIPES + 16;  // gather blocks finished with the current pass
constexpr int RES_STRIPE_WORDS = 2 * RES_STRIPES + 32;
constexpr int RES_DONE_WORD = RES_STRIPE_WORDS;  // the last batch's S->done for the conditional reset (not reset)
constexpr int RES_STRIPE_ALLOC = RES_STRIPE_WORDS + 16;

// A probe run of this many full buckets means the table is filling up (at
// load <= 1/2 it practically never happens): the pass stops as an overflow and
// runs again on a larger table -- instead of probing a full table for ever.
constexpr int RES_PROBE_MAX = 32;
constexpr int RES_BUCKET = 8;             // slots per bucket: one 64-B read checks them all

// Claim key r in a bucketed linear-probing table (slot order: bucket b's 8
// slots, then bucket b+1's, ...; a key sits before the first empty slot of
// its sequence).  1 = r was absent and this call inserted it, 0 = present,
// -1 = the probe run exceeded RES_PROBE_MAX buckets.  The bucket is read with
// plain loads: a slot only ever changes from HT_EMPTY to a key, so a stale
// EMPTY is settled by the CAS and a key read is never wrong.
__device__ __forceinline__ int bucket_claim(uint64_t *table, uint64_t bmask, uint64_t r) {
    uint64_t b = (mix64(r) >> 3) & bmask;
    for (int probes = 0; probes < RES_PROBE_MAX; ++probes) {
        uint64_t *bk = table + b * RES_BUCKET;
        const ulonglong2 *v = (const ulonglong2 *)bk;
        const ulonglong2 q0 = v[0], q1 = v[1], q2 = v[2], q3 = v[3];
        const uint64_t sl[RES_BUCKET] = {q0.x, q0.y, q1.x, q1.y, q2.x, q2.y, q3.x, q3.y};
        uint32_t empty = 0;
#pragma unroll
        for (int k = 0; k < RES_BUCKET; ++k) {
            if (sl[k] == r) return 0;
            empty |= (sl[k] == HT_EMPTY ? 1u : 0u) << k;
        }
        while (empty) {   // claim the first slot that is really empty, in slot order
            const int k = __builtin_ctz(empty);
            empty &= empty - 1;
            const uint64_t cur =
                atomicCAS((unsigned long long *)(bk + k), (unsigned long long)HT_EMPTY, (unsigned long long)r);
            if (cur == HT_EMPTY) return 1;
            if (cur == r) return 0;
        }
        b = (b + 1) & bmask;
    }
    return -1;
}

// keys [c0, c1) into the table (an input clause equal to an earlier one stays out)
__global__ void __launch_bounds__(256) res_seed_kernel(uint64_t *table, uint64_t bmask, const uint64_t *keys,
                                                       int64_t c0, int64_t c1, ResState *S) {
    for (int64_t c = c0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < c1; c += (int64_t)gridDim.x * blockDim.x)
        if (bucket_claim(table, bmask, keys[c]) < 0) S->overflow = 1;
}

// The packed path's clean slate, enqueued when a call ends (and before a
// workspace's first call): the table emptied, the state and the stripes' words
// set for the next saturation.  It runs while the host returns the result, so
// the next call starts with one prologue launch instead of four.
__global__ void __launch_bounds__(256) res_reset_kernel(uint64_t *table, uint64_t tslots, ResState *S,
                                                        unsigned long long *stripes, int64_t slot_base, int cond) {
    // cond: only when the batch before ended the saturation (res_copyout_kernel's word)
    if (cond && stripes[RES_DONE_WORD] == 0ull) return;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < tslots; i += (uint64_t)gridDim.x * blockDim.x)
        table[i] = HT_EMPTY;
    if (blockIdx.x == 0) {
        const int t = threadIdx.x;
        if (t < RES_STRIPE_WORDS) stripes[t] = t < RES_STRIPES ? (unsigned long long)slot_base : 0ull;
        if (t == 0) {
            ResState z{};
            z.result = -1;
            *S = z;
        }
    }
}

// A batch's state and per-pass counts (`bytes`, a multiple of 4) into pinned
// host memory, then the flag the host spins on (a stream wait wakes the host
// ~20 us after the work ends); S->done kept for the reset that follows.
__global__ void __launch_bounds__(64) res_copyout_kernel(const unsigned char *src, uint32_t bytes, unsigned char *dst,
                                                         uint32_t *flag, unsigned long long *stripes) {
    for (uint32_t i = threadIdx.x * 4u; i < bytes; i += 64u * 4u) *(uint32_t *)(dst + i) = *(const uint32_t *)(src + i);
    if (threadIdx.x == 0) stripes[RES_DONE_WORD] = (unsigned long long)((const ResState *)src)->done;
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A call's prologue (table clean, state reset): clause c's key P | N << 32
// from the CSR literals (REF.py:66's clause sets: a repeated literal is one
// bit), into keys[c] and the table (an input clause equal to an earlier one
// stays out of the table, as the reference's `seen` set); the state's clause
// count and the deadline's start.
__global__ void __launch_bounds__(256) res_prologue_kernel(int nclauses, const int32_t *off, const int32_t *lits,
                                                           const int32_t *var2dense, uint64_t *keys, uint64_t *table,
                                                           uint64_t bmask, ResState *S) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        S->ncl = nclauses;
        S->t0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < nclauses; c += gridDim.x * blockDim.x) {
        uint32_t P = 0u, N = 0u;
        for (int j = off[c]; j < off[c + 1]; ++j) {
            const int x = lits[j];
            const uint32_t bit = 1u << var2dense[x < 0 ? -x : x];
            P |= x < 0 ? 0u : bit;
            N |= x < 0 ? bit : 0u;
        }
        const uint64_t k = (uint64_t)P | ((uint64_t)N << 32);
        keys[c] = k;
        if (bucket_claim(table, bmask, k) < 0)
            __hip_atomic_store(&S->overflow, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// One pass (REF.py:67-95) over the pairs (i < j), j in [jlo, ncl), in tiles of
// tj clauses j x 256 clauses i: block (x, y) takes j-tiles x, x + gx, ... and
// i-tiles y, y + gy, ... (tiles above the diagonal exit at once).  The tile's
// j keys sit in LDS (read by broadcast), each lane holds one key i and walks
// the tile's j's -- a key is read from memory once per tile.  tj adapts to the
// pass (about RES_TILES tiles, 1 <= tj <= RES_TJ): a small pass gets short
// tiles (no lane walks a long chain of probes), a large one long tiles.  A
// tile's new keys collect in an LDS buffer and are appended with ONE atomic
// on the pass's counter (a single global counter serialises: one atomic per
// wavefront with a claim was the kernel's bound).
constexpr int RES_TJ = 32, RES_ABUF = 1024;
constexpr int64_t RES_TILES = 16384;
__global__ void __launch_bounds__(256) res_pass_packed_kernel(ResArgs A) {
    __shared__ uint64_t jk[RES_TJ];
    __shared__ uint64_t abuf[RES_ABUF];
    __shared__ int wsum[4];
    __shared__ int sh_stop, an;
    __shared__ unsigned long long abase;
    ResState *S = A.st;
    if (S->done) return;
    // the kernel's duration on the device clock: from its first block's start
    // to the next kernel's (res_gather_kernel) -- no events, so it also works
    // inside the replayed graph
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) S->tk_pass = __builtin_amdgcn_s_memrealtime();
    const int64_t jlo = S->jlo, ncl = S->ncl;
    const uint64_t t0 = S->t0;
    const int ln = lane_id(), tid = threadIdx.x;
    const int stripe = (int)((blockIdx.y * gridDim.x + blockIdx.x) % RES_STRIPES);
    // the live shader clock: one block in RES_STRIPES stamps both clocks around its work
    const bool clk_sample = stripe == 0 && threadIdx.x == 0;
    const uint64_t c_begin = clk_sample ? __builtin_amdgcn_s_memtime() : 0ull;
    const uint64_t r_begin = clk_sample ? __builtin_amdgcn_s_memrealtime() : 0ull;
    // tiles ~ (ncl - jlo) / tj x ncl / 512 (the triangle) ~ RES_TILES
    const int tj = (int)max<int64_t>(1, min<int64_t>(RES_TJ, (ncl - jlo) * (ncl / 512 + 1) / RES_TILES));
    int cand = 0;
    bool halt = false;   // block-uniform: a flag or the deadline ended the pass
    const int64_t njt = (ncl - jlo + tj - 1) / tj;
    for (int64_t jt = blockIdx.x; jt < njt && !halt; jt += gridDim.x) {
        const int64_t j0 = jlo + jt * tj, j1 = min<int64_t>(j0 + tj, ncl);
        const int nj = (int)(j1 - j0);
        for (int64_t i0 = (int64_t)blockIdx.y * 256; i0 < j1 - 1; i0 += (int64_t)gridDim.y * 256) {
            if (tid == 0) {
                int stop = __hip_atomic_load(&S->empty, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) |
                           __hip_atomic_load(&S->overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (!stop && A.limit_ticks && __builtin_amdgcn_s_memrealtime() - t0 > A.limit_ticks) {
                    __hip_atomic_store(&S->timeout, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    stop = 1;
                }
                sh_stop = stop;
                an = 0;
            }
            if (tid < nj) jk[tid] = A.keys[j0 + tid];
            __syncthreads();
            if (sh_stop) {   // block-uniform
                halt = true;
                break;
            }
            const int64_t i = i0 + tid;
            const uint64_t a = i < j1 ? A.keys[i] : 0ull;
            const uint32_t Pa = (uint32_t)a, Na = (uint32_t)(a >> 32);
            const int first = (int)max<int64_t>(0, i + 1 - j0);   // j's of this tile above i
            for (int jj = 0; jj < nj; ++jj) {
                // the deadline inside the tile too (per wave, every 8 clauses j)
                if ((jj & 7) == 7 && A.limit_ticks && __builtin_amdgcn_s_memrealtime() - t0 > A.limit_ticks) {
                    if (ln == 0) __hip_atomic_store(&S->timeout, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                bool win = false;
                uint64_t r = 0;
                if (jj >= first && i < j1) {
                    const uint64_t b = jk[jj];
                    const uint32_t Pb = (uint32_t)b, Nb = (uint32_t)(b >> 32);
                    const uint32_t clash = (Pa & Nb) | (Na & Pb);
                    // exactly one clashing variable: the resolvent (two or more
                    // make every resolvent a tautology, REF.py:81)
                    if (clash && !(clash & (clash - 1))) {
                        const uint32_t P = (Pa | Pb) & ~clash, N = (Na | Nb) & ~clash;
                        if (!(P & N)) {
                            if (!(P | N)) {
                                __hip_atomic_store(&S->empty, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // REF.py:84-85
                            } else {
                                ++cand;
                                r = (uint64_t)P | ((uint64_t)N << 32);
                                const int c = bucket_claim(A.table, A.tmask, r);
                                win = c > 0;
                                if (c < 0) __hip_atomic_store(&S->overflow, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            }
                        }
                    }
                }
                const uint64_t m = __ballot(win);
                if (m) {   // clauses.extend(new), staged in the tile's LDS buffer
                    int pos = 0;
                    if (ln == 0) pos = atomicAdd(&an, __popcll(m));
                    pos = __shfl(pos, 0) + __popcll(m & lanemask_lt());
                    if (win) {
                        if (pos < RES_ABUF) {
                            abuf[pos] = r;
                        } else {   // a full buffer (rare): append directly
                            const int64_t idx =
                                (int64_t)(atomicAdd(A.stripes + stripe, 1ull) - (unsigned long long)A.slot_base);
                            if (idx < A.stage_region)
                                A.stage[stripe * A.stage_region + idx] = r;
                            else   // counted, not stored: the pass goes on, so its count is exact
                                __hip_atomic_store(&S->spill, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        }
                    }
                }
            }
            __syncthreads();
            const int na = min(an, RES_ABUF);
            if (na) {   // the tile's new keys: one append atomic on the block's stripe
                if (tid == 0) abase = atomicAdd(A.stripes + stripe, (unsigned long long)na);
                __syncthreads();
                const int64_t f0 = (int64_t)(abase - (unsigned long long)A.slot_base);
                for (int t = tid; t < na; t += 256) {
                    if (f0 + t < A.stage_region)
                        A.stage[stripe * A.stage_region + f0 + t] = abuf[t];
                    else
                        __hip_atomic_store(&S->spill, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            __syncthreads();   // jk / abuf / sh_stop are rewritten by the next tile
        }
    }
    int tot;
    {   // block sum of the candidates (every thread reaches here)
        const int incl = wave_incl_scan(cand);
        if (ln == 63) wsum[tid >> 6] = incl;
        __syncthreads();
        tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    }
    if (tid == 0 && tot) atomicAdd(A.stripes + RES_STRIPES + stripe, (unsigned long long)tot);
    if (clk_sample) {
        const uint64_t dc = __builtin_amdgcn_s_memtime() - c_begin, dr = __builtin_amdgcn_s_memrealtime() - r_begin;
        atomicAdd(A.stripes + RES_CLK, (unsigned long long)dc);   // (off the state's polled line)
        atomicAdd(A.stripes + RES_CLK + 1, (unsigned long long)dr);
    }
}

// the verdict of a pass with nnew new clauses, or the next pass's bounds
__device__ void finish_pass(const ResArgs &A, ResState *S, int64_t nnew, int64_t cands) {
    if (S->overflow) {   // the host grows the buffers and runs this pass again (its work and time count then)
        S->done = 1;
        return;
    }
    S->candidates += cands;
    S->pass_ticks += S->tk_last;
    S->pairs += (S->ncl * (S->ncl - 1) - S->jlo * (S->jlo - 1)) / 2;
    if (S->empty) {   // an empty resolvent: unsatisfiable (REF.py:84-85)
        S->result = 0;
        S->done = 1;
        return;
    }
    if (S->timeout) {   // the deadline ended the pass early (REF.py:417-437)
        S->done = 1;
        return;
    }
    if (nnew == 0) {   // no new clauses can be derived (REF.py:91-92)
        S->result = 1;
        S->done = 1;
        return;
    }
    if (S->passes < A.pass_cap) A.pass_new[S->passes] = nnew;
    S->passes += 1;
    S->jlo = S->ncl;
    S->ncl += nnew;
    if ((A.max_passes > 0 && S->passes >= A.max_passes) || (A.clause_limit > 0 && S->ncl > A.clause_limit))
        S->done = 1;   // result stays -1
}

// After a pass: its new keys packed from the stripe regions behind the clause
// list (grid: x blocks per stripe, RES_STRIPES in y); then the block that
// finishes last sums the claims over the stripes, takes the verdict or sets
// the next pass's bounds and resets the counters -- one launch per pass
// instead of a gather and a one-workgroup finish kernel (each launch boundary
// was ~4.6 us of a php-res call).  The last block needs nothing else the
// other blocks wrote in this launch (the counts are the pass kernel's
// atomics, the overflow conditions it derives itself) except block (0,0)'s
// S->tk_last, so only that block's count is a release (and the last block
// fences); every block has read the stripes and the state before its count,
// so the last block may rewrite them.
__global__ void __launch_bounds__(256) res_gather_kernel(ResArgs A) {
    __shared__ int64_t pre[RES_STRIPES + 1];
    __shared__ int64_t cnt[RES_STRIPES], cand[RES_STRIPES];
    __shared__ int sh_last;
    ResState *S = A.st;
    const int tid = threadIdx.x;
    if (blockIdx.x == 0 && blockIdx.y == 0 && tid == 0 && !S->done)
        S->tk_last = __builtin_amdgcn_s_memrealtime() - S->tk_pass;
    // S->done changes only in the last block below, after every block has
    // read it: all blocks return here together
    if (S->done) return;
    const int64_t ncl = S->ncl;
    // the pass overflowed (table), or the stage held a part of its keys: the
    // host regrows and runs the pass again -- nothing to copy
    const bool skip = S->overflow || S->spill;
    if (tid == 0) {
        int64_t acc = 0;
        for (int t = 0; t < RES_STRIPES; ++t) {
            pre[t] = acc;
            acc += (int64_t)(A.stripes[t] - (unsigned long long)A.slot_base);
        }
        pre[RES_STRIPES] = acc;
    }
    __syncthreads();
    // (the next clause list must fit the key buffer)
    if (!skip && ncl + pre[RES_STRIPES] <= A.key_cap) {
        const int st = blockIdx.y;
        const int64_t n = pre[st + 1] - pre[st];
        for (int64_t t = (int64_t)blockIdx.x * blockDim.x + tid; t < n; t += (int64_t)gridDim.x * blockDim.x)
            A.keys[ncl + pre[st] + t] = A.stage[st * A.stage_region + t];
    }
    __syncthreads();
    if (tid == 0) {
        const unsigned long long nb = (unsigned long long)gridDim.x * gridDim.y;
        // block (0,0) wrote S->tk_last in this launch: its count is a release
        // (the other blocks' stay relaxed and continue its release sequence),
        // and the last block takes an acquire fence below before finish_pass
        // reads it
        const bool b00 = blockIdx.x == 0 && blockIdx.y == 0;
        const unsigned long long prev =
            b00 ? __hip_atomic_fetch_add(A.stripes + RES_GDONE, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT)
                : __hip_atomic_fetch_add(A.stripes + RES_GDONE, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sh_last = prev == nb - 1;
    }
    __syncthreads();
    if (!sh_last) return;
    if (tid == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (tid < RES_STRIPES) {
        cnt[tid] = (int64_t)(A.stripes[tid] - (unsigned long long)A.slot_base);
        cand[tid] = (int64_t)A.stripes[RES_STRIPES + tid];
        A.stripes[tid] = (unsigned long long)A.slot_base;
        A.stripes[RES_STRIPES + tid] = 0ull;
    }
    __syncthreads();
    if (tid != 0) return;
    A.stripes[RES_GDONE] = 0ull;
    int64_t claims = 0, cands = 0, smax = 0;
    for (int k = 0; k < RES_STRIPES; ++k) {
        claims += cnt[k];
        cands += cand[k];
        smax = max(smax, cnt[k]);
    }
    if (skip || ncl + claims > A.key_cap) S->overflow = 1;
    S->stripe_max = smax;
    S->count = (unsigned long long)claims;   // this pass's claims (a regrowth is sized by them)
    S->clk_cyc = A.stripes[RES_CLK];
    S->clk_ticks = A.stripes[RES_CLK + 1];
    finish_pass(A, S, claims, cands);
}

// ------------------------------------------------------------------ host side
namespace {

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    // grow to `bytes` (contents not kept); SATMI_ERR_NOMEM with a hint when the
    // device cannot hold it
    int reserve(size_t bytes) {
        if (bytes <= cap) return SATMI_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max(bytes, (size_t)256);
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && want > free_b) {
            set_error("satmi_resolution_host: out of device memory (" + std::to_string(want >> 20) + " MiB wanted, " +
                      std::to_string(free_b >> 20) + " MiB free); bound the saturation with clause_limit / "
                      "max_passes");
            return SATMI_ERR_NOMEM;
        }
        SATMI_HIP(hipMalloc(&p, want));
        cap = want;
        return SATMI_OK;
    }
    template <class T>
    T *as() const { return (T *)p; }
};

// Pinned host memory, grow-only: the call's inputs are gathered here and sent
// in one copy (a copy from pageable memory is staged synchronously, one per
// array), and small results come back through it.
struct PinBuf {
    unsigned char *p = nullptr;
    size_t cap = 0;
    ~PinBuf() {
        if (p) (void)hipHostFree(p);
    }
    int reserve(size_t bytes, unsigned flags = hipHostMallocDefault) {
        if (bytes <= cap) return SATMI_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max(bytes, (size_t)4096);
        SATMI_HIP(hipHostMalloc((void **)&p, want, flags));
        cap = want;
        return SATMI_OK;
    }
};

#define SATMI_TRY(x)                  \
    do {                              \
        int _rc = (x);                \
        if (_rc != SATMI_OK) return _rc; \
    } while (0)

uint64_t table_slots(int64_t keys) {
    uint64_t cap = 1024;
    while (cap < 2 * (uint64_t)keys) cap <<= 1;
    return cap;
}

// Pairs per chunk of a pass (the deadline is checked between chunks, so a long
// pass ends as a timeout, REF.py:417-437).  The candidate buffer holds a
// chunk's worst case (every pair a candidate) up to CAND_BYTES; past that it
// starts at CAND_BYTES, and a chunk whose candidates overflow it is re-run
// once with a buffer of the counted size.
constexpr int64_t PAIR_CHUNK = 1ll << 27;
constexpr size_t CAND_BYTES = (size_t)1 << 30;

int64_t g_slot_base = 0;            // test knob: first append slot of the pair kernel
size_t g_cand_bytes = CAND_BYTES;   // test knob: the candidate buffer's cap (forces the re-run path)

// Work and kernel time of the last satmi_resolution_host call (HIP events on
// its stream around the pair and claim launches): bench.py's roofline input.
struct ResStats {
    int64_t pairs = 0, candidates = 0, keys_tabled = 0;
    double pair_ms = 0.0, claim_ms = 0.0;
    double shader_hz = 0.0;   // the pass kernels' live shader clock (packed path; 0 = not sampled)
};
thread_local ResStats g_stats;   // the calling thread's last call

// Times launches on one stream: begin() / end() bracket them, total() sums.
struct EventTimer {
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
    size_t used = 0;
    ~EventTimer() {
        for (auto &e : ev) {
            (void)hipEventDestroy(e.first);
            (void)hipEventDestroy(e.second);
        }
    }
    hipEvent_t begin(hipStream_t s) {
        if (used == ev.size()) {
            hipEvent_t a = nullptr, b = nullptr;
            if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return nullptr;
            ev.push_back({a, b});
        }
        (void)hipEventRecord(ev[used].first, s);
        return ev[used].first;
    }
    void end(hipStream_t s) { (void)hipEventRecord(ev[used++].second, s); }
    void reset() { used = 0; }
    double total() {   // after the stream drained
        double ms = 0.0;
        for (size_t i = 0; i < used; ++i) {
            float t = 0.0f;
            if (hipEventElapsedTime(&t, ev[i].first, ev[i].second) == hipSuccess) ms += t;
        }
        return ms;
    }
};

// Device buffers of satmi_resolution_host, kept between calls (grow-only) in a
// process-wide pool: a call takes a free workspace of its device (or makes
// one) and returns it when done, so concurrent calls from any number of host
// threads each own one, overlap on the device (each its own non-blocking
// stream), and the number of workspaces is the peak number of concurrent
// calls.  A saturation of a small formula is a few passes of small launches,
// so allocating its buffers per call cost more than its kernels.
// The packed path's first segment of a call (state init, key packing, table
// seeding, the first batch of passes, the state's copy back), captured into a
// HIP graph the second time the same segment is enqueued and replayed from
// then on: one launch instead of ~16 host submissions, whose gaps were a
// quarter of a php-res call.  Keyed by everything its launches read from the
// host.
struct ResGraph {
    hipGraphExec_t exec = nullptr;
    ResArgs args;
    int64_t ncl = -1;
    uint64_t tslots = 0;
    int batch = 0;
    const void *down = nullptr;     // non-null: the segment copies the per-pass counts back too
    const void *pstate = nullptr;   // the pinned buffer the segment copies into
    ResGraph() { std::memset(&args, 0, sizeof(args)); }
    void reset() {
        if (exec) (void)hipGraphExecDestroy(exec);
        exec = nullptr;
        ncl = -1;
    }
};

struct ResWork {
    DevBuf clauses, cand, counters, table, flag, pos, slotv, tiles, grand;
    DevBuf keys, state, stage, stripes;            // the packed path (state: ResState, then the per-pass counts)
    DevBuf up;                                     // the call's inputs (one copy from up_h)
    PinBuf up_h, pstate;                           // pinned staging: inputs; the state and counts back
    struct Clean {   // the buffers the last reset (packed path) left clean; all null: not clean
        const void *table = nullptr, *state = nullptr, *stripes = nullptr;
        int64_t slot_base = -1;
        bool operator==(const Clean &o) const {
            return table == o.table && state == o.state && stripes == o.stripes && slot_base == o.slot_base &&
                   table != nullptr;
        }
    } clean;
    EventTimer t_pairs, t_claims;
    hipStream_t stream = nullptr;
    unsigned long long *pin = nullptr;   // pinned host words (coherent): the general path's counters and claim
                                         // count; pin[7]: the packed path's batch flag (res_copyout_kernel)
    int dev = 0;
    ResGraph graph;
    ~ResWork() {   // only a workspace that failed part-way is destroyed (after its stream drained)
        graph.reset();
        if (stream) (void)hipStreamDestroy(stream);
        if (pin) (void)hipHostFree(pin);
    }
};

struct ResPool {
    std::mutex mu;
    std::vector<ResWork *> free_list;
};
ResPool &res_pool() {
    static ResPool *p = new ResPool;   // never destroyed: no hipFree after the runtime's teardown
    return *p;
}
ResWork *res_acquire(int dev) {
    ResPool &P = res_pool();
    {
        std::lock_guard<std::mutex> g(P.mu);
        for (size_t i = 0; i < P.free_list.size(); ++i)
            if (P.free_list[i]->dev == dev) {
                ResWork *w = P.free_list[i];
                P.free_list.erase(P.free_list.begin() + (long)i);
                return w;
            }
    }
    ResWork *w = new ResWork;
    w->dev = dev;
    if (hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc((void **)&w->pin, 64, hipHostMallocCoherent) != hipSuccess) {
        delete w;
        return nullptr;
    }
    return w;
}
// A call's hold on a workspace: back to the pool after a call that completed,
// destroyed after one that failed part-way (its table may hold stale keys).
struct ResLease {
    ResWork *w;
    bool ok = false;
    ~ResLease() {
        if (!w) return;
        if (ok) {
            ResPool &P = res_pool();
            std::lock_guard<std::mutex> g(P.mu);
            P.free_list.push_back(w);
        } else {
            (void)hipStreamSynchronize(w->stream);
            delete w;
        }
    }
};

// decode a pass's new keys (packed or bitset words) into sorted literal lists
void record_pass(const std::vector<uint64_t> &hkeys, int64_t nnew, bool packed, int W, int V,
                 const std::vector<int32_t> &dense2var, int passes, int32_t *h_rec_lits, int64_t rec_lit_cap,
                 int64_t *h_rec_clause_off, int64_t rec_clause_cap, int64_t *h_rec_pass_off, int64_t &rec_clauses,
                 int64_t &rec_lits) {
    // each clause as ascending literals, the clauses in ascending order
    // (deterministic whatever the append order)
    std::vector<std::vector<int32_t>> pass((size_t)nnew);
    for (int64_t c = 0; c < nnew; ++c) {
        for (int d = 0; d < V; ++d) {
            bool pos, neg;
            if (packed) {
                const uint64_t k = hkeys[(size_t)c];
                pos = (k >> d) & 1ull;
                neg = (k >> (32 + d)) & 1ull;
            } else {
                const uint64_t *k = hkeys.data() + c * 2 * W;
                pos = (k[d >> 6] >> (d & 63)) & 1ull;
                neg = (k[W + (d >> 6)] >> (d & 63)) & 1ull;
            }
            if (pos) pass[(size_t)c].push_back(dense2var[(size_t)d]);
            if (neg) pass[(size_t)c].push_back(-dense2var[(size_t)d]);
        }
        std::sort(pass[(size_t)c].begin(), pass[(size_t)c].end());
    }
    std::sort(pass.begin(), pass.end());
    for (const auto &cl : pass) {
        if (rec_clauses + 1 >= rec_clause_cap || rec_lits + (int64_t)cl.size() > rec_lit_cap) break;
        std::copy(cl.begin(), cl.end(), h_rec_lits + rec_lits);
        rec_lits += (int64_t)cl.size();
        h_rec_clause_off[++rec_clauses] = rec_lits;
    }
    h_rec_pass_off[passes + 1] = rec_clauses;
}


// grow the packed key buffer to >= want keys, keeping keys [0, keep)
int grow_keys(ResWork &wk, int64_t want, int64_t keep, hipStream_t s) {
    if ((size_t)want * 8 <= wk.keys.cap) return SATMI_OK;
    DevBuf grown;
    SATMI_TRY(grown.reserve(8 * (size_t)want));
    if (keep > 0) SATMI_HIP(hipMemcpyAsync(grown.p, wk.keys.p, 8 * (size_t)keep, hipMemcpyDeviceToDevice, s));
    std::swap(grown.p, wk.keys.p);
    std::swap(grown.cap, wk.keys.cap);
    SATMI_HIP(hipStreamSynchronize(s));   // before `grown` frees the old buffer
    return SATMI_OK;
}

// The packed path (<= 31 variables): the clause keys, the table and the state
// stay on the device for the whole saturation; passes are enqueued in batches
// and the host waits once per batch (once per pass when recording).  A pass
// that ran out of key or table room is re-run after the host grows them.
// A call is: the upload (one copy), one prologue launch (keys + table seed on
// the table the previous call's reset left empty), the passes with the state
// and per-pass counts back in one copy -- replayed from a HIP graph when the
// same call repeats -- and, not waited for, the reset for the next call.
int resolution_packed(ResWork &wk, int nclauses, const unsigned char *up, size_t o_lits, size_t o_map,
                      int64_t max_passes, int64_t clause_limit, double time_limit_s,
                      int64_t slot_base, int V, const std::vector<int32_t> &dense2var, int32_t *h_result,
                      int32_t *h_passes, int64_t *h_pass_new, int pass_cap, int32_t *h_rec_lits,
                      int64_t rec_lit_cap, int64_t *h_rec_clause_off, int64_t rec_clause_cap, int64_t *h_rec_pass_off,
                      int rec_pass_cap) {
    hipStream_t s = wk.stream;
    const auto t_call = std::chrono::steady_clock::now();
    const int PCAP = std::max(1, std::min(pass_cap, 1 << 16));   // passes whose counts the device keeps
    // the state and the per-pass counts in one buffer (one copy back per batch)
    const size_t SOFF = (sizeof(ResState) + 255) & ~(size_t)255;
    SATMI_TRY(wk.keys.reserve(8 * (size_t)std::max<int64_t>(4 * (int64_t)nclauses, 1 << 14)));
    SATMI_TRY(wk.state.reserve(SOFF + 8 * (size_t)PCAP));
    SATMI_TRY(wk.stripes.reserve(8 * RES_STRIPE_ALLOC));
    SATMI_TRY(wk.pstate.reserve(SOFF + 8 * (size_t)PCAP, hipHostMallocCoherent));
    int64_t key_cap = (int64_t)(wk.keys.cap / 8);
    // stripe regions: twice the key room (the stripes fill unevenly)
    SATMI_TRY(wk.stage.reserve(8 * 2 * (size_t)key_cap));
    // the table: a power of two >= 2x the keys it can hold (load <= 1/2; a
    // table larger than needed only spreads the probes over more cache lines)
    const auto slots_for = [](int64_t nkeys) {   // a power of two, >= 8 buckets
        uint64_t c = 1 << 12;
        while (c < 2 * (uint64_t)nkeys) c <<= 1;
        return c;
    };
    uint64_t tslots = slots_for(key_cap);
    SATMI_TRY(wk.table.reserve(8 * tslots));
    // the clean slate of the next call (the whole table emptied); cond: only
    // if the batch just copied out ended the saturation
    const auto reset = [&](int cond) -> int {
        const uint64_t all = wk.table.cap / 8;
        hipLaunchKernelGGL(res_reset_kernel, dim3((unsigned)std::min<uint64_t>(1024, (all + 255) / 256)), dim3(256), 0,
                           s, wk.table.as<uint64_t>(), all, wk.state.as<ResState>(),
                           wk.stripes.as<unsigned long long>(), slot_base, cond);
        SATMI_HIP(hipGetLastError());
        return SATMI_OK;
    };
    // a workspace whose buffers moved since its last reset (or its first call)
    const ResWork::Clean now{wk.table.p, wk.state.p, wk.stripes.p, slot_base};
    if (!(wk.clean == now)) SATMI_TRY(reset(0));
    wk.clean = ResWork::Clean{};   // dirty from here until the reset this call enqueues
    ResState &st = *(ResState *)wk.pstate.p;   // the host's copy, refreshed after each batch of passes
    const int64_t *pst_counts = (const int64_t *)(wk.pstate.p + SOFF);
    st = ResState{};
    st.ncl = nclauses;
    st.result = -1;
    const auto seed = [&](int64_t nkeys) -> int {   // a fresh table holding keys [0, nkeys) (regrowth)
        SATMI_HIP(hipMemsetAsync(wk.table.p, 0xFF, 8 * tslots, s));   // HT_EMPTY
        if (nkeys > 0)
            hipLaunchKernelGGL(res_seed_kernel, dim3(grid_for(nkeys)), dim3(256), 0, s, wk.table.as<uint64_t>(),
                               tslots / RES_BUCKET - 1, wk.keys.as<uint64_t>(), (int64_t)0, nkeys,
                               wk.state.as<ResState>());
        SATMI_HIP(hipGetLastError());
        return SATMI_OK;
    };
    // keys, table seed, clause count and the deadline's start (t0): one launch
    hipLaunchKernelGGL(res_prologue_kernel, dim3(grid_for(std::max(nclauses, 1))), dim3(256), 0, s, nclauses,
                       (const int32_t *)up, (const int32_t *)(up + o_lits), (const int32_t *)(up + o_map),
                       wk.keys.as<uint64_t>(), wk.table.as<uint64_t>(), tslots / RES_BUCKET - 1,
                       wk.state.as<ResState>());
    SATMI_HIP(hipGetLastError());
    double hz = 1e8;
    (void)satmi_wallclock_hz(&hz);
    ResArgs A;
    std::memset(&A, 0, sizeof(A));   // padding too: the first segment's graph is keyed by these bytes
    const auto args = [&]() {
        A.st = wk.state.as<ResState>();
        A.keys = wk.keys.as<uint64_t>();
        A.key_cap = key_cap;
        A.table = wk.table.as<uint64_t>();
        A.tmask = tslots / RES_BUCKET - 1;   // bucket mask
        A.pass_new = (int64_t *)(wk.state.as<unsigned char>() + SOFF);
        A.pass_cap = PCAP;
        A.max_passes = max_passes;
        A.clause_limit = clause_limit;
        A.limit_ticks = time_limit_s > 0 ? (uint64_t)std::max(1.0, time_limit_s * hz) : 0;
        A.slot_base = slot_base;
        A.stage = wk.stage.as<uint64_t>();
        A.stage_region = (int64_t)(wk.stage.cap / 8) / RES_STRIPES;
        A.stripes = wk.stripes.as<unsigned long long>();
    };
    args();
    g_stats = ResStats{};
    const bool record = h_rec_lits && h_rec_clause_off && h_rec_pass_off;
    int64_t rec_clauses = 0, rec_lits = 0;
    std::vector<uint64_t> hkeys;
    const dim3 pass_grid(256, 32);   // j-tiles x i-tiles, grid-stride
    // A batch of passes, then the state and counts back into pinned memory
    // with a flag the host spins on, then the next call's reset if the batch
    // ended the saturation (S->done -- set by an overflow too, whose regrowth
    // re-uploads the state and re-seeds the table)
    volatile uint32_t *flag = (volatile uint32_t *)(wk.pin + 7);
    const auto passes = [&](int batch) -> int {
        for (int b = 0; b < batch; ++b) {
            hipLaunchKernelGGL(res_pass_packed_kernel, pass_grid, dim3(256), 0, s, A);
            hipLaunchKernelGGL(res_gather_kernel, dim3(2, RES_STRIPES), dim3(256), 0, s, A);
        }
        const int64_t ncopy = h_pass_new ? std::min<int64_t>(PCAP, st.passes + batch) : 0;
        hipLaunchKernelGGL(res_copyout_kernel, dim3(1), dim3(64), 0, s, wk.state.as<unsigned char>(),
                           (uint32_t)(SOFF + 8 * (size_t)ncopy), wk.pstate.p, (uint32_t *)flag,
                           wk.stripes.as<unsigned long long>());
        SATMI_HIP(hipGetLastError());
        return reset(1);
    };
    // the batch's copy-out: spin on its flag (a stream wait sleeps ~20 us past
    // the end of short work), then a stream wait if it takes longer than 2 ms
    // (a long pass, or a fault: the wait reports it)
    const auto wait_batch = [&]() -> int {
        const auto t0 = std::chrono::steady_clock::now();
        while (*flag == 0u) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
                SATMI_HIP(hipStreamSynchronize(s));
                if (*flag == 0u) {
                    set_error("satmi_resolution_host: a batch ended without its state");
                    return SATMI_ERR_HIP;
                }
                break;
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        return SATMI_OK;
    };
    bool first = true;
    for (;;) {
        // passes per wait: all of them when the count is bounded (<= 16)
        const int64_t left = max_passes > 0 ? max_passes - st.passes : 4;
        const int batch = record ? 1 : (int)std::max<int64_t>(1, std::min<int64_t>(left, 16));
        const int64_t ncl_before = st.ncl;
        *flag = 0u;
        std::atomic_thread_fence(std::memory_order_release);
        if (first) {   // the first batch: replayed from the graph when it repeats
            first = false;
            ResGraph &G = wk.graph;
            const void *down = h_pass_new ? (const void *)wk.pstate.p : nullptr;
            const bool same = G.ncl == nclauses && G.tslots == tslots && G.batch == batch && G.down == down &&
                              G.pstate == wk.pstate.p && std::memcmp(&G.args, &A, sizeof(ResArgs)) == 0;
            if (same && G.exec) {
                SATMI_HIP(hipGraphLaunch(G.exec, s));
            } else if (same) {
                hipGraph_t graph = nullptr;
                SATMI_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
                const int rc = passes(batch);
                const hipError_t ec = hipStreamEndCapture(s, &graph);
                if (rc != SATMI_OK || ec != hipSuccess) {
                    if (graph) (void)hipGraphDestroy(graph);
                    G.reset();
                    if (rc != SATMI_OK) return rc;
                    SATMI_HIP(ec);
                }
                const hipError_t ei = hipGraphInstantiate(&G.exec, graph, nullptr, nullptr, 0);
                (void)hipGraphDestroy(graph);
                SATMI_HIP(ei);
                SATMI_HIP(hipGraphLaunch(G.exec, s));
            } else {   // remember the segment: captured if it comes again
                G.reset();
                G.args = A;
                G.ncl = nclauses;
                G.tslots = tslots;
                G.batch = batch;
                G.down = down;
                G.pstate = wk.pstate.p;
                SATMI_TRY(passes(batch));
            }
        } else {
            SATMI_TRY(passes(batch));
        }
        SATMI_TRY(wait_batch());
        if (st.overflow) {   // grow the key buffer and / or the table, re-seed, run the pass again
            if (time_limit_s > 0 &&
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t_call).count() >= time_limit_s)
                break;   // past the deadline: a timeout after the completed passes (result -1)
            // twice the claims of the stopped pass (all of its new keys when
            // the pass ran to its end -- the key buffer or the stage ran out,
            // the stage's excess counted, not stored; a part of them when the
            // table stopped it early)
            const int64_t claims = (int64_t)st.count;
            const int64_t want = std::max<int64_t>(2 * key_cap, st.ncl + 2 * claims + 1024);
            SATMI_TRY(grow_keys(wk, want, st.ncl, s));
            key_cap = (int64_t)(wk.keys.cap / 8);
            // stripe regions: twice the key room, and 5/4 of the fullest stripe
            // of the stopped pass (the finish kernel reset the stripes)
            const int64_t region = std::max<int64_t>(2 * key_cap / RES_STRIPES, st.stripe_max + st.stripe_max / 4 + 1024);
            SATMI_TRY(wk.stage.reserve(8 * (size_t)RES_STRIPES * (size_t)region));
            tslots = slots_for(key_cap);
            SATMI_TRY(wk.table.reserve(8 * tslots));
            args();
            st.overflow = 0;
            st.spill = 0;
            st.done = 0;
            st.empty = 0;
            st.timeout = 0;
            st.count = 0;
            SATMI_HIP(hipMemcpyAsync(wk.state.p, wk.pstate.p, sizeof(ResState), hipMemcpyHostToDevice, s));
            SATMI_TRY(seed(st.ncl));   // (after the state: a seed overflow flag must survive)
            continue;
        }
        if (record && st.passes > 0 && st.ncl > ncl_before && st.passes < rec_pass_cap) {
            const int64_t nnew = st.ncl - ncl_before;   // batch == 1: this pass's additions
            hkeys.resize((size_t)nnew);
            SATMI_HIP(hipMemcpyAsync(hkeys.data(), wk.keys.as<uint64_t>() + ncl_before, 8 * (size_t)nnew,
                                     hipMemcpyDeviceToHost, s));
            SATMI_HIP(hipStreamSynchronize(s));
            record_pass(hkeys, nnew, true, 1, V, dense2var, (int)st.passes - 1, h_rec_lits, rec_lit_cap,
                        h_rec_clause_off, rec_clause_cap, h_rec_pass_off, rec_clauses, rec_lits);
        }
        if (st.done) break;
    }
    // the counts came back with the last batch's state (the stream has drained)
    const int np = (int)std::min<int64_t>(st.passes, std::min(pass_cap, PCAP));
    if (h_pass_new && np > 0) std::memcpy(h_pass_new, pst_counts, 8 * (size_t)np);
    *h_result = st.result;
    *h_passes = (int32_t)st.passes;
    g_stats.pairs = st.pairs;
    g_stats.candidates = st.candidates;
    g_stats.pair_ms = (double)st.pass_ticks / hz * 1e3;   // device clock, pass kernels only
    g_stats.claim_ms = 0.0;   // fused into the pass kernel
    g_stats.shader_hz = st.clk_ticks ? (double)st.clk_cyc / (double)st.clk_ticks * hz : 0.0;
    // the last batch ended the saturation (S->done), so its reset is queued:
    // it runs while this result goes back to the caller
    wk.clean = now;
    return SATMI_OK;
}

}  // namespace

}  // namespace satmi

using namespace satmi;

extern "C" int satmi_resolution_last_stats(int64_t *pairs, int64_t *candidates, double *pair_ms, double *claim_ms) {
    if (pairs) *pairs = g_stats.pairs;
    if (candidates) *candidates = g_stats.candidates;
    if (pair_ms) *pair_ms = g_stats.pair_ms;
    if (claim_ms) *claim_ms = g_stats.claim_ms;
    return SATMI_OK;
}

extern "C" int satmi_resolution_last_clock(double *shader_hz) {
    if (!shader_hz) {
        set_error("satmi_resolution_last_clock: null pointer");
        return SATMI_ERR_ARG;
    }
    *shader_hz = g_stats.shader_hz;
    return SATMI_OK;
}

extern "C" int satmi_resolution_debug_cand_bytes(int64_t bytes) {
    if (bytes < 0) {
        set_error("satmi_resolution_debug_cand_bytes: negative size");
        return SATMI_ERR_ARG;
    }
    g_cand_bytes = bytes ? (size_t)bytes : CAND_BYTES;
    return SATMI_OK;
}

extern "C" int satmi_resolution_debug_slot_base(int64_t base) {
    if (base < 0 || base > (1ll << 61)) {
        set_error("satmi_resolution_debug_slot_base: base out of range");
        return SATMI_ERR_ARG;
    }
    g_slot_base = base;
    return SATMI_OK;
}

extern "C" int satmi_resolution_host(int nclauses, const int32_t *h_clause_off, const int32_t *h_lits,
                                     int64_t max_passes, int64_t clause_limit, double time_limit_s,
                                     int32_t *h_result, int32_t *h_passes, int64_t *h_pass_new, int pass_cap,
                                     int32_t *h_rec_lits, int64_t rec_lit_cap, int64_t *h_rec_clause_off,
                                     int64_t rec_clause_cap, int64_t *h_rec_pass_off, int rec_pass_cap) {
    if (nclauses < 0 || (nclauses > 0 && (!h_clause_off || !h_lits)) || !h_result || !h_passes) {
        set_error("satmi_resolution_host: bad arguments");
        return SATMI_ERR_ARG;
    }
    const auto t_start = std::chrono::steady_clock::now();
    const auto expired = [&]() {
        return time_limit_s > 0 &&
               std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count() > time_limit_s;
    };
    *h_result = -1;
    *h_passes = 0;
    if (h_rec_pass_off && rec_pass_cap > 0) h_rec_pass_off[0] = 0;
    if (h_rec_clause_off && rec_clause_cap > 0) h_rec_clause_off[0] = 0;
    // dense variable index (variables sorted by id)
    const int64_t L = nclauses > 0 ? h_clause_off[nclauses] : 0;
    int maxvar = 0;
    for (int64_t i = 0; i < L; ++i) {
        if (h_lits[i] == 0 || h_lits[i] == INT32_MIN) {
            set_error("satmi_resolution_host: literal 0 / INT32_MIN");
            return SATMI_ERR_ARG;
        }
        maxvar = std::max(maxvar, std::abs(h_lits[i]));
    }
    std::vector<int32_t> var2dense(maxvar + 1, -1), dense2var;
    for (int64_t i = 0; i < L; ++i) var2dense[std::abs(h_lits[i])] = 1;
    for (int v = 1; v <= maxvar; ++v)
        if (var2dense[v] >= 0) {
            var2dense[v] = (int32_t)dense2var.size();
            dense2var.push_back(v);
        }
    const int V = (int)dense2var.size();
    const int W = std::max(1, (V + 63) / 64);
    const int K = 2 * W;
    const bool packed = V <= 31;   // the packed table (see pack_key) and the fused pass
    const int64_t slot_base = g_slot_base;
    int dev_id = 0;
    SATMI_HIP(hipGetDevice(&dev_id));
    ResLease lease{res_acquire(dev_id)};
    if (!lease.w) {
        set_error("satmi_resolution_host: hipStreamCreate failed");
        return SATMI_ERR_HIP;
    }
    ResWork *wk = lease.w;
    hipStream_t s = wk->stream;
    DevBuf &clauses = wk->clauses, &cand = wk->cand, &counters = wk->counters;
    // the clause offsets, the literals and the variable map in one pinned
    // staging buffer, sent in one copy
    const auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t o_lits = al(4 * (size_t)(nclauses + 1)), o_map = o_lits + al(4 * (size_t)std::max<int64_t>(L, 1));
    const size_t up_bytes = o_map + al(4 * (size_t)(maxvar + 1));
    SATMI_TRY(wk->up.reserve(up_bytes));
    SATMI_TRY(wk->up_h.reserve(up_bytes));
    int64_t ncl = nclauses;
    SATMI_TRY(clauses.reserve(8 * (size_t)std::max<int64_t>(ncl, 1) * K));
    SATMI_TRY(counters.reserve(64));
    if (nclauses > 0) {
        // (the previous call's copy out of up_h finished: every call ends with a wait)
        std::memcpy(wk->up_h.p, h_clause_off, 4 * (size_t)(nclauses + 1));
        if (L) std::memcpy(wk->up_h.p + o_lits, h_lits, 4 * (size_t)L);
        std::memcpy(wk->up_h.p + o_map, var2dense.data(), 4 * (size_t)(maxvar + 1));
        SATMI_HIP(hipMemcpyAsync(wk->up.p, wk->up_h.p, up_bytes, hipMemcpyHostToDevice, s));
        if (!packed) {   // (the packed path encodes its keys in its prologue launch)
            const unsigned char *up = (const unsigned char *)wk->up.p;
            hipLaunchKernelGGL(encode_keys_kernel, dim3(grid_for(nclauses)), dim3(PRIM_BLOCK), 0, s, nclauses,
                               (const int32_t *)up, (const int32_t *)(up + o_lits), (const int32_t *)(up + o_map), W,
                               clauses.as<uint64_t>());
            SATMI_HIP(hipGetLastError());
        }
    }
    if (packed) {
        const int rc = resolution_packed(*wk, nclauses, (const unsigned char *)wk->up.p, o_lits, o_map, max_passes,
                                         clause_limit, time_limit_s, slot_base, V,
                                         dense2var, h_result, h_passes, h_pass_new, pass_cap, h_rec_lits,
                                         rec_lit_cap, h_rec_clause_off, rec_clause_cap, h_rec_pass_off, rec_pass_cap);
        if (rc == SATMI_OK) lease.ok = true;
        return rc;
    }
    DevBuf &table = wk->table, &flag = wk->flag, &pos = wk->pos, &slotv = wk->slotv, &tiles = wk->tiles,
           &grand = wk->grand;
    // the general path fills the shared table with clause indices: a later
    // packed call on this workspace must empty it first (its prologue only
    // skips the reset when the previous packed call's reset left it clean)
    wk->clean = ResWork::Clean{};
    EventTimer &t_pairs = wk->t_pairs, &t_claims = wk->t_claims;
    t_pairs.reset();
    t_claims.reset();
    g_stats = ResStats{};
    uint64_t tcap = 0;
    unsigned long long *d_count = counters.as<unsigned long long>();
    int *d_empty = (int *)(counters.as<char>() + 8);
    // a fresh table holding clauses [0, nkeys) with room for `room` keys
    const auto rebuild_table = [&](int64_t nkeys, int64_t room) {
        tcap = table_slots(room);
        SATMI_TRY(table.reserve(8 * tcap));
        SATMI_HIP(hipMemsetAsync(table.p, 0xFF, 8 * tcap, s));   // HT_EMPTY
        if (nkeys > 0 && packed)
            hipLaunchKernelGGL(ht_clauses_packed_kernel, dim3(grid_for(nkeys)), dim3(PRIM_BLOCK), 0, s,
                               table.as<uint64_t>(), tcap - 1, clauses.as<uint64_t>(), (int64_t)0, nkeys);
        else if (nkeys > 0)
            hipLaunchKernelGGL(ht_clauses_kernel, dim3(grid_for(nkeys)), dim3(PRIM_BLOCK), 0, s, table.as<uint64_t>(),
                               tcap - 1, KeySrc{clauses.as<uint64_t>(), nullptr, 0, K}, (int64_t)0, nkeys);
        SATMI_HIP(hipGetLastError());
        return SATMI_OK;
    };
    const auto launch_pairs = [&](int64_t j0, int64_t j1, int64_t cap) {
        const int grid = (int)std::min<int64_t>(j1 - j0, 65536);
        switch (W) {
            case 1:
                hipLaunchKernelGGL(res_pairs_kernel<1>, dim3(grid), dim3(256), 0, s, clauses.as<uint64_t>(), W, j0, j1,
                                   d_count, d_empty, cand.as<uint64_t>(), cap, slot_base);
                break;
            case 2:
                hipLaunchKernelGGL(res_pairs_kernel<2>, dim3(grid), dim3(256), 0, s, clauses.as<uint64_t>(), W, j0, j1,
                                   d_count, d_empty, cand.as<uint64_t>(), cap, slot_base);
                break;
            case 3:
                hipLaunchKernelGGL(res_pairs_kernel<3>, dim3(grid), dim3(256), 0, s, clauses.as<uint64_t>(), W, j0, j1,
                                   d_count, d_empty, cand.as<uint64_t>(), cap, slot_base);
                break;
            case 4:
                hipLaunchKernelGGL(res_pairs_kernel<4>, dim3(grid), dim3(256), 0, s, clauses.as<uint64_t>(), W, j0, j1,
                                   d_count, d_empty, cand.as<uint64_t>(), cap, slot_base);
                break;
            default:
                hipLaunchKernelGGL(res_pairs_kernel<0>, dim3(grid), dim3(256), 0, s, clauses.as<uint64_t>(), W, j0, j1,
                                   d_count, d_empty, cand.as<uint64_t>(), cap, slot_base);
        }
    };
    const auto grow_clauses = [&](int64_t want) {
        if ((size_t)want * K * 8 <= clauses.cap) return SATMI_OK;
        DevBuf grown;
        SATMI_TRY(grown.reserve(8 * (size_t)want * K * 2));
        SATMI_HIP(hipMemcpyAsync(grown.p, clauses.p, clauses.cap, hipMemcpyDeviceToDevice, s));
        std::swap(grown.p, clauses.p);
        std::swap(grown.cap, clauses.cap);
        SATMI_HIP(hipStreamSynchronize(s));   // before `grown` frees the old array
        return SATMI_OK;
    };

    int64_t jlo = 0, rec_clauses = 0, rec_lits = 0;
    int passes = 0;
    bool stopped = false;   // a limit (deadline) ended a pass early
    std::vector<uint64_t> hkeys;
    while (!stopped) {
        if (max_passes > 0 && passes >= max_passes) break;
        if (expired()) break;
        // one pass: chunks of pairs (i < j, j in [jlo, ncl)) -> candidates ->
        // claims in the pass's table -> the winners appended after clause ncl
        int64_t nnew = 0;
        SATMI_TRY(rebuild_table(ncl, 2 * ncl + 65536));
        bool empty = false;
        for (int64_t j0 = jlo; j0 < ncl && !empty;) {
            if (j0 > jlo && expired()) {
                stopped = true;
                break;
            }
            // j1: about PAIR_CHUNK pairs past j0 (tri(j1) - tri(j0)), at least one j
            const double t1 = 0.5 * (double)j0 * (double)(j0 - 1) + (double)PAIR_CHUNK;
            int64_t j1 = (int64_t)(0.5 + std::sqrt(0.25 + 2.0 * t1));
            j1 = std::min(ncl, std::max(j1, j0 + 1));
            while (j1 > j0 + 1 && (j1 * (j1 - 1) - j0 * (j0 - 1)) / 2 > PAIR_CHUNK) --j1;
            const int64_t npairs = std::max<int64_t>(1, (j1 * (j1 - 1) - j0 * (j0 - 1)) / 2);
            SATMI_TRY(cand.reserve(std::min(8 * (size_t)npairs * K, std::max(g_cand_bytes, cand.cap))));
            struct {
                unsigned long long count;
                int empty;
                int pad;
            } hc{(unsigned long long)slot_base, 0, 0};
            for (int attempt = 0;; ++attempt) {
                const int64_t cap = (int64_t)(cand.cap / (8 * (size_t)K));
                hc = {(unsigned long long)slot_base, 0, 0};
                std::memcpy(wk->pin, &hc, 16);   // staged in pinned memory: a truly asynchronous copy
                SATMI_HIP(hipMemcpyAsync(counters.p, wk->pin, 16, hipMemcpyHostToDevice, s));
                t_pairs.begin(s);
                launch_pairs(j0, j1, cap);
                t_pairs.end(s);
                SATMI_HIP(hipGetLastError());
                SATMI_HIP(hipMemcpyAsync(wk->pin, counters.p, 16, hipMemcpyDeviceToHost, s));
                SATMI_HIP(hipStreamSynchronize(s));
                std::memcpy(&hc, wk->pin, 16);
                const int64_t counted = (int64_t)(hc.count - (unsigned long long)slot_base);
                if (hc.empty || counted <= cap) break;
                if (attempt > 0) {   // cannot happen: the re-run had room for every counted candidate
                    set_error("satmi_resolution_host: candidate buffer overflow after a re-run");
                    return SATMI_ERR_HIP;
                }
                SATMI_TRY(cand.reserve(8 * (size_t)counted * K));   // overflowed: re-run at the counted size
            }
            g_stats.pairs += npairs;
            j0 = j1;
            if (hc.empty) {   // an empty resolvent: unsatisfiable (REF.py:84-85)
                empty = true;
                break;
            }
            const int64_t nc = (int64_t)(hc.count - (unsigned long long)slot_base);
            if (nc <= 0) continue;
            if ((uint64_t)(ncl + nnew + nc) > tcap / 2) SATMI_TRY(rebuild_table(ncl + nnew, 2 * (ncl + nnew + nc)));
            SATMI_TRY(flag.reserve(8 * (size_t)nc));
            SATMI_TRY(pos.reserve(8 * (size_t)nc));
            SATMI_TRY(slotv.reserve(8 * (size_t)nc));
            SATMI_TRY(tiles.reserve(8 * (size_t)((nc + SCAN_TILE - 1) / SCAN_TILE + 1)));
            SATMI_TRY(grand.reserve(8));
            t_claims.begin(s);
            if (packed)
                hipLaunchKernelGGL(ht_cand_packed_kernel, dim3(grid_for(nc)), dim3(PRIM_BLOCK), 0, s,
                                   table.as<uint64_t>(), tcap - 1, cand.as<uint64_t>(), nc, flag.as<int64_t>());
            else
                hipLaunchKernelGGL(ht_cand_kernel, dim3(grid_for(nc)), dim3(PRIM_BLOCK), 0, s, table.as<uint64_t>(),
                                   tcap - 1, KeySrc{clauses.as<uint64_t>(), cand.as<uint64_t>(), slot_base, K}, nc,
                                   flag.as<int64_t>(), slotv.as<int64_t>());
            t_claims.end(s);
            g_stats.candidates += nc;
            SATMI_HIP(hipGetLastError());
            SATMI_TRY(exclusive_scan(flag.as<int64_t>(), pos.as<int64_t>(), nc, tiles.as<int64_t>(),
                                     grand.as<int64_t>(), s));
            int64_t nwin = 0;
            SATMI_HIP(hipMemcpyAsync(wk->pin + 2, grand.p, 8, hipMemcpyDeviceToHost, s));
            SATMI_HIP(hipStreamSynchronize(s));
            nwin = (int64_t)wk->pin[2];
            if (nwin == 0) continue;
            SATMI_TRY(grow_clauses(ncl + nnew + nwin));
            hipLaunchKernelGGL(res_append_kernel, dim3(grid_for(nc)), dim3(PRIM_BLOCK), 0, s, cand.as<uint64_t>(),
                               flag.as<int64_t>(), pos.as<int64_t>(), slotv.as<int64_t>(), nc, K,
                               clauses.as<uint64_t>(), ncl + nnew, packed ? nullptr : table.as<uint64_t>());
            SATMI_HIP(hipGetLastError());
            nnew += nwin;
        }
        if (empty) {
            *h_result = 0;
            break;
        }
        if (stopped) break;
        if (nnew == 0) {   // no new clauses can be derived (REF.py:91-92)
            *h_result = 1;
            break;
        }
        if (h_pass_new && passes < pass_cap) h_pass_new[passes] = nnew;
        if (h_rec_lits && h_rec_clause_off && h_rec_pass_off && passes + 1 < rec_pass_cap) {
            hkeys.resize((size_t)nnew * K);
            SATMI_HIP(hipMemcpyAsync(hkeys.data(), clauses.as<uint64_t>() + ncl * K, 8 * (size_t)nnew * K,
                                     hipMemcpyDeviceToHost, s));
            SATMI_HIP(hipStreamSynchronize(s));
            record_pass(hkeys, nnew, false, W, V, dense2var, passes, h_rec_lits, rec_lit_cap, h_rec_clause_off,
                        rec_clause_cap, h_rec_pass_off, rec_clauses, rec_lits);
        }
        ++passes;
        jlo = ncl;
        ncl += nnew;
        if (clause_limit > 0 && ncl > clause_limit) break;
    }
    SATMI_HIP(hipStreamSynchronize(s));
    *h_passes = passes;
    g_stats.pair_ms = t_pairs.total();
    g_stats.claim_ms = t_claims.total();
    lease.ok = true;
    return SATMI_OK;
}

// Free every idle workspace of this solver (device buffers, streams, pinned
// words); calls in flight keep theirs.  The next call allocates afresh.
extern "C" int satmi_resolution_trim(void) {
    std::vector<ResWork *> idle;
    {
        auto &P = res_pool();
        std::lock_guard<std::mutex> g(P.mu);
        idle.swap(P.free_list);
    }
    for (ResWork *w : idle) {
        (void)hipStreamSynchronize(w->stream);
        delete w;
    }
    return SATMI_OK;
}
