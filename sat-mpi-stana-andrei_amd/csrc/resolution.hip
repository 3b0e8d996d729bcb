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
//   * pair kernel (one thread per pair, grid-stride): clash = (Pi & Nj) | (Ni & Pj).
//     Two or more clashing variables make every resolvent a tautology (the
//     other clash survives in both signs); with exactly one, the resolvent is
//     (Pi|Pj, Ni|Nj) minus that variable, a tautology iff its two halves meet,
//     empty iff both are zero.  Candidates are appended with one atomic per
//     wavefront (ballot + popcount);
//   * hash dedup: one open-addressing table per pass over every clause key
//     (the reference's `seen`), then every candidate claims its key's slot
//     run with a 64-bit CAS; the claimers are the pass's new clauses,
//     compacted (flag scan) and appended to the clause array;
//   * a pass's pairs run in launches of PAIR_CHUNK, the deadline checked
//     between them, so a long pass ends as a timeout (REF.py:417-437);
//   * semi-naive passes: pairs whose newer clause was added in the previous pass
//     (all pairs in pass 1) -- every older pair was resolved in an earlier pass
//     and its resolvents are already in `seen`, so the new set is identical.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
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

// Pairs (i < j) with j in [jlo, N).  WRITE=false: count candidates; WRITE=true:
// append them to cand (slots from *count, which must start at 0).
// Pairs are numbered q = tri(j) + i over the whole pass; this launch takes
// q in [tri(jlo) + p_begin, tri(jlo) + p_begin + npairs) (a chunk of the pass).
// WRITE: candidate slot k (from *count, which starts at `slot_base`) goes to
// cand[k - slot_base].
template <bool WRITE>
__global__ void __launch_bounds__(256) res_pairs_kernel(const uint64_t *keys, int W, int64_t jlo, int64_t p_begin,
                                                        int64_t npairs, unsigned long long *count, int *empty_found,
                                                        uint64_t *cand, int64_t cand_cap, int64_t slot_base) {
    const int K = 2 * W;
    const int ln = lane_id();
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t base = tri(jlo) + p_begin;
    for (int64_t p0 = (int64_t)blockIdx.x * blockDim.x; p0 < npairs; p0 += stride) {
        const int64_t p = p0 + threadIdx.x;
        bool is_cand = false;
        int cw = 0;
        uint64_t cbit = 0;
        int64_t i = 0, j = 0;
        if (p < npairs) {
            const int64_t q = p + base;
            j = (int64_t)((1.0 + sqrt(1.0 + 8.0 * (double)q)) * 0.5);
            while (tri(j) > q) --j;
            while (tri(j + 1) <= q) ++j;
            i = q - tri(j);
            const uint64_t *a = keys + i * K, *b = keys + j * K;
            int nclash = 0;
            for (int w = 0; w < W; ++w) {
                const uint64_t c = (a[w] & b[W + w]) | (a[W + w] & b[w]);
                if (c) {
                    nclash += __popcll(c);
                    cw = w;
                    cbit = c & (~c + 1ull);
                }
            }
            if (nclash == 1) {
                bool taut = false, empty = true;
                for (int w = 0; w < W; ++w) {
                    uint64_t rp = a[w] | b[w], rn = a[W + w] | b[W + w];
                    if (w == cw) {
                        rp &= ~cbit;
                        rn &= ~cbit;
                    }
                    taut |= (rp & rn) != 0ull;
                    empty &= (rp | rn) == 0ull;
                }
                if (!taut) {
                    if (empty) *empty_found = 1;   // REF.py:84-85
                    else is_cand = true;
                }
            }
        }
        const uint64_t m = __ballot(is_cand);
        if (m == 0ull) continue;
        unsigned long long slot0 = 0;
        if (ln == 0) slot0 = atomicAdd(count, (unsigned long long)__popcll(m));
        // zero-extend each 32-bit half (a sign-extended low half past 2^31
        // candidates would turn the slot negative and the write out of bounds)
        slot0 = (unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)slot0) |
                ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(slot0 >> 32)) << 32);
        if (WRITE && is_cand) {
            const int64_t slot = (int64_t)slot0 + __popcll(m & lanemask_lt()) - slot_base;
            if (slot >= 0 && slot < cand_cap) {
                const uint64_t *a = keys + i * K, *b = keys + j * K;
                uint64_t *r = cand + slot * K;
                for (int w = 0; w < W; ++w) {
                    uint64_t rp = a[w] | b[w], rn = a[W + w] | b[W + w];
                    if (w == cw) {
                        rp &= ~cbit;
                        rn &= ~cbit;
                    }
                    r[w] = rp;
                    r[W + w] = rn;
                }
            }
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

// Claim a slot for value v (key x).  Returns true with *slot if x was absent.
__device__ bool ht_insert(uint64_t *table, uint64_t mask, const KeySrc &S, uint64_t v, const uint64_t *x) {
    uint64_t s = key_hash(x, S.K) & mask;
    for (;;) {
        uint64_t cur = __hip_atomic_load(table + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == HT_EMPTY) {
            cur = atomicCAS((unsigned long long *)(table + s), (unsigned long long)HT_EMPTY, (unsigned long long)v);
            if (cur == HT_EMPTY) return true;
        }
        if (key_eq(S.at(cur), x, S.K)) return false;
        s = (s + 1) & mask;
    }
}

__global__ void ht_clauses_kernel(uint64_t *table, uint64_t mask, KeySrc S, int64_t ncl) {
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < ncl; c += (int64_t)gridDim.x * blockDim.x)
        (void)ht_insert(table, mask, S, (uint64_t)c, S.clauses + c * S.K);
}

// flag[t] = candidate t claimed its key (new in this pass)
__global__ void ht_cand_kernel(uint64_t *table, uint64_t mask, KeySrc S, int64_t n, int64_t *flag) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x)
        flag[t] = ht_insert(table, mask, S, CAND_BIT | (uint64_t)(S.base + t), S.cand + t * S.K) ? 1 : 0;
}

// clauses.extend(new): the claimed candidates, in append order, after clause ncl
__global__ void res_append_kernel(const uint64_t *cand, const int64_t *flag, const int64_t *pos, int64_t n, int K,
                                  uint64_t *dst) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
        if (!flag[t]) continue;
        for (int w = 0; w < K; ++w) dst[pos[t] * K + w] = cand[t * K + w];
    }
}

// ------------------------------------------------------------------ host side
namespace {

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    int reserve(size_t bytes) {
        if (bytes <= cap) return SATMI_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max(bytes, (size_t)256);
        SATMI_HIP(hipMalloc(&p, want));
        cap = want;
        return SATMI_OK;
    }
    template <class T>
    T *as() const { return (T *)p; }
};

#define SATMI_TRY(x)                  \
    do {                              \
        int _rc = (x);                \
        if (_rc != SATMI_OK) return _rc; \
    } while (0)

// One pass's dedup (see ht_insert): a fresh table over every clause key, then
// the candidates' claims; flag / pos (exclusive scan) give the new keys in
// append order, *nnew their count.
struct HashDedup {
    DevBuf table, flag, pos, tiles, grand;
    static uint64_t table_slots(int64_t keys) {
        uint64_t cap = 64;
        while (cap < 2 * (uint64_t)keys) cap <<= 1;
        return cap;
    }
    int run(const uint64_t *clauses, int64_t ncl, const uint64_t *cand, int64_t n, int64_t slot_base, int K,
            int64_t *nnew, hipStream_t s) {
        *nnew = 0;
        if (n == 0) return SATMI_OK;
        const uint64_t cap = table_slots(ncl + n);
        SATMI_TRY(table.reserve(8 * cap));
        SATMI_TRY(flag.reserve(8 * (size_t)n));
        SATMI_TRY(pos.reserve(8 * (size_t)n));
        SATMI_TRY(tiles.reserve(8 * (size_t)((n + SCAN_TILE - 1) / SCAN_TILE + 1)));
        SATMI_TRY(grand.reserve(8));
        SATMI_HIP(hipMemsetAsync(table.p, 0xFF, 8 * cap, s));   // HT_EMPTY
        const KeySrc S{clauses, cand, slot_base, K};
        if (ncl > 0)
            hipLaunchKernelGGL(ht_clauses_kernel, dim3(grid_for(ncl)), dim3(PRIM_BLOCK), 0, s, table.as<uint64_t>(),
                               cap - 1, S, ncl);
        hipLaunchKernelGGL(ht_cand_kernel, dim3(grid_for(n)), dim3(PRIM_BLOCK), 0, s, table.as<uint64_t>(), cap - 1,
                           S, n, flag.as<int64_t>());
        SATMI_HIP(hipGetLastError());
        SATMI_TRY(exclusive_scan(flag.as<int64_t>(), pos.as<int64_t>(), n, tiles.as<int64_t>(),
                                 grand.as<int64_t>(), s));
        SATMI_HIP(hipMemcpyAsync(nnew, grand.p, 8, hipMemcpyDeviceToHost, s));
        SATMI_HIP(hipStreamSynchronize(s));
        return SATMI_OK;
    }
};

// pairs per launch: a pass is cut into launches of this many pairs so that the
// deadline is checked inside a long pass (REF.py:417-437's timeout)
constexpr int64_t PAIR_CHUNK = 1ll << 30;

int64_t g_slot_base = 0;   // test knob: first append slot of the pair kernel

}  // namespace

}  // namespace satmi

using namespace satmi;

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
        if (h_lits[i] == 0) {
            set_error("satmi_resolution_host: literal 0");
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
    const int64_t slot_base = g_slot_base;
    hipStream_t s = nullptr;

    DevBuf d_off, d_lits, d_map, clauses, cand, counters;
    SATMI_TRY(d_off.reserve(4 * (size_t)(nclauses + 1)));
    SATMI_TRY(d_lits.reserve(4 * (size_t)std::max<int64_t>(L, 1)));
    SATMI_TRY(d_map.reserve(4 * (size_t)(maxvar + 1)));
    int64_t ncl = nclauses;
    SATMI_TRY(clauses.reserve(8 * (size_t)std::max<int64_t>(ncl, 1) * K));
    SATMI_TRY(counters.reserve(64));
    if (nclauses > 0) {
        SATMI_HIP(hipMemcpyAsync(d_off.p, h_clause_off, 4 * (size_t)(nclauses + 1), hipMemcpyHostToDevice, s));
        if (L) SATMI_HIP(hipMemcpyAsync(d_lits.p, h_lits, 4 * (size_t)L, hipMemcpyHostToDevice, s));
        SATMI_HIP(hipMemcpyAsync(d_map.p, var2dense.data(), 4 * (size_t)(maxvar + 1), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(encode_keys_kernel, dim3(grid_for(nclauses)), dim3(PRIM_BLOCK), 0, s, nclauses,
                           d_off.as<int32_t>(), d_lits.as<int32_t>(), d_map.as<int32_t>(), W,
                           clauses.as<uint64_t>());
        SATMI_HIP(hipGetLastError());
    }
    HashDedup dd;
    unsigned long long *d_count = counters.as<unsigned long long>();
    int *d_empty = (int *)(counters.as<char>() + 8);
    // one sweep of the pass's pairs (count or write), a launch per PAIR_CHUNK;
    // false if the deadline passed between two launches
    const auto sweep = [&](bool write, int64_t npairs, int64_t jlo, int64_t ncand, int *rc) {
        *rc = SATMI_OK;
        for (int64_t p = 0; p < npairs; p += PAIR_CHUNK) {
            if (p > 0) {
                if (hipStreamSynchronize(s) != hipSuccess) {
                    *rc = hip_fail(hipGetLastError(), "resolution pair sweep");
                    return false;
                }
                if (expired()) return false;
            }
            const int64_t np = std::min(PAIR_CHUNK, npairs - p);
            if (write)
                hipLaunchKernelGGL(res_pairs_kernel<true>, dim3(grid_for(np)), dim3(256), 0, s,
                                   clauses.as<uint64_t>(), W, jlo, p, np, d_count, d_empty, cand.as<uint64_t>(),
                                   ncand, slot_base);
            else
                hipLaunchKernelGGL(res_pairs_kernel<false>, dim3(grid_for(np)), dim3(256), 0, s,
                                   clauses.as<uint64_t>(), W, jlo, p, np, d_count, d_empty, nullptr, (int64_t)0,
                                   (int64_t)0);
            if (hipGetLastError() != hipSuccess) {
                *rc = hip_fail(hipErrorLaunchFailure, "res_pairs_kernel");
                return false;
            }
        }
        return true;
    };

    int64_t jlo = 0, rec_clauses = 0, rec_lits = 0;
    int passes = 0;
    std::vector<uint64_t> hkeys;
    for (;;) {
        if (max_passes > 0 && passes >= max_passes) break;
        if (expired()) break;
        const int64_t npairs = (ncl * (ncl - 1) - jlo * (jlo - 1)) / 2;
        struct {
            unsigned long long count;
            int empty;
            int pad;
        } hc{0, 0, 0};
        int rc = SATMI_OK;
        SATMI_HIP(hipMemsetAsync(counters.p, 0, 16, s));
        if (!sweep(false, npairs, jlo, 0, &rc)) {
            if (rc) return rc;
            break;   // deadline inside the pass
        }
        SATMI_HIP(hipMemcpyAsync(&hc, counters.p, 16, hipMemcpyDeviceToHost, s));
        SATMI_HIP(hipStreamSynchronize(s));
        if (hc.empty) {   // an empty resolvent: unsatisfiable (REF.py:84-85)
            *h_result = 0;
            break;
        }
        const int64_t ncand = (int64_t)hc.count;
        int64_t nnew = 0;
        if (ncand > 0) {
            // the pass's working set: candidate keys, flag / pos, the hash table and
            // the grown clause array; refuse (SATMI_ERR_NOMEM) rather than oversubscribe HBM
            const double need = (double)ncand * (8.0 * K + 16.0) + 8.0 * (double)HashDedup::table_slots(ncl + ncand) +
                                8.0 * (double)(ncl + ncand) * K;
            size_t free_b = 0, total_b = 0;
            SATMI_HIP(hipMemGetInfo(&free_b, &total_b));
            if (need > 0.8 * (double)(free_b + cand.cap + dd.table.cap + dd.flag.cap + dd.pos.cap)) {
                set_error("satmi_resolution_host: pass " + std::to_string(passes + 1) + " has " +
                          std::to_string(ncand) + " candidate resolvents, needing " +
                          std::to_string(need / 1e9) + " GB of device memory (" + std::to_string(free_b / 1e9) +
                          " GB free); set clause_limit / max_passes");
                return SATMI_ERR_NOMEM;
            }
            SATMI_TRY(cand.reserve(8 * (size_t)ncand * K));
            const unsigned long long start = (unsigned long long)slot_base;
            SATMI_HIP(hipMemcpyAsync(d_count, &start, 8, hipMemcpyHostToDevice, s));
            if (!sweep(true, npairs, jlo, ncand, &rc)) {
                if (rc) return rc;
                break;
            }
            SATMI_TRY(dd.run(clauses.as<uint64_t>(), ncl, cand.as<uint64_t>(), ncand, slot_base, K, &nnew, s));
        }
        if (nnew == 0) {   // no new clauses can be derived (REF.py:91-92)
            *h_result = 1;
            break;
        }
        // clauses.extend(new) (REF.py:94-95): append the claimed candidates
        const int64_t ncl2 = ncl + nnew;
        if ((size_t)ncl2 * K * 8 > clauses.cap) {
            DevBuf grown;
            SATMI_TRY(grown.reserve(8 * (size_t)ncl2 * K * 2));
            SATMI_HIP(hipMemcpyAsync(grown.p, clauses.p, 8 * (size_t)ncl * K, hipMemcpyDeviceToDevice, s));
            std::swap(grown.p, clauses.p);
            std::swap(grown.cap, clauses.cap);
            SATMI_HIP(hipStreamSynchronize(s));   // before `grown` frees the old array
        }
        hipLaunchKernelGGL(res_append_kernel, dim3(grid_for(ncand)), dim3(PRIM_BLOCK), 0, s, cand.as<uint64_t>(),
                           dd.flag.as<int64_t>(), dd.pos.as<int64_t>(), ncand, K, clauses.as<uint64_t>() + ncl * K);
        SATMI_HIP(hipGetLastError());
        if (h_pass_new && passes < pass_cap) h_pass_new[passes] = nnew;
        if (h_rec_lits && h_rec_clause_off && h_rec_pass_off && passes + 1 < rec_pass_cap) {
            // the pass's new clause set, each clause as ascending literals, the
            // clauses in ascending order (deterministic whatever the append order)
            hkeys.resize((size_t)nnew * K);
            SATMI_HIP(hipMemcpyAsync(hkeys.data(), clauses.as<uint64_t>() + ncl * K, 8 * (size_t)nnew * K,
                                     hipMemcpyDeviceToHost, s));
            SATMI_HIP(hipStreamSynchronize(s));
            std::vector<std::vector<int32_t>> pass(nnew);
            for (int64_t c = 0; c < nnew; ++c) {
                const uint64_t *k = hkeys.data() + c * K;
                for (int d = 0; d < V; ++d) {
                    if ((k[d >> 6] >> (d & 63)) & 1ull) pass[c].push_back(dense2var[d]);
                    if ((k[W + (d >> 6)] >> (d & 63)) & 1ull) pass[c].push_back(-dense2var[d]);
                }
                std::sort(pass[c].begin(), pass[c].end());
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
        ++passes;
        jlo = ncl;
        ncl = ncl2;
        if (clause_limit > 0 && ncl > clause_limit) break;
    }
    SATMI_HIP(hipStreamSynchronize(s));
    *h_passes = passes;
    return SATMI_OK;
}
