// dp.hip -- Davis-Putnam variable elimination (REF.py:98-130) on gfx950.
//
// One elimination step of the reference: pick `var = variables.pop()`, split
// the clause list into clauses with var / with -var / without it, resolve
// every (pos, neg) pair in list order, drop tautologies, return False on an
// empty resolvent, keep a resolvent unless an earlier-listed clause of
// `remaining + unique_new` is a subset of it, continue with remaining + kept.
//
// GPU formulation, per step (host C++ drives the launches, data stays in HBM):
//   * every clause carries (a) a bitset key over the dense variable index for
//     the set algebra (split, tautology, emptiness, subsumption) and (b) its
//     CPython table image (pyset_dev.h), because the reference's elimination
//     order is decided by CPython's set layout;
//   * dp_firstpos: first-occurrence position of every variable in the order
//     `{abs(lit) for clause in clauses for lit in clause}` visits them (list
//     order, then each clause's table order); dp_pop: one workgroup ranks the
//     variables by that position and replays the comprehension's insertions
//     into a modelled set, then pops its first live slot;
//   * dp_split + scans: order-preserving compaction into pos / neg / rem lists;
//   * dp_diff: `pc - {var}` / `nc - {-var}` images, one thread per clause;
//   * dp_pairs: one thread per pair, resolvent bitset, tautology / empty flags;
//   * dp_subsume: greedy `unique_new` filter.  A new clause is dropped iff a
//     remaining clause or an *earlier* new clause is a subset of it (an earlier
//     new clause that was itself dropped was dropped for a subset that is also
//     a subset of this one), so the greedy loop becomes one parallel test;
//   * dp_build: `AX | BY` images of the kept resolvents; dp_assemble: the next
//     clause list (rem in order, then kept in pair order).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <mutex>
#include <vector>

#include "common.h"
#include "prims.h"
#include "pyset_dev.h"

namespace satmi {

// smallest power of two >= 8 that exceeds 8*u: room for every table a set of u
// keys passes through (add: < 8u, merge: < 4u)
static inline int64_t cap_for(int64_t u) {
    int64_t c = PY_MINSIZE;
    while (c <= 8 * u) c <<= 1;
    return c;
}

struct ClauseList {   // device arrays of one generation
    int64_t *off;      // table image offset in pool
    int32_t *mask, *fill, *used;
    uint64_t *bits;    // K words per clause
    int32_t *pool;
};

__device__ __forceinline__ DView cl_view(const ClauseList &L, int64_t c) {
    return {L.pool + L.off[c], (int64_t)L.mask[c], (int64_t)L.fill[c], (int64_t)L.used[c]};
}

// clauses = [set(clause) for clause in formula]  (REF.py:99); image c at pool + 2*cap*c
__global__ void dp_encode_kernel(int nclauses, const int32_t *off, const int32_t *lits, const int32_t *var2dense,
                                 int W, int64_t cap, ClauseList L, int *overflow) {
    const int K = 2 * W;
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < nclauses; c += gridDim.x * blockDim.x) {
        int32_t *a = L.pool + (int64_t)c * 2 * cap;
        DSet s;
        dset_init(s, a, a + cap, cap);
        uint64_t *k = L.bits + (int64_t)c * K;
        for (int w = 0; w < K; ++w) k[w] = 0ull;
        for (int j = off[c]; j < off[c + 1]; ++j) {
            const int x = lits[j];
            py_add(s, x);
            const int d = var2dense[x < 0 ? -x : x];
            k[(x < 0 ? W : 0) + (d >> 6)] |= 1ull << (d & 63);
        }
        if (s.overflow) *overflow = 1;
        L.off[c] = s.t - L.pool;
        L.mask[c] = (int32_t)s.mask;
        L.fill[c] = (int32_t)s.fill;
        L.used[c] = (int32_t)s.used;
    }
}

__global__ void dp_used_kernel(ClauseList L, int64_t n, int64_t *used) {
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n; c += (int64_t)gridDim.x * blockDim.x)
        used[c] = L.used[c];
}

// first position of every variable in the comprehension's visiting order
__global__ void dp_firstpos_kernel(ClauseList L, int64_t n, const int64_t *base, const int32_t *var2dense,
                                   unsigned long long *firstpos) {
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n; c += (int64_t)gridDim.x * blockDim.x) {
        const DView s = cl_view(L, c);
        int64_t p = base[c];
        for (int64_t i = 0; i <= s.mask; ++i) {
            const int32_t k = s.t[i];
            if (k == PY_EMPTY || k == PY_DUMMY) continue;
            atomicMin(&firstpos[var2dense[k < 0 ? -k : k]], (unsigned long long)p);
            ++p;
        }
    }
}

// variables.pop() (REF.py:100-103, :128): one workgroup.  out[0] = popped
// variable (0: the set is empty), out[1] = number of distinct variables.
__global__ void __launch_bounds__(256) dp_pop_kernel(const unsigned long long *firstpos, const int32_t *dense2var,
                                                     int V, int32_t *order, int32_t *scratch, int64_t cap,
                                                     int32_t *out) {
    __shared__ int nlive;
    if (threadIdx.x == 0) nlive = 0;
    __syncthreads();
    for (int d = threadIdx.x; d < V; d += blockDim.x) {
        const unsigned long long f = firstpos[d];
        if (f == ~0ull) continue;
        int rank = 0;
        for (int e = 0; e < V; ++e) rank += firstpos[e] < f ? 1 : 0;   // positions are distinct
        order[rank] = dense2var[d];
        atomicAdd(&nlive, 1);
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    const int nv = nlive;
    int32_t popped = 0;
    if (nv > 0) {
        DSet s;
        dset_init(s, scratch, scratch + cap, cap);
        for (int r = 0; r < nv; ++r) py_add(s, order[r]);
        if (s.overflow) {
            out[2] = 1;
        } else {
            for (int64_t i = 0; i <= s.mask; ++i)   // a fresh set's finger is 0: first live slot
                if (s.t[i] != PY_EMPTY && s.t[i] != PY_DUMMY) {
                    popped = s.t[i];
                    break;
                }
        }
    }
    out[0] = popped;
    out[1] = nv;
}

// split flags (REF.py:106-108)
// Also the largest image (`used`) among the clauses holding var / -var into
// mx[0] / mx[1] (zeroed by the host): the capacities of the step's images,
// read back with the split counts instead of after the filter.
__global__ void dp_split_kernel(ClauseList L, int64_t n, int W, int d, int64_t *fpos, int64_t *fneg, int64_t *frem,
                                unsigned long long *mx) {
    const int K = 2 * W;
    int up = 0, un = 0;
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n; c += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t *k = L.bits + c * K;
        const bool p = (k[d >> 6] >> (d & 63)) & 1ull;
        const bool q = (k[W + (d >> 6)] >> (d & 63)) & 1ull;
        fpos[c] = p;
        fneg[c] = q;
        frem[c] = !p && !q;
        const int u = (p || q) ? L.used[c] : 0;
        up = p ? max(up, u) : up;
        un = q ? max(un, u) : un;
    }
    up = wave_max_i32(up);   // every lane reaches here (grid-stride loop)
    un = wave_max_i32(un);
    if (lane_id() == 0) {
        if (up) atomicMax(mx, (unsigned long long)up);
        if (un) atomicMax(mx + 1, (unsigned long long)un);
    }
}

__global__ void dp_compact_kernel(const int64_t *flag, const int64_t *pos, int64_t n, int64_t *out) {
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n; c += (int64_t)gridDim.x * blockDim.x)
        if (flag[c]) out[pos[c]] = c;
}

struct Images {   // per-entry images built into 2*cap slots each
    int32_t *pool;
    int64_t *off;
    int32_t *mask, *fill, *used;
    int64_t cap;
};

__device__ __forceinline__ DView img_view(const Images &I, int64_t e) {
    return {I.pool + I.off[e], (int64_t)I.mask[e], (int64_t)I.fill[e], (int64_t)I.used[e]};
}

// AX = pc - {var} for the pos list, BY = nc - {-var} for the neg list
__global__ void dp_diff_kernel(ClauseList L, const int64_t *list, int64_t n, int32_t key, Images I, int *overflow) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
        int32_t *a = I.pool + e * 2 * I.cap;
        DSet s;
        dset_init(s, a, a + I.cap, I.cap);
        py_difference1(s, cl_view(L, list[e]), key);
        if (s.overflow) *overflow = 1;
        I.off[e] = s.t - I.pool;
        I.mask[e] = (int32_t)s.mask;
        I.fill[e] = (int32_t)s.fill;
        I.used[e] = (int32_t)s.used;
    }
}

// pair p = i*nn + j: resolvent bitset, tautology (REF.py:115) and empty (REF.py:117) flags
__global__ void dp_pairs_kernel(ClauseList L, const int64_t *plist, const int64_t *nlist, int64_t nn, int64_t npairs,
                                int W, int d, uint64_t *rbits, int64_t *nontaut, unsigned long long *first_empty) {
    const int K = 2 * W;
    const uint64_t vb = 1ull << (d & 63);
    const int vw = d >> 6;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < npairs;
         p += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t *a = L.bits + plist[p / nn] * K, *b = L.bits + nlist[p % nn] * K;
        uint64_t *r = rbits + p * K;
        bool taut = false, empty = true;
        for (int w = 0; w < W; ++w) {
            // (pc - {var}) | (nc - {-var}): var leaves pc's positive half and
            // -var nc's negative half only (a tautological pc keeps its -var)
            const uint64_t keep = w == vw ? ~vb : ~0ull;
            const uint64_t rp = (a[w] & keep) | b[w], rn = a[W + w] | (b[W + w] & keep);
            r[w] = rp;
            r[W + w] = rn;
            taut |= (rp & rn) != 0ull;
            empty &= (rp | rn) == 0ull;
        }
        nontaut[p] = !taut;
        if (empty) atomicMin(first_empty, (unsigned long long)p);
    }
}

__device__ __forceinline__ bool bits_subset(const uint64_t *a, const uint64_t *b, int K) {
    for (int w = 0; w < K; ++w)
        if (a[w] & ~b[w]) return false;
    return true;
}

// unique_new (REF.py:122-125): kept[k] iff no rem clause and no earlier new
// clause is a subset.  One wavefront per new clause: its 64 lanes test 64
// candidate subsets per step and the wave stops at the first hit (ballot), so
// the O(m (nrem + m)) tests spread over every wave slot of the chip instead of
// one serial loop per thread.
__global__ void __launch_bounds__(256) dp_subsume_kernel(ClauseList L, const int64_t *rlist, int64_t nrem,
                                                         const uint64_t *rbits, const int64_t *ntlist, int64_t m,
                                                         int K, int64_t *kept) {
    const int ln = lane_id();
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t k = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; k < m; k += nwaves) {
        const uint64_t *x = rbits + ntlist[k] * K;
        bool sub = false;
        for (int64_t e0 = 0; e0 < nrem && !sub; e0 += 64) {
            const int64_t e = e0 + ln;
            sub = __ballot(e < nrem && bits_subset(L.bits + rlist[e] * K, x, K)) != 0ull;
        }
        for (int64_t e0 = 0; e0 < k && !sub; e0 += 64) {
            const int64_t e = e0 + ln;
            sub = __ballot(e < k && bits_subset(rbits + ntlist[e] * K, x, K)) != 0ull;
        }
        if (ln == 0) kept[k] = !sub;
    }
}

// The same filter for K <= 8 words per clause (<= 256 variables), one LANE per
// new clause with its key in registers.  Candidates are numbered c = 0 ..
// nrem + m: remaining clauses first, then new clauses (new clause e is a
// candidate of k only when e < k).  Block (x, y) tests the new clauses
// sel[256x .. 256x + 256) (sel == nullptr: k = 256x + lane) against candidates
// [c_lo + y*SUB_CHUNK, +SUB_CHUNK) below c_hi, staging 256 candidate keys at a
// time in LDS: every lane reads the same LDS address (a broadcast, no bank
// conflicts), so one key load serves 256 tests and a candidate is read once per
// block.  A hit clears kept[k] (all ones before the first pass); a lane also
// stops once another block cleared its clause, the block once all lanes stopped.
// The host runs it twice: a short prefix of the candidates for every new clause
// (most are subsumed early), then the rest for the survivors only, so the
// long scans run on full waves.  tests_out: subset tests performed.
constexpr int SUB_TILE = 256, SUB_CHUNK = 4096, SUB_PREFIX = 1024;
template <int K>
__global__ void __launch_bounds__(SUB_TILE) dp_subsume_tiled_kernel(ClauseList L, const int64_t *rlist, int64_t nrem,
                                                                    const uint64_t *rbits, const int64_t *ntlist,
                                                                    const int64_t *sel, int64_t nsel, int64_t c_lo,
                                                                    int64_t c_hi, int64_t *kept,
                                                                    unsigned long long *tests_out) {
    __shared__ uint64_t tile[SUB_TILE][K];
    __shared__ unsigned long long tsum;
    __shared__ int64_t kmax_s;
    const int tid = threadIdx.x;
    const int64_t s = (int64_t)blockIdx.x * SUB_TILE + tid;
    const bool valid = s < nsel;
    const int64_t k = valid ? (sel ? sel[s] : s) : 0;
    if (tid == 0) {
        tsum = 0;
        kmax_s = 0;
    }
    __syncthreads();
    if (valid) atomicMax((unsigned long long *)&kmax_s, (unsigned long long)k);
    __syncthreads();
    const int64_t c_beg = c_lo + (int64_t)blockIdx.y * SUB_CHUNK;
    const int64_t c_end = min(min(c_beg + SUB_CHUNK, c_hi), nrem + kmax_s);   // no candidate beyond the last clause's
    if (c_beg >= c_end) return;                                               // (block-uniform)
    uint64_t x[K];
#pragma unroll
    for (int w = 0; w < K; ++w) x[w] = valid ? rbits[ntlist[k] * K + w] : 0ull;
    const int64_t mine = valid ? nrem + k : 0;   // candidates of clause k: c < nrem + k
    bool alive = valid && c_beg < mine;
    uint64_t tests = 0;
    for (int64_t e0 = c_beg; e0 < c_end; e0 += SUB_TILE) {
        if (alive && __hip_atomic_load(&kept[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) alive = false;
        if (!__syncthreads_or(alive)) break;
        const int64_t e = e0 + tid;
        if (e < c_end) {
            const uint64_t *src = e < nrem ? L.bits + rlist[e] * K : rbits + ntlist[e - nrem] * K;
#pragma unroll
            for (int w = 0; w < K; ++w) tile[tid][w] = src[w];
        }
        __syncthreads();
        if (alive) {
            const int cnt = (int)(min(min(e0 + SUB_TILE, c_end), mine) - e0);
            for (int j = 0; j < cnt; ++j) {
                uint64_t out = 0;
#pragma unroll
                for (int w = 0; w < K; ++w) out |= tile[j][w] & ~x[w];
                ++tests;
                if (out == 0ull) {
                    alive = false;
                    __hip_atomic_store(&kept[k], (int64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
            if (alive && e0 + SUB_TILE >= mine) alive = false;   // this lane's candidates are done
        }
        __syncthreads();
    }
    // one atomic per block
    atomicAdd(&tsum, (unsigned long long)tests);
    __syncthreads();
    if (tid == 0) atomicAdd(tests_out, tsum);
}

__global__ void dp_ones_kernel(int64_t *a, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        a[i] = 1;
}

// kept resolvent images: (pc - {var}) | (nc - {-var})  (REF.py:114)
__global__ void dp_build_kernel(Images A, Images B, const int64_t *ntlist, const int64_t *kflag, const int64_t *kpos,
                                int64_t m, int64_t nn, Images R, int *overflow) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        if (!kflag[k]) continue;
        const int64_t p = ntlist[k], e = kpos[k];
        int32_t *a = R.pool + e * 2 * R.cap;
        DSet s;
        dset_init(s, a, a + R.cap, R.cap);
        py_merge(s, img_view(A, p / nn));   // set_copy(AX)
        py_merge(s, img_view(B, p % nn));   // |= BY
        if (s.overflow) *overflow = 1;
        R.off[e] = s.t - R.pool;
        R.mask[e] = (int32_t)s.mask;
        R.fill[e] = (int32_t)s.fill;
        R.used[e] = (int32_t)s.used;
    }
}

__global__ void dp_sizes_kernel(ClauseList L, const int64_t *rlist, int64_t nrem, Images R, int64_t nkept,
                                int64_t *size) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nrem + nkept;
         t += (int64_t)gridDim.x * blockDim.x)
        size[t] = (t < nrem ? L.mask[rlist[t]] : R.mask[t - nrem]) + 1;
}

// next generation: remaining_clauses + unique_new (REF.py:127)
__global__ void dp_assemble_kernel(ClauseList L, const int64_t *rlist, int64_t nrem, Images R, const int64_t *klist,
                                   int64_t nkept, const uint64_t *rbits, const int64_t *ntlist, const int64_t *off,
                                   int K, ClauseList O) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nrem + nkept;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int32_t *src;
        const uint64_t *bsrc;
        int32_t mask, fill, used;
        if (t < nrem) {
            const int64_t c = rlist[t];
            src = L.pool + L.off[c];
            bsrc = L.bits + c * K;
            mask = L.mask[c];
            fill = L.fill[c];
            used = L.used[c];
        } else {
            const int64_t e = t - nrem;
            src = R.pool + R.off[e];
            bsrc = rbits + ntlist[klist[e]] * K;
            mask = R.mask[e];
            fill = R.fill[e];
            used = R.used[e];
        }
        int32_t *dst = O.pool + off[t];
        for (int32_t i = 0; i <= mask; ++i) dst[i] = src[i];
        for (int w = 0; w < K; ++w) O.bits[t * K + w] = bsrc[w];
        O.off[t] = off[t];
        O.mask[t] = mask;
        O.fill[t] = fill;
        O.used[t] = used;
    }
}

// ------------------------------------------------------------------ host side
namespace {

struct Buf {
    void *p = nullptr;
    size_t cap = 0;
    ~Buf() {
        if (p) (void)hipFree(p);
    }
    Buf() = default;
    Buf(const Buf &) = delete;
    int need(size_t bytes) {
        if (bytes <= cap) return SATMI_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(bytes + bytes / 2, 256);
        SATMI_HIP(hipMalloc(&p, want));
        cap = want;
        return SATMI_OK;
    }
    template <class T>
    T *as() const { return (T *)p; }
};

#define DP_TRY(x)                        \
    do {                                 \
        int _rc = (x);                   \
        if (_rc != SATMI_OK) return _rc; \
    } while (0)

struct Gen {   // one generation of the clause list
    Buf off, mask, fill, used, bits, pool;
    int reserve(int64_t n, int K, int64_t pool_slots) {
        DP_TRY(off.need(8 * (size_t)std::max<int64_t>(n, 1)));
        DP_TRY(mask.need(4 * (size_t)std::max<int64_t>(n, 1)));
        DP_TRY(fill.need(4 * (size_t)std::max<int64_t>(n, 1)));
        DP_TRY(used.need(4 * (size_t)std::max<int64_t>(n, 1)));
        DP_TRY(bits.need(8 * (size_t)std::max<int64_t>(n, 1) * K));
        DP_TRY(pool.need(4 * (size_t)std::max<int64_t>(pool_slots, 1)));
        return SATMI_OK;
    }
    ClauseList view() const {
        return {off.as<int64_t>(), mask.as<int32_t>(), fill.as<int32_t>(), used.as<int32_t>(), bits.as<uint64_t>(),
                pool.as<int32_t>()};
    }
};

struct Img {
    Buf pool, off, mask, fill, used;
    int64_t cap = 8;
    int reserve(int64_t n, int64_t c) {
        cap = c;
        n = std::max<int64_t>(n, 1);
        DP_TRY(pool.need(4 * (size_t)n * 2 * c));
        DP_TRY(off.need(8 * (size_t)n));
        DP_TRY(mask.need(4 * (size_t)n));
        DP_TRY(fill.need(4 * (size_t)n));
        DP_TRY(used.need(4 * (size_t)n));
        return SATMI_OK;
    }
    Images view() const {
        return {pool.as<int32_t>(), off.as<int64_t>(), mask.as<int32_t>(), fill.as<int32_t>(), used.as<int32_t>(),
                cap};
    }
};

// Work and device time of the last satmi_dp_host call's subsumption filter
// (HIP events on its stream), for bench.py's roofline.
struct DpStats {
    int64_t steps = 0, tests = 0, new_clauses = 0, candidates_bytes = 0;
    double subsume_ms = 0.0;
    int words = 0;
};
thread_local DpStats g_dp_stats;   // the calling thread's last call

// Everything one satmi_dp_host call allocates, kept between calls (grow-only)
// per host thread and device, with the thread's own non-blocking stream: a
// solve of a small formula is dozens of steps of small launches with a few
// host read-backs each, so allocating its ~40 buffers per call cost more than
// its kernels, and solves from several host threads overlap on the device
// (each fills a fraction of it).  Never destroyed: no hipFree after the
// runtime's teardown.
struct DpWork {
    Buf d_off, d_lits, d_v2d, d_d2v, misc, firstpos, order, popscratch, base, usedtmp;
    Buf fpos, fneg, frem, plist, nlist, rlist, scanpos, tiles, grand, counts3, rbits, nontaut, ntlist, kept, klist, kpos,
        sizes, offs;
    Gen g[2];
    Img A, B, R;
    std::vector<hipEvent_t> ev;   // subsumption-filter timing: one pair per step, read once per call
    hipStream_t stream = nullptr;
    int64_t *pin = nullptr;       // pinned host word: a step's pool size, read after the next step's first wait
};
DpWork *dp_work(int dev) {
    thread_local std::vector<DpWork *> mine;
    if ((int)mine.size() <= dev) mine.resize(dev + 1, nullptr);
    if (!mine[dev]) {
        DpWork *w = new DpWork;
        if (hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking) != hipSuccess ||
            hipHostMalloc((void **)&w->pin, 64, hipHostMallocDefault) != hipSuccess) {
            delete w;
            return nullptr;
        }
        mine[dev] = w;
    }
    return mine[dev];
}

// ordered compaction of flag[n] into out (indices); returns the count
// compact() without the count read-back: `out` is sized for all n, the count
// lands in *count_dev; several of these share one read-back (same stream, so
// pos / tiles are reused in order)
int compact_deferred(const int64_t *flag, int64_t n, Buf &pos, Buf &tiles, int64_t *count_dev, Buf &out,
                     hipStream_t s) {
    DP_TRY(pos.need(8 * (size_t)std::max<int64_t>(n, 1)));
    DP_TRY(tiles.need(8 * (size_t)((n + SCAN_TILE - 1) / SCAN_TILE + 1)));
    DP_TRY(out.need(8 * (size_t)std::max<int64_t>(n, 1)));
    DP_TRY(exclusive_scan(flag, pos.as<int64_t>(), n, tiles.as<int64_t>(), count_dev, s));
    if (n > 0)
        hipLaunchKernelGGL(dp_compact_kernel, dim3(grid_for(n)), dim3(PRIM_BLOCK), 0, s, flag, pos.as<int64_t>(), n,
                           out.as<int64_t>());
    SATMI_HIP(hipGetLastError());
    return SATMI_OK;
}

int compact(const int64_t *flag, int64_t n, Buf &pos, Buf &tiles, Buf &grand, Buf &out, int64_t *count,
            hipStream_t s) {
    *count = 0;
    if (n == 0) return SATMI_OK;
    DP_TRY(pos.need(8 * (size_t)n));
    DP_TRY(tiles.need(8 * (size_t)((n + SCAN_TILE - 1) / SCAN_TILE + 1)));
    DP_TRY(grand.need(8));
    DP_TRY(exclusive_scan(flag, pos.as<int64_t>(), n, tiles.as<int64_t>(), grand.as<int64_t>(), s));
    SATMI_HIP(hipMemcpyAsync(count, grand.p, 8, hipMemcpyDeviceToHost, s));
    SATMI_HIP(hipStreamSynchronize(s));
    DP_TRY(out.need(8 * (size_t)std::max<int64_t>(*count, 1)));
    hipLaunchKernelGGL(dp_compact_kernel, dim3(grid_for(n)), dim3(PRIM_BLOCK), 0, s, flag, pos.as<int64_t>(), n,
                       out.as<int64_t>());
    SATMI_HIP(hipGetLastError());
    return SATMI_OK;
}

}  // namespace
}  // namespace satmi

using namespace satmi;

extern "C" int satmi_dp_host(int nclauses, const int32_t *h_clause_off, const int32_t *h_lits, int64_t step_limit,
                             int64_t clause_limit, double time_limit_s, int32_t *h_result, int32_t *h_trace_vars,
                             int trace_cap, int32_t *h_steps, int32_t *h_rec_lits, int64_t rec_lit_cap,
                             int64_t *h_rec_clause_off, int64_t rec_clause_cap, int64_t *h_rec_step_off,
                             int rec_step_cap) {
    if (nclauses < 0 || (nclauses > 0 && (!h_clause_off || !h_lits)) || !h_result || !h_steps) {
        set_error("satmi_dp_host: bad arguments");
        return SATMI_ERR_ARG;
    }
    const auto t_start = std::chrono::steady_clock::now();
    *h_result = -1;
    *h_steps = 0;
    if (h_rec_step_off && rec_step_cap > 0) h_rec_step_off[0] = 0;
    if (h_rec_clause_off && rec_clause_cap > 0) h_rec_clause_off[0] = 0;
    const int64_t Ltot = nclauses > 0 ? h_clause_off[nclauses] : 0;
    int maxvar = 0, maxlen = 0;
    for (int c = 0; c < nclauses; ++c) maxlen = std::max(maxlen, h_clause_off[c + 1] - h_clause_off[c]);
    for (int64_t i = 0; i < Ltot; ++i) {
        if (h_lits[i] == 0 || h_lits[i] == INT32_MIN) {
            set_error("satmi_dp_host: literal 0 / INT32_MIN");
            return SATMI_ERR_ARG;
        }
        maxvar = std::max(maxvar, std::abs(h_lits[i]));
    }
    std::vector<int32_t> var2dense(maxvar + 1, -1), dense2var;
    for (int64_t i = 0; i < Ltot; ++i) var2dense[std::abs(h_lits[i])] = 1;
    for (int v = 1; v <= maxvar; ++v)
        if (var2dense[v] >= 0) {
            var2dense[v] = (int32_t)dense2var.size();
            dense2var.push_back(v);
        }
    const int V = (int)dense2var.size();
    const int W = std::max(1, (V + 63) / 64);
    const int K = 2 * W;
    int dev_id = 0;
    SATMI_HIP(hipGetDevice(&dev_id));
    DpWork *wk = dp_work(dev_id);
    if (!wk) {
        set_error("satmi_dp_host: hipStreamCreate failed");
        return SATMI_ERR_HIP;
    }
    DpWork &Wk = *wk;
    hipStream_t s = Wk.stream;
    Buf &d_off = Wk.d_off, &d_lits = Wk.d_lits, &d_v2d = Wk.d_v2d, &d_d2v = Wk.d_d2v, &misc = Wk.misc,
        &firstpos = Wk.firstpos, &order = Wk.order, &popscratch = Wk.popscratch, &base = Wk.base,
        &usedtmp = Wk.usedtmp;
    Buf &fpos = Wk.fpos, &fneg = Wk.fneg, &frem = Wk.frem, &plist = Wk.plist, &nlist = Wk.nlist, &rlist = Wk.rlist,
        &scanpos = Wk.scanpos, &tiles = Wk.tiles, &grand = Wk.grand, &counts3 = Wk.counts3, &rbits = Wk.rbits,
        &nontaut = Wk.nontaut, &ntlist = Wk.ntlist, &kept = Wk.kept, &klist = Wk.klist, &kpos = Wk.kpos,
        &sizes = Wk.sizes, &offs = Wk.offs;
    Gen *g = Wk.g;
    Img &A = Wk.A, &B = Wk.B, &R = Wk.R;
    DP_TRY(d_off.need(4 * (size_t)(nclauses + 1)));
    DP_TRY(d_lits.need(4 * (size_t)std::max<int64_t>(Ltot, 1)));
    DP_TRY(d_v2d.need(4 * (size_t)(maxvar + 1)));
    DP_TRY(d_d2v.need(4 * (size_t)std::max(V, 1)));
    DP_TRY(misc.need(64));
    int cur = 0;
    int64_t ncl = nclauses;
    int64_t pool_cur = 0;         // pool slots of g[cur] (exact, or this step's bound until read back)
    bool pool_pending = false;    // Wk.pin[0] holds g[cur]'s exact pool size after the next wait
    {
        const int64_t cap0 = cap_for(maxlen);
        pool_cur = ncl * 2 * cap0;
        DP_TRY(g[0].reserve(ncl, K, pool_cur));
        if (nclauses > 0) {
            SATMI_HIP(hipMemcpyAsync(d_off.p, h_clause_off, 4 * (size_t)(nclauses + 1), hipMemcpyHostToDevice, s));
            if (Ltot) SATMI_HIP(hipMemcpyAsync(d_lits.p, h_lits, 4 * (size_t)Ltot, hipMemcpyHostToDevice, s));
            SATMI_HIP(hipMemcpyAsync(d_v2d.p, var2dense.data(), 4 * (size_t)(maxvar + 1), hipMemcpyHostToDevice, s));
        }
        if (V) SATMI_HIP(hipMemcpyAsync(d_d2v.p, dense2var.data(), 4 * (size_t)V, hipMemcpyHostToDevice, s));
        SATMI_HIP(hipMemsetAsync(misc.p, 0, 64, s));
        if (nclauses > 0) {
            hipLaunchKernelGGL(dp_encode_kernel, dim3(grid_for(nclauses)), dim3(PRIM_BLOCK), 0, s, nclauses,
                               d_off.as<int32_t>(), d_lits.as<int32_t>(), d_v2d.as<int32_t>(), W, cap0,
                               g[0].view(), misc.as<int>());
            SATMI_HIP(hipGetLastError());
        }
    }
    // subsumption-filter timing (satmi_dp_last_stats): an event pair per step,
    // read after the loop (no per-step wait); misc[40..48) counts its subset tests
    size_t nev = 0;   // event pairs recorded this call
    const auto next_events = [&]() -> hipEvent_t * {
        if (2 * nev + 2 > Wk.ev.size()) {
            hipEvent_t a = nullptr, b = nullptr;
            if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return nullptr;
            Wk.ev.push_back(a);
            Wk.ev.push_back(b);
        }
        return &Wk.ev[2 * nev++];
    };
    g_dp_stats = DpStats{};
    g_dp_stats.words = K;
    DP_TRY(firstpos.need(8 * (size_t)std::max(V, 1)));
    DP_TRY(order.need(4 * (size_t)std::max(V, 1)));
    const int64_t popcap = cap_for(V);
    DP_TRY(popscratch.need(4 * (size_t)2 * popcap));
    int steps = 0, result = 1;
    int64_t rec_clauses = 0, rec_lits = 0;
    std::vector<int32_t> h_pool;
    std::vector<int64_t> h_off;
    std::vector<int32_t> h_mask;
    for (;;) {
        // variables = {abs(lit) ...}; while variables: var = variables.pop()
        if (ncl == 0) break;   // no clauses, no variables: True
        ClauseList Lc = g[cur].view();
        DP_TRY(base.need(8 * (size_t)ncl));
        DP_TRY(usedtmp.need(8 * (size_t)ncl));
        DP_TRY(tiles.need(8 * (size_t)((ncl + SCAN_TILE - 1) / SCAN_TILE + 1)));
        DP_TRY(grand.need(8));
        hipLaunchKernelGGL(dp_used_kernel, dim3(grid_for(ncl)), dim3(PRIM_BLOCK), 0, s, Lc, ncl,
                           usedtmp.as<int64_t>());
        DP_TRY(exclusive_scan(usedtmp.as<int64_t>(), base.as<int64_t>(), ncl, tiles.as<int64_t>(),
                              grand.as<int64_t>(), s));
        SATMI_HIP(hipMemsetAsync(firstpos.p, 0xff, 8 * (size_t)std::max(V, 1), s));
        hipLaunchKernelGGL(dp_firstpos_kernel, dim3(grid_for(ncl)), dim3(PRIM_BLOCK), 0, s, Lc, ncl,
                           base.as<int64_t>(), d_v2d.as<int32_t>(), firstpos.as<unsigned long long>());
        hipLaunchKernelGGL(dp_pop_kernel, dim3(1), dim3(256), 0, s, firstpos.as<unsigned long long>(),
                           d_d2v.as<int32_t>(), V, order.as<int32_t>(), popscratch.as<int32_t>(), popcap,
                           misc.as<int32_t>() + 4);
        SATMI_HIP(hipGetLastError());
        int32_t pop[3] = {0, 0, 0};
        int32_t ovf = 0;
        SATMI_HIP(hipMemcpyAsync(pop, misc.as<int32_t>() + 4, 12, hipMemcpyDeviceToHost, s));
        SATMI_HIP(hipMemcpyAsync(&ovf, misc.p, 4, hipMemcpyDeviceToHost, s));
        SATMI_HIP(hipStreamSynchronize(s));
        if (ovf || pop[2]) {
            set_error("satmi_dp_host: set model table overflow");
            return SATMI_ERR_TOO_LARGE;
        }
        if (pool_pending) {   // the previous step's exact pool size, copied behind its assembly
            pool_cur = Wk.pin[0];
            pool_pending = false;
        }
        if (pop[1] == 0) break;   // `while variables` ends: True (REF.py:130)
        if (step_limit > 0 && steps >= step_limit) {
            result = -1;
            break;
        }
        if (time_limit_s > 0 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count() > time_limit_s) {
            result = -1;
            break;
        }
        const int32_t var = pop[0];
        const int d = var2dense[var];
        if (h_trace_vars && steps < trace_cap) h_trace_vars[steps] = var;
        ++steps;
        // split (REF.py:106-108)
        DP_TRY(fpos.need(8 * (size_t)ncl));
        DP_TRY(fneg.need(8 * (size_t)ncl));
        DP_TRY(frem.need(8 * (size_t)ncl));
        unsigned long long *d_mx = (unsigned long long *)(misc.as<char>() + 48);
        SATMI_HIP(hipMemsetAsync(d_mx, 0, 16, s));
        hipLaunchKernelGGL(dp_split_kernel, dim3(grid_for(ncl)), dim3(PRIM_BLOCK), 0, s, Lc, ncl, W, d,
                           fpos.as<int64_t>(), fneg.as<int64_t>(), frem.as<int64_t>(), d_mx);
        // the three lists with one count read-back
        DP_TRY(counts3.need(3 * sizeof(int64_t)));
        int64_t *c3 = counts3.as<int64_t>();
        DP_TRY(compact_deferred(fpos.as<int64_t>(), ncl, scanpos, tiles, c3 + 0, plist, s));
        DP_TRY(compact_deferred(fneg.as<int64_t>(), ncl, scanpos, tiles, c3 + 1, nlist, s));
        DP_TRY(compact_deferred(frem.as<int64_t>(), ncl, scanpos, tiles, c3 + 2, rlist, s));
        int64_t h3[3] = {0, 0, 0};
        unsigned long long mx[2] = {0, 0};
        SATMI_HIP(hipMemcpyAsync(h3, c3, sizeof(h3), hipMemcpyDeviceToHost, s));
        SATMI_HIP(hipMemcpyAsync(mx, d_mx, sizeof(mx), hipMemcpyDeviceToHost, s));
        SATMI_HIP(hipStreamSynchronize(s));
        const int64_t np = h3[0], nn = h3[1], nr = h3[2];
        const int64_t npairs = np * nn;
        // resolvent bitsets + flags (REF.py:111-119)
        int64_t m = 0;
        unsigned long long first_empty = ~0ull;
        if (npairs > 0) {
            DP_TRY(rbits.need(8 * (size_t)npairs * K));
            DP_TRY(nontaut.need(8 * (size_t)npairs));
            SATMI_HIP(hipMemsetAsync(misc.as<char>() + 32, 0xff, 8, s));
            hipLaunchKernelGGL(dp_pairs_kernel, dim3(grid_for(npairs)), dim3(PRIM_BLOCK), 0, s, Lc,
                               plist.as<int64_t>(), nlist.as<int64_t>(), nn, npairs, W, d, rbits.as<uint64_t>(),
                               nontaut.as<int64_t>(), (unsigned long long *)(misc.as<char>() + 32));
            SATMI_HIP(hipGetLastError());
            SATMI_HIP(hipMemcpyAsync(&first_empty, misc.as<char>() + 32, 8, hipMemcpyDeviceToHost, s));
            DP_TRY(compact(nontaut.as<int64_t>(), npairs, scanpos, tiles, grand, ntlist, &m, s));
        }
        // the reference stops at the first empty resolvent, or (clause_limit) when
        // remaining + new grows past the limit, whichever comes first in pair order
        int64_t limit_pair = -1;
        const int64_t kth = std::max<int64_t>(clause_limit - nr, 0);   // 0-based index of the offending new clause
        if (clause_limit > 0 && m > kth) {
            int64_t p = 0;
            SATMI_HIP(hipMemcpyAsync(&p, ntlist.as<int64_t>() + kth, 8, hipMemcpyDeviceToHost, s));
            SATMI_HIP(hipStreamSynchronize(s));
            limit_pair = p;
        }
        if (first_empty != ~0ull && (limit_pair < 0 || (int64_t)first_empty <= limit_pair)) {
            result = 0;   // empty clause: unsatisfiable (REF.py:117-118)
            break;
        }
        if (limit_pair >= 0) {
            result = -1;
            break;
        }
        // unique_new (REF.py:122-125)
        int64_t nkept = 0;
        if (m > 0) {
            DP_TRY(kept.need(8 * (size_t)m));
            const int64_t *rl = rlist.as<int64_t>(), *ntl = ntlist.as<int64_t>();
            const uint64_t *rb = rbits.as<uint64_t>();
            int64_t *kp = kept.as<int64_t>();
            unsigned long long *tc = (unsigned long long *)(misc.as<char>() + 40);
            hipEvent_t *ev_sub = next_events();
            if (!ev_sub) {
                set_error("satmi_dp_host: hipEventCreate failed");
                return SATMI_ERR_HIP;
            }
            SATMI_HIP(hipEventRecord(ev_sub[0], s));
            if (K <= 8 && (K & 1) == 0) {
                auto tiled = [&](const int64_t *sel, int64_t nsel, int64_t lo, int64_t hi) {
                    const dim3 g((unsigned)((nsel + SUB_TILE - 1) / SUB_TILE),
                                 (unsigned)std::max<int64_t>(1, (hi - lo + SUB_CHUNK - 1) / SUB_CHUNK));
                    if (K == 2)
                        hipLaunchKernelGGL((dp_subsume_tiled_kernel<2>), g, dim3(SUB_TILE), 0, s, Lc, rl, nr, rb, ntl,
                                           sel, nsel, lo, hi, kp, tc);
                    else if (K == 4)
                        hipLaunchKernelGGL((dp_subsume_tiled_kernel<4>), g, dim3(SUB_TILE), 0, s, Lc, rl, nr, rb, ntl,
                                           sel, nsel, lo, hi, kp, tc);
                    else if (K == 6)
                        hipLaunchKernelGGL((dp_subsume_tiled_kernel<6>), g, dim3(SUB_TILE), 0, s, Lc, rl, nr, rb, ntl,
                                           sel, nsel, lo, hi, kp, tc);
                    else
                        hipLaunchKernelGGL((dp_subsume_tiled_kernel<8>), g, dim3(SUB_TILE), 0, s, Lc, rl, nr, rb, ntl,
                                           sel, nsel, lo, hi, kp, tc);
                };
                hipLaunchKernelGGL(dp_ones_kernel, dim3(grid_for(m)), dim3(PRIM_BLOCK), 0, s, kp, m);
                const int64_t total = nr + m;
                const int64_t pre = std::min<int64_t>(SUB_PREFIX, total);
                tiled(nullptr, m, 0, pre);   // every new clause: the first candidates
                if (pre < total) {           // survivors: the rest
                    int64_t nsurv = 0;
                    DP_TRY(compact(kp, m, kpos, tiles, grand, klist, &nsurv, s));
                    if (nsurv > 0) tiled(klist.as<int64_t>(), nsurv, pre, total);
                }
            } else {
                hipLaunchKernelGGL(dp_subsume_kernel, dim3(grid_for(m * 64)), dim3(PRIM_BLOCK), 0, s, Lc, rl, nr, rb,
                                   ntl, m, K, kp);
            }
            SATMI_HIP(hipEventRecord(ev_sub[1], s));
            SATMI_HIP(hipGetLastError());
            g_dp_stats.new_clauses += m;
            g_dp_stats.candidates_bytes += (nr + m) * K * 8;
            DP_TRY(compact(kept.as<int64_t>(), m, kpos, tiles, grand, klist, &nkept, s));
        }
        if (nkept > 0) {
            // images of AX, BY and the kept resolvents (capacities from the split's mx)
            DP_TRY(A.reserve(np, cap_for((int64_t)mx[0])));
            DP_TRY(B.reserve(nn, cap_for((int64_t)mx[1])));
            DP_TRY(R.reserve(nkept, cap_for((int64_t)mx[0] + (int64_t)mx[1])));
            hipLaunchKernelGGL(dp_diff_kernel, dim3(grid_for(np)), dim3(PRIM_BLOCK), 0, s, Lc, plist.as<int64_t>(),
                               np, var, A.view(), misc.as<int>());
            hipLaunchKernelGGL(dp_diff_kernel, dim3(grid_for(nn)), dim3(PRIM_BLOCK), 0, s, Lc, nlist.as<int64_t>(),
                               nn, -var, B.view(), misc.as<int>());
            hipLaunchKernelGGL(dp_build_kernel, dim3(grid_for(m)), dim3(PRIM_BLOCK), 0, s, A.view(), B.view(),
                               ntlist.as<int64_t>(), kept.as<int64_t>(), kpos.as<int64_t>(), m, nn, R.view(),
                               misc.as<int>());
            SATMI_HIP(hipGetLastError());
        }
        // clauses = remaining_clauses + unique_new (REF.py:127)
        const int64_t ncl2 = nr + nkept;
        int64_t pool2 = 0;
        if (ncl2 > 0) {
            DP_TRY(sizes.need(8 * (size_t)ncl2));
            DP_TRY(offs.need(8 * (size_t)ncl2));
            hipLaunchKernelGGL(dp_sizes_kernel, dim3(grid_for(ncl2)), dim3(PRIM_BLOCK), 0, s, Lc, rlist.as<int64_t>(),
                               nr, R.view(), nkept, sizes.as<int64_t>());
            DP_TRY(tiles.need(8 * (size_t)((ncl2 + SCAN_TILE - 1) / SCAN_TILE + 1)));
            DP_TRY(exclusive_scan(sizes.as<int64_t>(), offs.as<int64_t>(), ncl2, tiles.as<int64_t>(),
                                  grand.as<int64_t>(), s));
            // the next generation's pool: reserved for a bound (the remaining
            // clauses' tables are regions of g[cur]'s pool; a kept resolvent's
            // image has <= 2 x R.cap slots), the exact size copied back behind
            // the assembly and read after the next step's first wait (no wait
            // here; recording reads it at once)
            const int64_t pool_ub = pool_cur + nkept * 2 * R.cap;
            SATMI_HIP(hipMemcpyAsync(Wk.pin, grand.p, 8, hipMemcpyDeviceToHost, s));
            const int nxt = cur ^ 1;
            DP_TRY(g[nxt].reserve(ncl2, K, pool_ub));
            hipLaunchKernelGGL(dp_assemble_kernel, dim3(grid_for(ncl2)), dim3(PRIM_BLOCK), 0, s, Lc,
                               rlist.as<int64_t>(), nr, R.view(), klist.as<int64_t>(), nkept, rbits.as<uint64_t>(),
                               ntlist.as<int64_t>(), offs.as<int64_t>(), K, g[nxt].view());
            SATMI_HIP(hipGetLastError());
            cur = nxt;
            pool_cur = pool_ub;
            pool_pending = true;
        }
        ncl = ncl2;
        // record the clause list after the step, each clause in its set iteration order
        if (h_rec_lits && h_rec_clause_off && h_rec_step_off && steps < rec_step_cap) {
            h_off.resize((size_t)std::max<int64_t>(ncl, 1));
            h_mask.resize((size_t)std::max<int64_t>(ncl, 1));
            h_pool.resize((size_t)std::max<int64_t>(pool2, 1));
            if (ncl > 0) {
                SATMI_HIP(hipStreamSynchronize(s));   // Wk.pin[0] = pool2
                pool2 = Wk.pin[0];
                h_pool.resize((size_t)std::max<int64_t>(pool2, 1));
                SATMI_HIP(hipMemcpyAsync(h_off.data(), g[cur].off.p, 8 * (size_t)ncl, hipMemcpyDeviceToHost, s));
                SATMI_HIP(hipMemcpyAsync(h_mask.data(), g[cur].mask.p, 4 * (size_t)ncl, hipMemcpyDeviceToHost, s));
                SATMI_HIP(hipMemcpyAsync(h_pool.data(), g[cur].pool.p, 4 * (size_t)pool2, hipMemcpyDeviceToHost, s));
                SATMI_HIP(hipStreamSynchronize(s));
            }
            for (int64_t c = 0; c < ncl && rec_clauses + 1 < rec_clause_cap; ++c) {
                for (int64_t i = 0; i <= h_mask[c]; ++i) {
                    const int32_t k = h_pool[h_off[c] + i];
                    if (k != PY_EMPTY && k != PY_DUMMY && rec_lits < rec_lit_cap) h_rec_lits[rec_lits++] = k;
                }
                h_rec_clause_off[++rec_clauses] = rec_lits;
            }
            h_rec_step_off[steps] = rec_clauses;
        }
        // the set-model overflow flag (misc[0]) of this step is read with the
        // next step's pop, or after the loop
    }
    {
        int32_t ovf2 = 0;
        SATMI_HIP(hipMemcpyAsync(&ovf2, misc.p, 4, hipMemcpyDeviceToHost, s));
        SATMI_HIP(hipStreamSynchronize(s));
        if (ovf2) {
            set_error("satmi_dp_host: set model table overflow");
            return SATMI_ERR_TOO_LARGE;
        }
    }
    {
        unsigned long long tests = 0;
        SATMI_HIP(hipMemcpyAsync(&tests, misc.as<char>() + 40, 8, hipMemcpyDeviceToHost, s));
        SATMI_HIP(hipStreamSynchronize(s));
        g_dp_stats.tests = (int64_t)tests;
        g_dp_stats.steps = steps;
        for (size_t i = 0; i < nev; ++i) {   // the stream has drained
            float ms = 0.0f;
            if (hipEventElapsedTime(&ms, Wk.ev[2 * i], Wk.ev[2 * i + 1]) == hipSuccess) g_dp_stats.subsume_ms += ms;
        }
    }
    *h_result = result;
    *h_steps = steps;
    return SATMI_OK;
}

extern "C" int satmi_dp_last_stats(int64_t *steps, int64_t *subset_tests, int64_t *new_clauses,
                                   int64_t *candidate_bytes, int *words, double *subsume_ms) {
    if (steps) *steps = g_dp_stats.steps;
    if (subset_tests) *subset_tests = g_dp_stats.tests;
    if (new_clauses) *new_clauses = g_dp_stats.new_clauses;
    if (candidate_bytes) *candidate_bytes = g_dp_stats.candidates_bytes;
    if (words) *words = g_dp_stats.words;
    if (subsume_ms) *subsume_ms = g_dp_stats.subsume_ms;
    return SATMI_OK;
}
