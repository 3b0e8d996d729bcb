// dp.hip -- Davis-Putnam variable elimination (REF.py:98-130) on gfx950.
//
// One elimination step of the reference: pick `var = variables.pop()`, split
// the clause list into clauses with var / with -var / without it, resolve
// every (pos, neg) pair in list order, drop tautologies, return False on an
// empty resolvent, keep a resolvent unless an earlier-listed clause of
// `remaining + unique_new` is a subset of it, continue with remaining + kept.
//
// GPU formulation.  Every clause carries (a) a bitset key over the dense
// variable index for the set algebra and (b) its CPython table image
// (pyset_dev.h) in an image arena, because the reference's elimination order
// is decided by CPython's set layout.  A step is a fixed sequence of eight
// launches whose sizes live on the device (DpState): the host enqueues whole
// batches of steps and waits once per batch -- a step never waits on the host.
//
//   pop_split  (1 workgroup) variables.pop() from the first-position table the
//              previous step left, then the order-preserving split into the
//              pos / neg / rem lists (block prefix sums);
//   pairs      resolvent key of every (pos, neg) pair, tautology / empty
//              flags, the non-tautological pairs as a bitmap;
//   hash       one representative per distinct resolvent: the FIRST pair (in
//              pair order) holding that key, by atomicMin in a hash table; each
//              key's table slot into a stripe region (read in stripe order
//              as the representatives' list by the next two kernels);
//   remtest    every representative against the remaining clauses (2-D grid:
//              representative tiles x rem chunks, rem keys broadcast from LDS);
//   survlist   the representatives no rem clause subsumes (and the table
//              cleared for the next step);
//   survtest   every survivor against the survivors earlier in pair order;
//   kept       (1 workgroup) the empty-clause / clause-limit verdict, the kept
//              survivors in pair order (bitmap + block scan), capacities;
//   assemble   the next clause list: rem clauses (their images stay where they
//              are) + the kept resolvents' images `(pc - {var}) | (nc - {-var})`
//              built in the arena, and the next step's first-position table.
//
// Why this equals the reference's greedy `unique_new` (REF.py:122-125): a new
// clause x is dropped iff a rem clause or an earlier KEPT new clause is a
// subset of it.  That equals "a rem clause or ANY earlier new clause is a
// subset": an earlier new clause y that was itself dropped was dropped for a
// subset z (rem or kept before y) that is also a subset of x.  The earlier
// new clauses can further be narrowed to earlier representatives that
// survived the rem test: a duplicate of an earlier clause has that earlier
// representative, and a y with a rem subset r gives x the same r.  So x is
// kept iff x is its key's first occurrence, no rem clause is a subset of x,
// and no earlier rem-surviving representative is a subset of x.
//
// Capacities are host-known; a step whose sizes exceed one sets `overflow`
// (nothing of the step's input is lost), the host grows the buffer and
// resumes from that step.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <vector>

#include "common.h"
#include "prims.h"
#include "pyset_dev.h"

namespace satmi {

// smallest power of two >= 8 that exceeds 8*u: room for every table a set of u
// keys passes through (add: < 8u, merge: < 4u)
__host__ __device__ static inline int64_t cap_for(int64_t u) {
    int64_t c = PY_MINSIZE;
    while (c <= 8 * u) c <<= 1;
    return c;
}

// overflow bits (DpState::overflow) and what the host grows for each
enum : int32_t { OVF_PAIRS = 1, OVF_NCL = 2, OVF_ARENA = 4, OVF_XS = 8 };

constexpr uint64_t DP_EMPTY = ~0ull;
constexpr int DP_STRIPES = 64;
#ifndef DP_GRID_PAIRS   // grid caps of the step's kernels (grid-stride: a cap only bounds the dispatch)
#define DP_GRID_PAIRS 1024
#endif
#ifndef DP_GRID_TEST
#define DP_GRID_TEST 2048
#endif
#ifndef DP_GRID_ASM
#define DP_GRID_ASM 2048
#endif
constexpr int DP_LAUNCHES_PER_STEP = 8;   // pop_split, pairs, hash, remtest, survlist, survtest, kept, assemble

// The solve's state, on the device.  Host writes it once per solve (and on a
// resume); kernels read sizes from it and one thread of the single-workgroup
// kernels updates it.
struct DpState {
    int64_t ncl, ncl2;             // clauses of g[cur]; of the generation being assembled (pending)
    int64_t np, nn, nr, npairs;    // this step's split
    int64_t nontaut, nuniq, nsurv, nkept;
    int64_t arena_top, arena_base;   // image arena bump pointer; this step's kept images
    int64_t tests, new_total;        // subset tests, non-tautological resolvents (whole solve)
    int64_t need[4];                 // sizes wanted on overflow (pairs, ncl, arena, xs)
    uint64_t first_empty;            // first pair (in pair order) with an empty resolvent
    uint64_t t0;                     // s_memrealtime at the solve's start
    int32_t cur, pending, done, result, steps, overflow, set_ovf, var, d;
    int32_t mxA, mxB, capA, capB, capR, epoch;
    int32_t skip;    // this step slot's pipeline kernels have nothing to do (an inline step ended the slot)
    int32_t slots;   // step slots that ran (the host sizes its next batch by them)
    uint64_t ph[8];  // wall-clock ticks of dp_pop_split_kernel's phases (SATMI_DP_PHASES=1 prints them)
    int64_t inl_steps;   // steps run inline
};

struct ClauseList {   // one generation of the clause list
    int64_t *off;     // image offset in the arena
    int32_t *mask, *fill, *used;
    uint64_t *bits;   // K words per clause: positive then negative literal bits
};

// Everything a step's kernels touch, by value (pointers + host-known capacities).
struct DpArgs {
    DpState *st;
    ClauseList g[2];
    int32_t *arena;
    int64_t arena_cap;
    const int32_t *v2d, *d2v;
    int V, W, K;
    unsigned long long *firstpos;   // per dense variable: (clause << 32 | slot) of its first visit
    int32_t *order, *popscratch;
    int64_t popcap;
    int64_t *plist, *nlist, *rlist;
    int64_t ncl_cap;
    uint64_t *rbits, *ntbits;       // resolvent keys; non-tautological pairs bitmap (64 per word)
    int64_t pair_cap;               // < 2^31: pair indices are 32-bit
    uint64_t *table;                // hash table of representatives (pair index, DP_EMPTY)
    uint64_t tmask;
    uint32_t *uslot;                // table slot of each distinct key
    int32_t *dropped, *hit;         // epoch stamps: representative subsumed by rem / survivor hit
    uint32_t *surv, *klist;         // survivors' pair indices; kept pairs in pair order
    uint64_t *rkeys, *skeys;          // contiguous keys: rem clauses, survivors
    // Per-step counters striped over DP_STRIPES words each (stripe = block
    // index mod DP_STRIPES): [0, S) representatives claimed per stripe, [S, 2S)
    // non-tautological pairs, [2S, 3S) subset tests.  One hot counter
    // serialises its atomics (~60 ns each under contention).  A stripe's claimed
    // table slots go to its own region of ustage (pair_cap entries each).
    unsigned long long *stripes;
    uint32_t *ustage;
    uint32_t *keptbits;             // kept pairs (32 per word), cleared as compacted
    int32_t *xs;                    // per kept resolvent: AX and BY image scratch
    int64_t xs_cap;
    int32_t *trace;
    int trace_cap;
    int64_t step_limit, clause_limit;
    uint64_t limit_ticks;
    int32_t inline_steps;   // steps one slot may run inside dp_pop_split_kernel (see "Inline steps")
    int32_t pad_;
};

__device__ __forceinline__ DView cl_view(const ClauseList &L, const int32_t *arena, int64_t c) {
    return {arena + L.off[c], (int64_t)L.mask[c], (int64_t)L.fill[c], (int64_t)L.used[c]};
}

// block-wide exclusive prefix sum (every thread of the block calls it)
__device__ __forceinline__ int block_excl_scan(int x, int *wsum, int &total) {
    const int lane = lane_id(), wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int incl = wave_incl_scan(x);
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    int off = 0, tot = 0;
    for (int w = 0; w < nw; ++w) {
        const int v = wsum[w];
        off += w < wid ? v : 0;
        tot += v;
    }
    __syncthreads();
    total = tot;
    return off + incl - x;
}

__device__ __forceinline__ int block_sum(int x, int *wsum) {
    int t;
    (void)block_excl_scan(x, wsum, t);
    return t;
}

__device__ __forceinline__ int block_max(int x, int *wsum) {
    const int m = wave_max_i32(x);
    const int wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if (lane_id() == 0) wsum[wid] = m;
    __syncthreads();
    int r = 0;
    for (int w = 0; w < nw; ++w) r = max(r, wsum[w]);
    __syncthreads();
    return r;
}

// A value loaded before a kernel's early-exit test stays loaded there (the
// compiler would otherwise sink the load below the test: a second round trip)
#define DP_KEEP(x) asm volatile("" ::"s"(x))

// Several block reductions in one LDS exchange (two barriers in all; the
// single-workgroup kernels are chains of such exchanges).  ws: 16 ints per
// value (up to 16 waves).
__device__ __forceinline__ int wave_sum_i32(int x) {
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
    return x;
}
// a summed, b and c maxed (all >= 0)
__device__ __forceinline__ void block_sum_max_max(int &a, int &b, int &c, int *ws) {
    const int sa = wave_sum_i32(a), mb = wave_max_i32(b), mc = wave_max_i32(c);
    const int wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if (lane_id() == 0) {
        ws[wid] = sa;
        ws[16 + wid] = mb;
        ws[32 + wid] = mc;
    }
    __syncthreads();
    int ra = 0, rb = 0, rc = 0;
    for (int w = 0; w < nw; ++w) {
        ra += ws[w];
        rb = max(rb, ws[16 + w]);
        rc = max(rc, ws[32 + w]);
    }
    __syncthreads();
    a = ra;
    b = rb;
    c = rc;
}
// exclusive prefix sums of x and y (block totals in tx, ty)
__device__ __forceinline__ void block_excl_scan2(int &x, int &y, int *ws, int &tx, int &ty) {
    const int lane = lane_id(), wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int ix = wave_incl_scan(x), iy = wave_incl_scan(y);
    if (lane == 63) {
        ws[wid] = ix;
        ws[16 + wid] = iy;
    }
    __syncthreads();
    int ox = 0, oy = 0, sx = 0, sy = 0;
    for (int w = 0; w < nw; ++w) {
        const int vx = ws[w], vy = ws[16 + w];
        ox += w < wid ? vx : 0;
        oy += w < wid ? vy : 0;
        sx += vx;
        sy += vy;
    }
    __syncthreads();
    tx = sx;
    ty = sy;
    x = ox + ix - x;
    y = oy + iy - y;
}

// The visiting order of `{abs(lit) for clause in clauses for lit in clause}`
// (REF.py:100/:128): clause t's table slot i is position (t << 32 | i).  The
// first position of every variable is an atomicMin, reduced in LDS per block
// when the variables fit (lfp: the block's LDS table, used iff A.V <= FP_LDS).
constexpr int FP_LDS = 2048;
__device__ __forceinline__ void firstpos_clause(const DpArgs &A, unsigned long long *lfp, const int32_t *t, int64_t mask,
                                                int64_t c) {
    for (int64_t i = 0; i <= mask; ++i) {
        const int32_t k = t[i];
        if (k == PY_EMPTY || k == PY_DUMMY) continue;
        const int d = A.v2d[k < 0 ? -k : k];
        const unsigned long long pos = ((unsigned long long)c << 32) | (unsigned long long)i;
        if (A.V <= FP_LDS)
            atomicMin(&lfp[d], pos);
        else
            atomicMin(&A.firstpos[d], pos);
    }
}
__device__ __forceinline__ void firstpos_begin(const DpArgs &A, unsigned long long *lfp) {
    if (A.V <= FP_LDS)
        for (int d = threadIdx.x; d < A.V; d += blockDim.x) lfp[d] = ~0ull;
    __syncthreads();
}
__device__ __forceinline__ void firstpos_flush(const DpArgs &A, unsigned long long *lfp) {
    __syncthreads();
    if (A.V <= FP_LDS)
        for (int d = threadIdx.x; d < A.V; d += blockDim.x)
            if (lfp[d] != ~0ull) atomicMin(&A.firstpos[d], lfp[d]);
}

// clauses = [set(clause) for clause in formula]  (REF.py:99): image c at arena + 2*cap*c
__global__ void __launch_bounds__(256) dp_encode_kernel(DpArgs A, int nclauses, const int32_t *off,
                                                        const int32_t *lits, int64_t cap) {
    __shared__ unsigned long long lfp_sh[FP_LDS];
    unsigned long long *lfp = lfp_sh;   // used when A.V <= FP_LDS (an LDS pointer: ds_* atomics)
    if (blockIdx.x == 0 && threadIdx.x == 0) A.st->t0 = __builtin_amdgcn_s_memrealtime();
    firstpos_begin(A, lfp);
    const ClauseList L = A.g[0];
    const int W = A.W, K = A.K;
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < nclauses; c += gridDim.x * blockDim.x) {
        int32_t *a = A.arena + (int64_t)c * 2 * cap;
        DSet s;
        dset_init(s, a, a + cap, cap);
        uint64_t *k = L.bits + (int64_t)c * K;
        for (int w = 0; w < K; ++w) k[w] = 0ull;
        for (int j = off[c]; j < off[c + 1]; ++j) {
            const int x = lits[j];
            py_add(s, x);
            const int d = A.v2d[x < 0 ? -x : x];
            k[(x < 0 ? W : 0) + (d >> 6)] |= 1ull << (d & 63);
        }
        if (s.overflow) A.st->set_ovf = 1;
        L.off[c] = s.t - A.arena;
        L.mask[c] = (int32_t)s.mask;
        L.fill[c] = (int32_t)s.fill;
        L.used[c] = (int32_t)s.used;
        firstpos_clause(A, lfp, s.t, s.mask, c);
    }
    firstpos_flush(A, lfp);
}

// the first-position table of g[cur] from scratch (a resumed solve)
__global__ void __launch_bounds__(256) dp_firstpos_kernel(DpArgs A) {
    __shared__ unsigned long long lfp_sh[FP_LDS];
    unsigned long long *lfp = lfp_sh;   // used when A.V <= FP_LDS (an LDS pointer: ds_* atomics)
    firstpos_begin(A, lfp);
    const DpState *S = A.st;
    const ClauseList L = A.g[S->cur];
    const int64_t n = S->ncl;
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n; c += (int64_t)gridDim.x * blockDim.x)
        firstpos_clause(A, lfp, A.arena + L.off[c], L.mask[c], c);
    firstpos_flush(A, lfp);
}

// variables.pop() (REF.py:100-103, :128) and the split (REF.py:106-108): one
// workgroup of 1024 threads.
constexpr int POP_THREADS = 1024;
constexpr int POP_LDS = 2048;   // model-set table slots kept in LDS (cap_for(V) <= this: V <= 255)

// ---- Inline steps.  Most steps of a solve are small (PHP(6,5): 22 of its 30
// steps resolve <= 5,400 pairs; the other 8 up to 3.3 * 10^5), and a small
// step is nine kernel launches of a few microseconds each -- a dependent chain
// whose latency, not its work, is the step's time.  So a step whose pairs fit
// one workgroup runs to its end inside dp_pop_split_kernel, with barriers
// between the phases instead of launch boundaries, and the kernel goes on to
// the next step's pop while the steps stay small; the first step that does
// not fit is split and left to the pipeline kernels queued behind (S->skip
// tells them whether the slot left them a step).  The phases restate the
// pipeline's exactly: resolvent keys in pair order, the first pair of each
// distinct key as its representative (a hash table with atomicMin), the rem
// subset test, the earlier-survivor subset test, the verdict / clause limit,
// the kept resolvents in pair order, and the next clause list with the kept
// resolvents' CPython set images built as dp_assemble_kernel builds them.
constexpr int INL_PMAX = 8192;                 // pairs of an inline step
constexpr int INL_TILE_WORDS = 4096;           // candidate-key tile of the subset tests (32 KB); the
                                               // assembly's per-wave scratch in the same LDS
constexpr int INL_ASM_SCRATCH = 2 * INL_TILE_WORDS / (POP_THREADS / 64);   // int32 per wave: AX, BY, R tables
constexpr int INL_ASM_MAX = 32;                // kept resolvents assembled here (more: dp_assemble_kernel)
struct InlLds {
    uint32_t ntb[INL_PMAX / 32];   // non-tautological pairs
    uint32_t flg[INL_PMAX / 32];   // representatives (by pair), dropped (by representative), hit (by survivor)
    uint16_t ua[INL_PMAX];         // representatives' pair indices, later the kept ones (pair order)
    uint16_t ub[INL_PMAX];         // survivors' pair indices (pair order)
    uint64_t tile[INL_TILE_WORDS];
    uint32_t fe;                   // first pair with an empty resolvent
    int64_t arena_top;
};

// thread 0's phase clock: ticks since the last mark into S->ph[k]
__device__ __forceinline__ void ph_mark(DpState *S, uint64_t &t, int k) {
    if (threadIdx.x == 0) {
        const uint64_t x = __builtin_amdgcn_s_memrealtime();
        S->ph[k] += x - t;
        t = x;
    }
}

// phase boundary inside the workgroup: its waves share the CU's L1, so a
// workgroup-scope release / acquire (waits, no cache maintenance) suffices
__device__ __forceinline__ void wg_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// flag(x) for x in [0, n) into bitmap words: each wave's 64 consecutive x are
// one ballot, two words written by its lane 0
template <class F>
__device__ __forceinline__ void inl_bits(uint32_t *words, int n, F &&flag) {
    const int tid = threadIdx.x, lane = lane_id(), wb = 64 * (tid >> 6);
    for (int x0 = 0; x0 < n; x0 += POP_THREADS) {
        const int x = x0 + tid;
        const bool b = x < n && flag(x);
        const uint64_t m = __ballot(b);
        if (lane == 0 && x0 + wb < n) {
            words[(x0 + wb) >> 5] = (uint32_t)m;
            words[((x0 + wb) >> 5) + 1] = (uint32_t)(m >> 32);
        }
    }
}

// the set (want = 1) or clear (want = 0) bits of words [0, n) in order:
// out[k] = val(x) of the k-th such x; returns their count (every thread)
template <class F>
__device__ __forceinline__ int inl_compact(const uint32_t *words, int n, int want, uint16_t *out, int *wsum, F &&val) {
    const int tid = threadIdx.x, nw = (n + 31) >> 5;
    uint32_t m = 0;
    if (tid < nw) {
        m = want ? words[tid] : ~words[tid];
        const int rest = n - 32 * tid;
        if (rest < 32) m &= (1u << rest) - 1u;
    }
    int total;
    int off = block_excl_scan(__popc(m), wsum, total);
    while (m) {
        const int b = __builtin_ctz(m);
        m &= m - 1u;
        out[off++] = (uint16_t)val(32 * tid + b);
    }
    wg_sync();
    return total;
}

__device__ __forceinline__ bool key_subset(const uint64_t *y, const uint64_t *x, int K) {
    uint64_t o = 0;
    for (int w = 0; w < K; ++w) o |= y[w] & ~x[w];
    return o == 0ull;
}

// L.flg bit x (x < nx) = some candidate y (y < ny; earlier = only y < x) is
// a subset of x's key.  The candidates' keys go through LDS in tiles and
// every lane reads the same tile
// entry at a time (a broadcast), x's key in registers (K <= INL_KMAX words);
// a tile loop ends once no x of the workgroup is still open.
constexpr int INL_KMAX = 8;
template <int KT, class FX, class FY>   // KT: key words known at compile time (0: Kr, up to INL_KMAX)
__device__ void inl_tests(InlLds &L, int nx, int ny, int Kr, bool earlier, FX &&xkey, FY &&ykey, uint32_t &tests) {
    constexpr int KR = KT ? KT : INL_KMAX;   // key words held in registers
    const int K = KT ? KT : Kr;
    const int tid = threadIdx.x;
    uint64_t *tile = L.tile;
    const int tcap = INL_TILE_WORDS / K;   // keys per tile
    for (int x0 = 0; x0 < nx; x0 += POP_THREADS) {
        const int x = x0 + tid;
        bool open = x < nx;
        bool hit = false;
        uint64_t xk[KR];
#pragma unroll
        for (int w = 0; w < KR; ++w) xk[w] = (open && w < K) ? xkey(x)[w] : ~0ull;
        // candidates that can matter to this chunk: all, or those before its last x
        const int yend = earlier ? min(ny, x0 + POP_THREADS) : ny;
        for (int y0 = 0; y0 < yend; y0 += tcap) {
            const int cnt = min(tcap, yend - y0);
            __syncthreads();   // the previous tile is no longer read
            for (int e = tid; e < cnt * K; e += POP_THREADS) tile[e] = ykey(y0 + e / K)[e % K];
            wg_sync();
            if (open) {
                const int lim = earlier ? min(cnt, x - y0) : cnt;
                int j = 0;
                for (; j < lim; ++j) {
                    uint64_t o = 0;
#pragma unroll
                    for (int w = 0; w < KR; ++w)
                        if (KT || w < K) o |= tile[j * K + w] & ~xk[w];
                    if (o == 0ull) {
                        hit = true;
                        ++j;
                        break;
                    }
                }
                tests += (uint32_t)max(j, 0);
                if (hit || (earlier && y0 + cnt >= x)) open = false;
            }
            if (!__syncthreads_or(open)) break;
        }
        const uint64_t m = __ballot(hit);
        const int wb = 64 * (tid >> 6);
        if (lane_id() == 0 && x0 + wb < nx) {
            L.flg[(x0 + wb) >> 5] = (uint32_t)m;
            L.flg[((x0 + wb) >> 5) + 1] = (uint32_t)(m >> 32);
        }
    }
    wg_sync();
}

// inl_tests with the key width as a constant for one-word-per-sign keys (<= 64
// variables: every configs[3] formula), else up to INL_KMAX words at run time
#define INL_TESTS_K(K, L_, NX, NY, EARLIER, FX, FY, T)                  \
    do {                                                                \
        if ((K) == 2) inl_tests<2>(L_, NX, NY, K, EARLIER, FX, FY, T);  \
        else inl_tests<0>(L_, NX, NY, K, EARLIER, FX, FY, T);           \
    } while (0)
constexpr int64_t INL_TESTS_MAX = 1 << 18;   // subset tests of a phase run inline (~2 per ns on one CU)

__device__ __forceinline__ uint64_t inl_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// One elimination step of the current split (g[cur], plist / nlist / rlist /
// rkeys), phases of dp_pairs .. dp_assemble in one workgroup.  Returns 1 when
// the solve ends here (an empty resolvent or the clause limit), 2 when the
// assembly of the next list is left to dp_assemble_kernel (S->skip = 2), else
// 0 with lfp (the first-position table in LDS, V <= FP_LDS) holding the next
// list's.
__device__ int dp_inline_step(const DpArgs &A, DpState *S, InlLds &L, int *wsum, unsigned long long *lfp, int cur,
                               int64_t np, int64_t nn, int64_t nr, int32_t var, int d, int capA, int capB, int capR,
                               uint64_t &tclk) {
    const int tid = threadIdx.x;
    const int K = A.K, W = A.W;
    const ClauseList CL = A.g[cur], O = A.g[cur ^ 1];
    const int P = (int)(np * nn);
    const uint64_t vb = 1ull << (d & 63);
    const int vw = d >> 6;
    if (tid == 0) L.fe = DP_EMPTY >> 32;
    wg_sync();
    // pairs (dp_pairs_kernel): resolvent keys, tautology / empty flags
    int ntc = 0;
    inl_bits(L.ntb, P, [&](int p) {
        const int i = p / (int)nn, j = p - i * (int)nn;
        const uint64_t *a = CL.bits + A.plist[i] * K, *b = CL.bits + A.nlist[j] * K;
        uint64_t *r = A.rbits + (uint64_t)p * K;
        bool taut = false, empty = true;
        for (int w = 0; w < W; ++w) {
            const uint64_t keep = w == vw ? ~vb : ~0ull;
            const uint64_t rp = (a[w] & keep) | b[w], rn = a[W + w] | (b[W + w] & keep);
            r[w] = rp;
            r[W + w] = rn;
            taut |= (rp & rn) != 0ull;
            empty &= (rp | rn) == 0ull;
        }
        if (empty) atomicMin(&L.fe, (uint32_t)p);
        ntc += (!taut && !empty) ? 1 : 0;
        return !taut && !empty;
    });
    const int nontaut = block_sum(ntc, wsum);
    wg_sync();
    ph_mark(S, tclk, 1);
    const uint32_t fe = L.fe;
    const auto nt = [&](int p) { return ((L.ntb[p >> 5] >> (p & 31)) & 1u) != 0u; };
    uint32_t tests = 0;   // (statistics; wraps past 2^32 per thread)
    int nuniq = 0, ns = 0, nkept = 0;
    if (fe == (uint32_t)(DP_EMPTY >> 32)) {
        // distinct resolvents (dp_hash_kernel): the smallest pair index per key
        for (int p = tid; p < P; p += POP_THREADS) {
            if (!nt(p)) continue;
            const uint64_t *x = A.rbits + (uint64_t)p * K;
            uint64_t h = 0x9E3779B97F4A7C15ull;
            for (int w = 0; w < K; ++w) h = inl_mix64(h ^ x[w]) + (uint64_t)w;
            uint64_t sl = h & A.tmask;
            for (;;) {
                uint64_t c = __hip_atomic_load(A.table + sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (c == DP_EMPTY) {
                    c = atomicCAS((unsigned long long *)(A.table + sl), (unsigned long long)DP_EMPTY,
                                  (unsigned long long)p);
                    if (c == DP_EMPTY) break;
                }
                if (key_subset(A.rbits + c * K, x, K) && key_subset(x, A.rbits + c * K, K)) {
                    if ((uint64_t)p < c) atomicMin((unsigned long long *)(A.table + sl), (unsigned long long)p);
                    break;
                }
                sl = (sl + 1) & A.tmask;
            }
            A.uslot[p] = (uint32_t)sl;
        }
        wg_sync();
        inl_bits(L.flg, P, [&](int p) {
            return nt(p) && __hip_atomic_load(A.table + A.uslot[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                                (uint64_t)p;
        });
        wg_sync();
        nuniq = inl_compact(L.flg, P, 1, L.ua, wsum, [](int p) { return p; });
        for (int k = tid; k < nuniq; k += POP_THREADS)   // the table clean for the next step
            __hip_atomic_store(A.table + A.uslot[L.ua[k]], DP_EMPTY, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ph_mark(S, tclk, 2);
        // rem test (dp_remtest_kernel): dropped when a remaining clause is a
        // subset.  One CU runs ~2 tests per ns: a step with many tests leaves
        // here (nothing it did matters to the pipeline, which redoes the step)
        if ((int64_t)nuniq * nr > INL_TESTS_MAX) return 3;
        const auto rx = [&](int u) { return A.rbits + (uint64_t)L.ua[u] * K; };
        const auto ry = [&](int j) { return A.rkeys + (uint64_t)j * K; };
        INL_TESTS_K(K, L, nuniq, (int)nr, false, rx, ry, tests);
        ns = inl_compact(L.flg, nuniq, 0, L.ub, wsum, [&](int u) { return (int)L.ua[u]; });
        if ((int64_t)ns * ns / 2 > INL_TESTS_MAX) return 3;
        ph_mark(S, tclk, 3);
        // survivor test (dp_survtest_kernel): hit by an earlier survivor (pair order)
        const auto sx = [&](int k) { return A.rbits + (uint64_t)L.ub[k] * K; };
        INL_TESTS_K(K, L, ns, ns, true, sx, sx, tests);
        ph_mark(S, tclk, 4);
    }
    // the verdict (dp_kept_kernel): the first empty resolvent or the clause
    // limit (the kth non-tautological non-empty pair), whichever comes first
    int64_t limit_pair = -1;
    const int64_t kth = max<int64_t>(A.clause_limit - nr, 0);
    if (A.clause_limit > 0 && nontaut > kth) {
        int c = tid < ((P + 31) >> 5) ? __popc(L.ntb[tid] & (P - 32 * tid < 32 ? (1u << (P - 32 * tid)) - 1u : ~0u))
                                        : 0;
        int tot;
        const int ex = block_excl_scan(c, wsum, tot);
        if (tid == 0) L.arena_top = -1;
        wg_sync();
        if (kth >= ex && kth < ex + c) {
            uint32_t m = L.ntb[tid];
            for (int64_t need = kth - ex; need > 0; --need) m &= m - 1u;
            L.arena_top = 32 * tid + __builtin_ctz(m);   // (borrowed: the limit pair)
        }
        wg_sync();
        limit_pair = L.arena_top;
        wg_sync();
    }
    const uint32_t ttests = (uint32_t)block_sum((int)tests, wsum);
    if (fe != (uint32_t)(DP_EMPTY >> 32) || limit_pair >= 0) {
        if (tid == 0) {
            S->nontaut = nontaut;
            S->tests += ttests;
            S->first_empty = fe == (uint32_t)(DP_EMPTY >> 32) ? DP_EMPTY : (uint64_t)fe;
            S->result = (fe != (uint32_t)(DP_EMPTY >> 32) && (limit_pair < 0 || (int64_t)fe < limit_pair)) ? 0 : -1;
            S->done = 1;
        }
        return 1;
    }
    nkept = inl_compact(L.flg, ns, 0, L.ua, wsum, [&](int k) { return (int)L.ub[k]; });
    const int64_t ncl2 = nr + nkept;
    ph_mark(S, tclk, 5);
    if (tid == 0) S->inl_steps += 1;
    // many kept resolvents: their images (a serial chain of CPython set
    // operations each) are built by the pipeline's assemble kernel across the
    // GPU, one wave each; a few are built here, one wave each in LDS
    const bool here = nkept <= INL_ASM_MAX && 2 * (capA + capB + capR) <= INL_ASM_SCRATCH;
    if (tid == 0) {
        const int64_t base = S->arena_top;
        L.arena_top = base;
        S->nontaut = nontaut;
        S->nuniq = nuniq;
        S->nsurv = ns;
        S->nkept = nkept;
        S->tests += ttests;
        S->ncl2 = ncl2;
        S->arena_base = base;
        S->arena_top = base + (int64_t)nkept * 2 * capR;
        S->new_total += nontaut;
        S->pending = 1;
        if (!here) S->skip = 2;   // the slot's kernels: only dp_assemble_kernel runs
    }
    if (!here) {
        for (int k = tid; k < nkept; k += POP_THREADS) A.klist[k] = L.ua[k];
        return 2;
    }
    for (int x = tid; x < A.V; x += POP_THREADS) lfp[x] = ~0ull;
    wg_sync();
    // the next clause list (dp_assemble_kernel): rem clauses, then the kept
    // resolvents' images built by lane 0 of a wave in its LDS scratch
    const int lane = lane_id(), wid = tid >> 6;
    const int64_t base = L.arena_top;
    for (int64_t t = tid; t < nr; t += POP_THREADS) {   // rem clauses: one per thread
        const int64_t c = A.rlist[t];
        const int64_t off = CL.off[c];
        const int32_t mask = CL.mask[c];
        O.off[t] = off;
        O.mask[t] = mask;
        O.fill[t] = CL.fill[c];
        O.used[t] = CL.used[c];
        for (int w = 0; w < K; ++w) O.bits[t * K + w] = CL.bits[c * K + w];
        const int32_t *img = A.arena + off;
        for (int32_t x = 0; x <= mask; ++x) {   // first positions (REF.py:128's comprehension order)
            const int32_t key = img[x];
            if (key == PY_EMPTY || key == PY_DUMMY) continue;
            atomicMin(&lfp[A.v2d[key < 0 ? -key : key]], ((unsigned long long)t << 32) | (unsigned long long)x);
        }
    }
    for (int64_t t = nr + wid; t < ncl2; t += POP_THREADS / 64) {   // kept resolvents: one per wave
        const int32_t *img;
        int64_t mask;
        {
            const int64_t k = t - nr;
            const uint32_t p = L.ua[k];
            int32_t *xa = (int32_t *)L.tile + wid * INL_ASM_SCRATCH;
            int32_t *xb = xa + 2 * capA;
            int32_t *ra = xb + 2 * capB;
            int32_t *dst = A.arena + base + k * 2 * capR;
            int64_t rm = 0, rf = 0, ru = 0, roff = 0;
            if (lane == 0) {
                const uint32_t i = p / (uint32_t)nn, j = p - i * (uint32_t)nn;
                DSet ax, by, r;
                dset_init(ax, xa, xa + capA, capA);
                py_difference1(ax, cl_view(CL, A.arena, A.plist[i]), var);    // pc - {var}
                dset_init(by, xb, xb + capB, capB);
                py_difference1(by, cl_view(CL, A.arena, A.nlist[j]), -var);   // nc - {-var}
                dset_init(r, ra, ra + capR, capR);
                py_merge(r, dset_view(ax));   // set_copy(AX)
                py_merge(r, dset_view(by));   // |= BY
                if (ax.overflow || by.overflow || r.overflow) S->set_ovf = 1;
                rm = r.mask;
                rf = r.fill;
                ru = r.used;
                roff = r.t - ra;
            }
            wave_sync();
            rm = __shfl(rm, 0);
            rf = __shfl(rf, 0);
            ru = __shfl(ru, 0);
            roff = __shfl(roff, 0);
            const int32_t *src = ra + roff;
            for (int64_t x = lane; x <= rm; x += 64) dst[x] = src[x];
            if (lane == 0) {
                O.off[t] = dst - A.arena;
                O.mask[t] = (int32_t)rm;
                O.fill[t] = (int32_t)rf;
                O.used[t] = (int32_t)ru;
            }
            if (lane < K) O.bits[t * K + lane] = A.rbits[(uint64_t)p * K + lane];
            img = src;
            mask = rm;
        }
        for (int64_t x = lane; x <= mask; x += 64) {   // first positions (REF.py:128's comprehension order)
            const int32_t key = img[x];
            if (key == PY_EMPTY || key == PY_DUMMY) continue;
            atomicMin(&lfp[A.v2d[key < 0 ? -key : key]], ((unsigned long long)t << 32) | (unsigned long long)x);
        }
        wave_sync();   // the wave's scratch is rewritten by its next clause
    }
    wg_sync();
    for (int x = tid; x < A.V; x += POP_THREADS)   // (the pipeline's next pop reads them from memory)
        if (lfp[x] != ~0ull) atomicMin(&A.firstpos[x], lfp[x]);
    ph_mark(S, tclk, 6);
    return 0;
}

// INL: the form with inline steps (opt-in, SATMI_DP_INLINE=1: measured slower
// than the pipeline); the default form has none of that code
// (its register budget is the pop / split's alone)
template <bool INL>
__global__ void __launch_bounds__(POP_THREADS) dp_pop_split_kernel(DpArgs A) {
    __shared__ unsigned long long fp_sh[FP_LDS];
    __shared__ int32_t ord_sh[FP_LDS];
    __shared__ int32_t pop_sh[2 * POP_LDS];
    __shared__ int wsum[48];
    __shared__ int64_t sh_ncl;
    __shared__ int sh_cur, sh_quit, sh_var;
    __shared__ std::conditional_t<INL, InlLds, char> inl;
    DpState *S = A.st;
    if (S->done) return;
    const int tid = threadIdx.x;
    const int V = A.V;
    const bool lds_fp = V <= FP_LDS;
    uint64_t tclk = __builtin_amdgcn_s_memrealtime();
    for (int it = 0;; ++it) {
    if (tid == 0) {
        if (S->pending) {   // the previous step's generation becomes the clause list
            S->cur ^= 1;
            S->ncl = S->ncl2;
            S->pending = 0;
        }
        if (it == 0) {
            S->skip = 0;
            S->slots += 1;
        }
        sh_cur = S->cur;
        sh_ncl = S->ncl;
        sh_quit = 0;
    }
    // (after an inline step its first-position table is already in fp_sh)
    if (lds_fp && it == 0)
        for (int d = tid; d < V; d += POP_THREADS) fp_sh[d] = A.firstpos[d];
    __syncthreads();
    // the variables that occur: their count and range
    int live = 0, vmax = 0, vlow = 0;   // vlow: INT32_MAX - the smallest
    for (int d = tid; d < V; d += POP_THREADS) {
        const unsigned long long f = lds_fp ? fp_sh[d] : A.firstpos[d];
        if (f == ~0ull) continue;
        ++live;
        const int32_t v = A.d2v[d];
        vmax = max(vmax, v);
        vlow = max(vlow, INT32_MAX - v);
    }
    block_sum_max_max(live, vmax, vlow, wsum);
    const int nv = live;
    const int32_t vmin = INT32_MAX - vlow;
    // every variable below the set's final table size: pop() is the smallest
    // (pyset_dev.h py_size_after); otherwise the set is built in insertion order
    const bool small_ints = nv > 0 && (int64_t)vmax < py_size_after(nv);
    if (!small_ints) {   // rank the variables by first position (positions are distinct)
        for (int d = tid; d < V; d += POP_THREADS) {
            const unsigned long long f = lds_fp ? fp_sh[d] : A.firstpos[d];
            if (f == ~0ull) continue;
            int rank = 0;
            for (int e = 0; e < V; ++e) rank += (lds_fp ? fp_sh[e] : A.firstpos[e]) < f ? 1 : 0;
            (lds_fp ? ord_sh : A.order)[rank] = A.d2v[d];
        }
        __syncthreads();
    }
    if (tid == 0) {
        int32_t popped = 0;
        if (nv == 0) {   // `while variables` ends: True (REF.py:130)
            S->result = 1;
            S->done = 1;
            sh_quit = 1;
        } else if (small_ints) {
            popped = vmin;
        } else {
            // the model set in LDS when it fits (a chain of dependent probes)
            DSet s;
            int32_t *ps = A.popcap <= POP_LDS ? pop_sh : A.popscratch;
            dset_init(s, ps, ps + A.popcap, A.popcap);
            const int32_t *ord = lds_fp ? ord_sh : A.order;
            for (int r = 0; r < nv; ++r) py_add(s, ord[r]);
            if (s.overflow) {
                S->set_ovf = 1;
                S->done = 1;
                sh_quit = 1;
            } else {
                for (int64_t i = 0; i <= s.mask; ++i)   // a fresh set's finger is 0: first live slot
                    if (s.t[i] != PY_EMPTY && s.t[i] != PY_DUMMY) {
                        popped = s.t[i];
                        break;
                    }
            }
        }
        if (!sh_quit && A.step_limit > 0 && S->steps >= A.step_limit) {
            S->result = -1;
            S->done = 1;
            sh_quit = 1;
        }
        if (!sh_quit && A.limit_ticks && __builtin_amdgcn_s_memrealtime() - S->t0 > A.limit_ticks) {
            S->result = -1;
            S->done = 1;
            sh_quit = 1;
        }
        sh_var = popped;
    }
    __syncthreads();
    if (sh_quit) return;
    const int32_t var = sh_var;
    const int d = A.v2d[var];
    const int W = A.W, K = A.K, dw = d >> 6, db = d & 63;
    const ClauseList L = A.g[sh_cur];
    const int64_t ncl = sh_ncl;
    // each thread a contiguous run of clauses: its flag loads are independent
    // (one memory latency), one block scan places every run
    int mxA = 0, mxB = 0;
    const int64_t per = (ncl + POP_THREADS - 1) / POP_THREADS;
    const int64_t c0 = min<int64_t>(ncl, tid * per), c1 = min<int64_t>(ncl, c0 + per);
    int cp = 0, cq = 0, cr = 0;
    uint32_t fl = 0;   // bit 2k: clause c0+k holds var, bit 2k+1: -var (runs of <= 16 clauses)
    const bool small = per <= 16;
    for (int64_t c = c0; c < c1; ++c) {
        const bool p = (L.bits[c * K + dw] >> db) & 1ull;
        const bool q = (L.bits[c * K + W + dw] >> db) & 1ull;
        const int u = L.used[c];   // (read with the flags: no second dependent load)
        if (small) fl |= (p ? 1u : 0u) << (2 * (c - c0)) | (q ? 2u : 0u) << (2 * (c - c0));
        cp += p;
        cq += q;
        cr += !p && !q;
        mxA = p ? max(mxA, u) : mxA;
        mxB = q ? max(mxB, u) : mxB;
    }
    int tot, tr, ep, en, er;
    int64_t np, nn;
    if (ncl < 65536) {   // pos and neg counts in one word (halves < 2^16), rem beside them: one exchange
        int ex = cp | (cq << 16);
        er = cr;
        block_excl_scan2(ex, er, wsum, tot, tr);
        ep = ex & 0xFFFF;
        en = ex >> 16;
        np = tot & 0xFFFF;
        nn = tot >> 16;
    } else {
        int tn;
        ep = block_excl_scan(cp, wsum, tot);
        en = block_excl_scan(cq, wsum, tn);
        er = block_excl_scan(cr, wsum, tr);
        np = tot;
        nn = tn;
    }
    const int64_t nr = tr;
    for (int64_t c = c0; c < c1; ++c) {   // a clause may be in both the pos and the neg list
        bool p, q;
        if (small) {
            p = (fl >> (2 * (c - c0))) & 1u;
            q = (fl >> (2 * (c - c0) + 1)) & 1u;
        } else {
            p = (L.bits[c * K + dw] >> db) & 1ull;
            q = (L.bits[c * K + W + dw] >> db) & 1ull;
        }
        if (p) A.plist[ep++] = c;
        if (q) A.nlist[en++] = c;
        if (!p && !q) {
            for (int w = 0; w < K; ++w) A.rkeys[er * K + w] = L.bits[c * K + w];
            A.rlist[er++] = c;
        }
    }
    {
        int zero = 0;
        block_sum_max_max(zero, mxA, mxB, wsum);
    }
    const int64_t npairs = np * nn;
    if (npairs > A.pair_cap) {   // grow the pair buffers and run this step again
        if (tid == 0) {
            S->need[0] = npairs;
            S->overflow |= OVF_PAIRS;
            S->done = 1;
        }
        return;
    }
    if (tid == 0) {
        if (S->steps < A.trace_cap) A.trace[S->steps] = var;
        S->steps += 1;
        S->var = var;
        S->d = d;
        S->np = np;
        S->nn = nn;
        S->nr = nr;
        S->npairs = npairs;
        S->mxA = mxA;
        S->mxB = mxB;
        S->capA = (int32_t)cap_for(mxA);
        S->capB = (int32_t)cap_for(mxB);
        S->capR = (int32_t)cap_for((int64_t)mxA + mxB);
        S->first_empty = DP_EMPTY;
        S->nontaut = 0;
        S->nuniq = 0;
        S->nsurv = 0;
        S->nkept = 0;
        S->epoch += 1;
    }
    for (int e = tid; e < V; e += POP_THREADS) A.firstpos[e] = ~0ull;   // for the next step's assembly
    if (tid < 3 * DP_STRIPES) A.stripes[tid] = 0ull;
    if constexpr (!INL) {
        (void)inl;
        (void)tclk;
        return;
    } else {
    // run this step here (Inline steps) if it fits the workgroup; else the
    // pipeline kernels queued behind this one run it
    const int capA = (int)cap_for(mxA), capB = (int)cap_for(mxB), capR = (int)cap_for((int64_t)mxA + mxB);
    if (tid == 0) {
        const bool fit = it < A.inline_steps && npairs <= INL_PMAX && lds_fp && K <= INL_KMAX &&
                         nr + npairs <= A.ncl_cap && S->arena_top + npairs * 2 * capR <= A.arena_cap;
        sh_quit = fit ? 0 : 1;
    }
    wg_sync();
    ph_mark(S, tclk, 0);
    if (sh_quit) return;
    if (dp_inline_step(A, S, inl, wsum, fp_sh, sh_cur, np, nn, nr, var, d, capA, capB, capR, tclk)) return;   // 1, 2
    wg_sync();
    if (it + 1 >= A.inline_steps) {   // (recording: one step per slot) the slot's pipeline kernels skip
        if (tid == 0) S->skip = 1;
        return;
    }
    }
    }
}

// pair p = i*nn + j: resolvent key, tautology (REF.py:115) and empty (REF.py:117)
// flags; rbits[p] for non-tautological pairs, ntbits bit p.
__global__ void __launch_bounds__(256) dp_pairs_kernel(DpArgs A) {
    __shared__ int wsum[4];
    DpState *S = A.st;
    // (the state fields loaded together before any test: one round trip, see dp_kept_kernel)
    const int done = S->done, skip = S->skip, cur = S->cur, d = S->d;
    const uint32_t npairs = (uint32_t)S->npairs, nn = (uint32_t)S->nn;
    DP_KEEP(cur);
    DP_KEEP(d);
    DP_KEEP(npairs);
    DP_KEEP(nn);
    if (done || skip) return;
    const int W = A.W, K = A.K;
    const ClauseList L = A.g[cur];
    const uint64_t vb = 1ull << (d & 63);
    const int vw = d >> 6, lane = lane_id();
    int cnt = 0;
    for (uint32_t p0 = blockIdx.x * 256u + (threadIdx.x & ~63u); p0 < npairs; p0 += gridDim.x * 256u) {
        const uint32_t p = p0 + lane;
        bool nt = false;
        if (p < npairs) {
            const uint32_t i = p / nn, j = p - i * nn;
            const uint64_t *a = L.bits + A.plist[i] * K, *b = L.bits + A.nlist[j] * K;
            uint64_t *r = A.rbits + (uint64_t)p * K;
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
            if (empty) atomicMin((unsigned long long *)&S->first_empty, (unsigned long long)p);
            nt = !taut && !empty;
        }
        const uint64_t m = __ballot(nt);
        if (lane == 0) A.ntbits[p0 >> 6] = m;
        cnt += lane == 0 ? __popcll(m) : 0;
    }
    const int tot = block_sum(cnt, wsum);
    if (threadIdx.x == 0 && tot) atomicAdd(A.stripes + DP_STRIPES + blockIdx.x % DP_STRIPES, (unsigned long long)tot);
}

__device__ __forceinline__ uint64_t dp_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// one representative per distinct resolvent key: the table slot holds the
// smallest pair index with that key (atomicMin); the slot of each key's first
// claim goes to uslot.
__global__ void __launch_bounds__(256) dp_hash_kernel(DpArgs A) {
    DpState *S = A.st;
    const int done = S->done, skip = S->skip;
    const uint64_t fe = S->first_empty;
    const uint32_t npairs = (uint32_t)S->npairs;
    DP_KEEP(npairs);
    if (done || skip || fe != DP_EMPTY) return;   // the step ends in an empty clause
    const int K = A.K, lane = lane_id();
    for (uint32_t p0 = blockIdx.x * 256u + (threadIdx.x & ~63u); p0 < npairs; p0 += gridDim.x * 256u) {
        const uint32_t p = p0 + lane;
        const bool nt = p < npairs && ((A.ntbits[p0 >> 6] >> lane) & 1ull);
        bool claimed = false;
        uint64_t slot = 0;
        if (nt) {
            const uint64_t *x = A.rbits + (uint64_t)p * K;
            uint64_t h = 0x9E3779B97F4A7C15ull;
            for (int w = 0; w < K; ++w) h = dp_mix64(h ^ x[w]) + (uint64_t)w;
            uint64_t s = h & A.tmask;
            for (;;) {
                uint64_t cur = __hip_atomic_load(A.table + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (cur == DP_EMPTY) {
                    cur = atomicCAS((unsigned long long *)(A.table + s), (unsigned long long)DP_EMPTY,
                                    (unsigned long long)p);
                    if (cur == DP_EMPTY) {
                        claimed = true;
                        slot = s;
                        break;
                    }
                }
                const uint64_t *y = A.rbits + cur * K;
                bool eq = true;
                for (int w = 0; w < K; ++w) eq &= y[w] == x[w];
                if (eq) {
                    if (p < cur) atomicMin((unsigned long long *)(A.table + s), (unsigned long long)p);
                    break;
                }
                s = (s + 1) & A.tmask;
            }
        }
        const uint64_t bal = __ballot(claimed);
        if (bal) {   // the slot into this block's stripe region (rep_slot reads the regions in order)
            const int st = blockIdx.x % DP_STRIPES;
            uint32_t base = 0;
            if (lane == 0) base = (uint32_t)atomicAdd(A.stripes + st, (unsigned long long)__popcll(bal));
            base = uniform_u32(base);
            if (claimed) A.ustage[(uint64_t)st * A.pair_cap + base + __popcll(bal & lanemask_lt())] = (uint32_t)slot;
        }
    }
}

// Subset tests "y is a subset of x" with x (the tested clause) in registers
// and the candidate keys y staged 256 at a time in LDS from a contiguous copy
// (every lane reads the same address: a broadcast); four tests per step of
// the candidate loop, so four LDS reads are in flight before the branch.  KT =
// key words (2W) known at compile time, 0 = any width (keys read from memory).
template <int KT>
struct KeyReg {
    uint64_t w[KT ? KT : 1];
};

constexpr int TEST_TILE = 256;
#ifndef DP_TEST_STEP
#define DP_TEST_STEP 16   // candidates per step of the test loop (a multiple of 4 dividing TEST_TILE)
#endif
static_assert(DP_TEST_STEP % 4 == 0 && TEST_TILE % DP_TEST_STEP == 0, "DP_TEST_STEP");

template <int KT>
__device__ __forceinline__ bool subset_of(const uint64_t *y, const KeyReg<KT> &x, const uint64_t *xg, int K) {
    uint64_t out = 0;
    if constexpr (KT > 0) {
#pragma unroll
        for (int w = 0; w < KT; ++w) out |= y[w] & ~x.w[w];
    } else {
        for (int w = 0; w < K; ++w) out |= y[w] & ~xg[w];
    }
    return out == 0ull;
}

// Items = (x tile of 256 tested clauses) x (y tile of 256 candidates); block b
// takes items b, b + gridDim.x, ...  Lane l of an item tests x = tile x, lane
// l against the candidates of tile y with cand_ok(j) (all rem clauses; the
// survivors earlier in pair order), marking stamp[x] = epoch at the first
// subset; a lane whose x another block already marked stops.
template <int KT, bool SURV, class XK>
__device__ __forceinline__ void dp_test_items(const DpArgs &A, int64_t nx, int64_t ny, XK &&xkey,
                                              const uint64_t *ykeys, const uint32_t *ypair, int32_t *stamp,
                                              int32_t epoch, int &tests) {
    __shared__ __attribute__((aligned(16))) uint64_t tile[TEST_TILE * (KT ? KT : 1)];
    __shared__ __attribute__((aligned(16))) uint32_t tp[TEST_TILE];
    const int K = A.K, tid = threadIdx.x;
    const int64_t ntx = (nx + TEST_TILE - 1) / TEST_TILE, nty = (ny + TEST_TILE - 1) / TEST_TILE;
    for (int64_t item = blockIdx.x; item < ntx * nty; item += gridDim.x) {
        const int64_t tx = item % ntx, ty = item / ntx;
        const int64_t u = tx * TEST_TILE + tid;
        const bool valid = u < nx;
        const uint64_t *xg = xkey(valid ? u : 0);   // x's key words
        KeyReg<KT> x;
        if constexpr (KT > 0) {
#pragma unroll
            for (int w = 0; w < KT; ++w) x.w[w] = valid ? xg[w] : ~0ull;
        }
        const uint32_t px = SURV && valid ? ypair[u] : 0u;
        bool alive = valid && __hip_atomic_load(stamp + u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch;
        const int64_t e0 = ty * TEST_TILE;
        const int cnt = (int)min<int64_t>(TEST_TILE, ny - e0);
        if (__syncthreads_or(alive)) {
            if (tid < cnt) {
                if constexpr (KT > 0) {
#pragma unroll
                    for (int w = 0; w < KT; ++w) tile[tid * KT + w] = ykeys[(e0 + tid) * KT + w];
                }
                if (SURV) tp[tid] = ypair[e0 + tid];
            }
            __syncthreads();
            if (alive && KT > 0) {
                // DP_TEST_STEP candidates per step, every LDS read of the step
                // issued before any test (their pair indices as 16-B reads): the
                // tests are branch-free, so no read waits on an earlier read's
                // value (a short-circuit form made each step of four a chain of
                // 8 dependent LDS round trips)
                constexpr int KW = KT ? KT : 1, NC = DP_TEST_STEP;
                int j = 0;
                for (; j < cnt; j += NC) {
                    uint32_t tq[NC];
#pragma unroll
                    for (int q = 0; q < NC; ++q) tq[q] = 0u;
                    if constexpr (SURV) {
#pragma unroll
                        for (int q = 0; q < NC; q += 4) {
                            const uint4 t4 = *reinterpret_cast<const uint4 *>(tp + j + q);
                            tq[q] = t4.x;
                            tq[q + 1] = t4.y;
                            tq[q + 2] = t4.z;
                            tq[q + 3] = t4.w;
                        }
                    }
                    uint64_t y[NC][KW];
#pragma unroll
                    for (int q = 0; q < NC; ++q)
#pragma unroll
                        for (int w = 0; w < KW; ++w) y[q][w] = tile[(j + q) * KW + w];
                    // (the reads stay above the tests: the scheduler would otherwise
                    // sink each one to its test and reuse one register set)
                    __builtin_amdgcn_sched_barrier(0);
                    bool hit = false;
#pragma unroll
                    for (int q = 0; q < NC; ++q) {
                        uint64_t out = 0;
#pragma unroll
                        for (int w = 0; w < KW; ++w) out |= y[q][w] & ~x.w[w];
                        const bool okq = (j + q < cnt) & (!SURV | (tq[q] < px));
                        hit |= okq & (out == 0ull);
                    }
                    if (hit) {
                        __hip_atomic_store(stamp + u, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        j += NC;
                        break;
                    }
                }
                tests += min(j, cnt);
            } else if (alive) {   // key width known only at run time: keys read from memory
                const auto yk = [&](int j) { return KT ? tile + j * (KT ? KT : 1) : ykeys + (e0 + j) * K; };
                const auto ok = [&](int j) { return j < cnt && (!SURV || tp[j] < px); };
                int j = 0;
                for (; j < cnt; j += 4) {
                    const bool s0 = ok(j) && subset_of<KT>(yk(j), x, xg, K);
                    const bool s1 = ok(j + 1) && subset_of<KT>(yk(j + 1), x, xg, K);
                    const bool s2 = ok(j + 2) && subset_of<KT>(yk(j + 2), x, xg, K);
                    const bool s3 = ok(j + 3) && subset_of<KT>(yk(j + 3), x, xg, K);
                    if (s0 | s1 | s2 | s3) {
                        __hip_atomic_store(stamp + u, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        j += 4;
                        break;
                    }
                }
                tests += min(j, cnt);
            }
        }
        __syncthreads();   // the tile is rewritten by the next item
    }
}

// The distinct representatives are the hash kernel's claims, in stripe
// regions (ustage: stripe st holds stripes[st] table slots).  Representative u
// is slot t = u - pre[st] of the stripe st with pre[st] <= u < pre[st + 1];
// remtest and survlist read them there (no packing launch between them).
// pre: DP_STRIPES + 1 prefix sums in LDS, filled by every thread calling this.
__device__ __forceinline__ int64_t rep_prefix(const DpArgs &A, int64_t *pre) {
    if (threadIdx.x == 0) {
        int64_t acc = 0;
        for (int t = 0; t < DP_STRIPES; ++t) {
            pre[t] = acc;
            acc += (int64_t)A.stripes[t];
        }
        pre[DP_STRIPES] = acc;
    }
    __syncthreads();
    return pre[DP_STRIPES];
}
// the table slot of representative u (u < pre[DP_STRIPES])
__device__ __forceinline__ uint32_t rep_slot(const DpArgs &A, const int64_t *pre, int64_t u) {
    int lo = 0;   // the last stripe whose region starts at or before u
#pragma unroll
    for (int half = DP_STRIPES / 2; half >= 1; half >>= 1)
        lo = pre[lo + half] <= u ? lo + half : lo;
    return A.ustage[(uint64_t)lo * A.pair_cap + (uint64_t)(u - pre[lo])];
}

// every representative against the remaining clauses (REF.py:124, remaining
// part); a representative's key is read through its table slot (x side)
template <int KT>
__global__ void __launch_bounds__(TEST_TILE) dp_remtest_kernel(DpArgs A) {
    __shared__ int wsum[4];
    __shared__ int64_t pre[DP_STRIPES + 1];
    DpState *S = A.st;
    const int done = S->done, skip = S->skip;
    const uint64_t fe = S->first_empty;
    const int64_t nr = S->nr;
    const int32_t epoch = S->epoch;
    DP_KEEP(nr);
    DP_KEEP(epoch);
    if (done || skip || fe != DP_EMPTY) return;
    const int64_t nuniq = rep_prefix(A, pre);
    if (blockIdx.x == 0 && threadIdx.x == 0) S->nuniq = nuniq;
    const int K = A.K;
    int tests = 0;
    dp_test_items<KT, false>(
        A, nuniq, nr, [&](int64_t u) { return A.rbits + A.table[rep_slot(A, pre, u)] * (uint64_t)K; }, A.rkeys,
        nullptr, A.dropped, epoch, tests);
    const int tot = block_sum(tests, wsum);
    if (threadIdx.x == 0 && tot) atomicAdd(A.stripes + 2 * DP_STRIPES + blockIdx.x % DP_STRIPES, (unsigned long long)tot);
}

// the representatives no rem clause subsumes (pair index + key, contiguous);
// every used table slot cleared for the next step
__global__ void __launch_bounds__(256) dp_survlist_kernel(DpArgs A) {
    __shared__ int64_t pre[DP_STRIPES + 1];
    DpState *S = A.st;
    const int done = S->done, skip = S->skip;
    const uint64_t fe = S->first_empty;
    const int32_t epoch = S->epoch;
    DP_KEEP(epoch);
    if (done || skip || fe != DP_EMPTY) return;
    const int64_t nuniq = rep_prefix(A, pre);
    const int lane = lane_id(), K = A.K, tid = threadIdx.x;
    __shared__ int wcnt[4];
    __shared__ uint32_t bbase;
    // one block round: 256 representatives; the block's survivors take ONE
    // append atomic (a hot counter serialises)
    for (int64_t b0 = (int64_t)blockIdx.x * 256; b0 < nuniq; b0 += (int64_t)gridDim.x * 256) {   // block-uniform
        const int64_t u = b0 + tid;
        bool keep = false;
        uint32_t p = 0;
        if (u < nuniq) {
            const uint32_t s = rep_slot(A, pre, u);
            p = (uint32_t)A.table[s];
            A.table[s] = DP_EMPTY;
            keep = A.dropped[u] != epoch;
        }
        const uint64_t bal = __ballot(keep);
        if (lane == 0) wcnt[tid >> 6] = __popcll(bal);
        __syncthreads();
        const int nb = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
        if (tid == 0 && nb) bbase = (uint32_t)atomicAdd((unsigned long long *)&S->nsurv, (unsigned long long)nb);
        __syncthreads();
        if (keep) {
            uint32_t at = bbase + __popcll(bal & lanemask_lt());
            for (int w = 0; w < (tid >> 6); ++w) at += wcnt[w];
            A.surv[at] = p;
            for (int w = 0; w < K; ++w) A.skeys[(uint64_t)at * K + w] = A.rbits[(uint64_t)p * K + w];
        }
        __syncthreads();
    }
}

// every survivor x against the survivors y earlier in pair order (REF.py:124,
// unique_new part): hit[x] = epoch when some y is a subset of x
template <int KT>
__global__ void __launch_bounds__(TEST_TILE) dp_survtest_kernel(DpArgs A) {
    __shared__ int wsum[4];
    DpState *S = A.st;
    const int done = S->done, skip = S->skip;
    const uint64_t fe = S->first_empty;
    const int64_t nsurv = S->nsurv;
    const int32_t epoch = S->epoch;
    DP_KEEP(nsurv);
    DP_KEEP(epoch);
    if (done || skip || fe != DP_EMPTY) return;
    int tests = 0;
    const int K = A.K;
    dp_test_items<KT, true>(
        A, nsurv, nsurv, [&](int64_t u) { return A.skeys + u * K; }, A.skeys, A.surv, A.hit, epoch, tests);
    const int tot = block_sum(tests, wsum);
    if (threadIdx.x == 0 && tot) atomicAdd(A.stripes + 2 * DP_STRIPES + blockIdx.x % DP_STRIPES, (unsigned long long)tot);
}

// One workgroup: the step's verdict (the first empty resolvent, or the clause
// limit, whichever comes first in pair order -- REF.py:117-118), else the kept
// survivors in pair order and the capacities of the next generation.
__global__ void __launch_bounds__(POP_THREADS) dp_kept_kernel(DpArgs A) {
    __shared__ int wsum[16];
    __shared__ int64_t sh_lim;
    DpState *S = A.st;
    if (S->done || S->skip) return;
    const int tid = threadIdx.x;
    const uint64_t fe = S->first_empty;
    // every state field this kernel reads, up front: one round trip, not one
    // per phase (a barrier keeps a later load from being hoisted above it);
    // none of them is written here before it is read
    const int64_t npairs = S->npairs, nr = S->nr, ns = S->nsurv;
    const int32_t epoch = S->epoch;
    const int64_t capA = S->capA, capB = S->capB, capR = S->capR, arena_top = S->arena_top;
    __shared__ int64_t sh_nt;
    if (tid < 64) {   // the striped counters of this step (one wave)
        int64_t nt = (int64_t)A.stripes[DP_STRIPES + tid], ts = (int64_t)A.stripes[2 * DP_STRIPES + tid];
        for (int o = 32; o >= 1; o >>= 1) {
            nt += __shfl_xor(nt, o);
            ts += __shfl_xor(ts, o);
        }
        if (tid == 0) {
            sh_nt = nt;
            S->nontaut = nt;
            S->tests += ts;
        }
    }
    __syncthreads();
    const int64_t nontaut = sh_nt;
    // clause_limit: the reference stops when remaining + new passes the limit,
    // i.e. at the kth non-tautological non-empty pair (0-based)
    int64_t limit_pair = -1;
    const int64_t kth = max<int64_t>(A.clause_limit - nr, 0);
    if (A.clause_limit > 0 && nontaut > kth) {
        if (tid == 0) sh_lim = -1;
        const int64_t nw = (npairs + 63) >> 6;
        const int64_t per = (nw + POP_THREADS - 1) / POP_THREADS;
        const int64_t w0 = min<int64_t>(nw, tid * per), w1 = min<int64_t>(nw, w0 + per);
        int c = 0;
        for (int64_t w = w0; w < w1; ++w) c += __popcll(A.ntbits[w]);
        int tot;
        int ex = block_excl_scan(c, wsum, tot);
        if (kth >= ex && kth < ex + c) {   // this thread's words hold the kth bit
            int64_t need = kth - ex;
            for (int64_t w = w0; w < w1; ++w) {
                uint64_t m = A.ntbits[w];
                const int pc = __popcll(m);
                if (need < pc) {
                    for (; need > 0; --need) m &= m - 1;
                    sh_lim = w * 64 + __builtin_ctzll(m);
                    break;
                }
                need -= pc;
            }
        }
        __syncthreads();
        limit_pair = sh_lim;
    }
    if (fe != DP_EMPTY || limit_pair >= 0) {
        if (tid == 0) {
            S->result = (fe != DP_EMPTY && (limit_pair < 0 || (int64_t)fe < limit_pair)) ? 0 : -1;
            S->done = 1;
        }
        return;
    }
    int kc = 0;
    for (int64_t i = tid; i < ns; i += POP_THREADS) kc += A.hit[i] != epoch ? 1 : 0;
    const int nkept = block_sum(kc, wsum);
    const int64_t ncl2 = nr + nkept;
    const int64_t arena_need = arena_top + (int64_t)nkept * 2 * capR;
    const int64_t xs_need = (int64_t)nkept * 2 * (capA + capB);
    int ovf = 0;
    if (ncl2 > A.ncl_cap) ovf |= OVF_NCL;
    if (arena_need > A.arena_cap) ovf |= OVF_ARENA;
    if (xs_need > A.xs_cap) ovf |= OVF_XS;
    if (ovf) {   // grow and run this step again (its input generation is untouched)
        if (tid == 0) {
            S->need[1] = ncl2;
            S->need[2] = arena_need;
            S->need[3] = xs_need;
            S->overflow |= ovf;
            S->steps -= 1;
            S->done = 1;
        }
        return;
    }
    for (int64_t i = tid; i < ns; i += POP_THREADS)
        if (A.hit[i] != epoch) {
            const uint32_t p = A.surv[i];
            atomicOr(A.keptbits + (p >> 5), 1u << (p & 31));
        }
    __syncthreads();
    // ordered compaction of the kept bitmap (words cleared as read)
    const int64_t nw = (npairs + 31) >> 5;
    const int64_t per = (nw + POP_THREADS - 1) / POP_THREADS;
    const int64_t w0 = min<int64_t>(nw, tid * per), w1 = min<int64_t>(nw, w0 + per);
    int c = 0;
    for (int64_t w = w0; w < w1; ++w)
        c += __popc(__hip_atomic_load(A.keptbits + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    int tot;
    int pos = block_excl_scan(c, wsum, tot);
    for (int64_t w = w0; w < w1; ++w) {
        uint32_t m = __hip_atomic_load(A.keptbits + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!m) continue;
        A.keptbits[w] = 0u;
        while (m) {
            A.klist[pos++] = (uint32_t)(w * 32 + __builtin_ctz(m));
            m &= m - 1;
        }
    }
    if (tid == 0) {
        S->nkept = nkept;
        S->ncl2 = ncl2;
        S->arena_base = arena_top;
        S->arena_top = arena_need;
        S->new_total += nontaut;
        S->pending = 1;
    }
}

// clauses = remaining_clauses + unique_new (REF.py:127): one wavefront per
// clause of the next list.  A rem clause keeps its image; kept resolvent k =
// pair (i, j) gets the image of (pc - {var}) | (nc - {-var}) (REF.py:114),
// built by lane 0 -- CPython's insertions are a serial chain of dependent
// probes -- then copied to the arena at arena_base + 2*capR*k by the whole
// wave.  When the step's capacities fit the wave's LDS scratch, the chain runs
// on LDS only: the wave first copies pc's and nc's images there (one parallel
// read each), so every probe of the chain is an LDS round trip, not an L2 one;
// else the tables are built in HBM scratch.  (A form running the chain on
// tables held across the wave's registers, a probe a readlane, measured 2x
// slower: the inlined chains left the kernel SGPR-starved.)  The lanes then
// read the clause's table slots at once for the next step's first positions.
#ifndef DP_ASM_WAVE
#define DP_ASM_WAVE 1   // the chain run by the whole wave (0: by lane 0, the r06 form before)
#endif
#ifndef DP_ASM_SCRATCH
#define DP_ASM_SCRATCH 2048
#endif
constexpr int ASM_WAVES = 4, ASM_SCRATCH = DP_ASM_SCRATCH;   // per wave: int32 slots of AX, BY, R and the two sources

// lane 0's chain: ax = a - {var}, by = b - {-var}, r = ax | by, tables at xa /
// xb / ra (2*cap slots each: the table and its resize spare)
__device__ __forceinline__ void asm_build(const DView &a, const DView &b, int32_t var, int32_t *xa, int32_t *xb,
                                          int32_t *ra, int64_t capA, int64_t capB, int64_t capR, DpState *S,
                                          int64_t &rm, int64_t &rf, int64_t &ru, int64_t &roff) {
    DSet ax, by, r;
    dset_init(ax, xa, xa + capA, capA);
    py_difference1(ax, a, var);    // pc - {var}
    dset_init(by, xb, xb + capB, capB);
    py_difference1(by, b, -var);   // nc - {-var}
    dset_init(r, ra, ra + capR, capR);
    py_merge(r, dset_view(ax));   // set_copy(AX)
    py_merge(r, dset_view(by));   // |= BY
    if (ax.overflow || by.overflow || r.overflow) S->set_ovf = 1;
    rm = r.mask;
    rf = r.fill;
    ru = r.used;
    roff = r.t - ra;
}

// the same chain run by the whole wave (pyset_dev.h wpy_*: a probe run per
// LDS round trip, scans and copies across the lanes), every table in LDS
__device__ __forceinline__ void asm_build_wave(const DView &a, const DView &b, int32_t var, int32_t *xa, int32_t *xb,
                                               int32_t *ra, int64_t capA, int64_t capB, int64_t capR, DpState *S,
                                               int64_t &rm, int64_t &rf, int64_t &ru, int64_t &roff) {
    DSet ax, by, r;
    wdset_init(ax, xa, xa + capA, capA);
    wpy_difference1(ax, a, var);    // pc - {var}
    wdset_init(by, xb, xb + capB, capB);
    wpy_difference1(by, b, -var);   // nc - {-var}
    wdset_init(r, ra, ra + capR, capR);
    wpy_merge(r, dset_view(ax));   // set_copy(AX)
    wpy_merge(r, dset_view(by));   // |= BY
    if (__lane_id() == 0 && (ax.overflow || by.overflow || r.overflow)) S->set_ovf = 1;
    rm = r.mask;
    rf = r.fill;
    ru = r.used;
    roff = r.t - ra;
}

__global__ void __launch_bounds__(64 * ASM_WAVES) dp_assemble_kernel(DpArgs A) {
    __shared__ unsigned long long lfp_sh[FP_LDS];
    __shared__ int32_t scratch_sh[ASM_WAVES][ASM_SCRATCH];
    DpState *S = A.st;
    const int done = S->done, skip = S->skip, cur = S->cur;
    const int64_t ncl2 = S->ncl2, nr = S->nr, nn = S->nn, base = S->arena_base;
    const int64_t capA = S->capA, capB = S->capB, capR = S->capR;
    const int32_t var = S->var;
    DP_KEEP(cur);
    DP_KEEP(ncl2);
    DP_KEEP(nr);
    DP_KEEP(nn);
    DP_KEEP(base);
    DP_KEEP(capA);
    DP_KEEP(capB);
    DP_KEEP(capR);
    DP_KEEP(var);
    if (done) return;
    if (skip == 1) return;   // (2: an inline step left this kernel its assembly)
    unsigned long long *lfp = lfp_sh;   // used when A.V <= FP_LDS (an LDS pointer: ds_* atomics)
    firstpos_begin(A, lfp);
    const ClauseList L = A.g[cur], O = A.g[cur ^ 1];
    const int K = A.K, lane = lane_id(), wid = threadIdx.x >> 6;
    const int64_t tab = 2 * (capA + capB + capR);   // the three tables' slots
    const bool lds_ok = tab <= ASM_SCRATCH;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    // (t is wave-uniform: one clause per wavefront)
    const int64_t t0 = __builtin_amdgcn_readfirstlane((int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6));
    for (int64_t t = t0; t < ncl2; t += nwaves) {
        // first positions (REF.py:128's comprehension order) of clause t's
        // table, called where the table's address space is known
        const auto first_positions = [&](const int32_t *img, int64_t mask) {
            for (int64_t x = lane; x <= mask; x += 64) {
                const int32_t key = img[x];
                if (key == PY_EMPTY || key == PY_DUMMY) continue;
                const int d = A.v2d[key < 0 ? -key : key];
                const unsigned long long pos = ((unsigned long long)t << 32) | (unsigned long long)x;
                if (A.V <= FP_LDS)
                    atomicMin(&lfp[d], pos);
                else
                    atomicMin(&A.firstpos[d], pos);
            }
        };
        if (t < nr) {
            const int64_t c = A.rlist[t];
            const int64_t mask = L.mask[c];
            if (lane == 0) {
                O.off[t] = L.off[c];
                O.mask[t] = (int32_t)mask;
                O.fill[t] = L.fill[c];
                O.used[t] = L.used[c];
            }
            if (lane < K) O.bits[t * K + lane] = L.bits[c * K + lane];
            first_positions(A.arena + L.off[c], mask);
        } else {
            const int64_t k = t - nr;
            const uint32_t p = A.klist[k];
            const uint32_t i = p / (uint32_t)nn, j = p - i * (uint32_t)nn;
            const DView va = cl_view(L, A.arena, A.plist[i]), vb = cl_view(L, A.arena, A.nlist[j]);
            int32_t *dst = A.arena + base + k * 2 * capR;
            int64_t rm = 0, rf = 0, ru = 0, roff = 0;
            int32_t *out;
            if (lds_ok) {
                int32_t *xa = scratch_sh[wid], *xb = xa + 2 * capA, *ra = xb + 2 * capB;
                if (tab + va.mask + vb.mask + 2 <= ASM_SCRATCH) {   // the sources too: an LDS-only chain
                    int32_t *ca = scratch_sh[wid] + tab, *cb = ca + va.mask + 1;
                    for (int64_t x = lane; x <= va.mask; x += 64) ca[x] = va.t[x];
                    for (int64_t x = lane; x <= vb.mask; x += 64) cb[x] = vb.t[x];
                    wave_sync();
#if DP_ASM_WAVE
                    asm_build_wave({ca, va.mask, va.fill, va.used}, {cb, vb.mask, vb.fill, vb.used}, var, xa, xb, ra,
                                   capA, capB, capR, S, rm, rf, ru, roff);
#else
                    if (lane == 0)
                        asm_build({ca, va.mask, va.fill, va.used}, {cb, vb.mask, vb.fill, vb.used}, var, xa, xb, ra,
                                  capA, capB, capR, S, rm, rf, ru, roff);
#endif
                } else if (lane == 0) {
                    asm_build(va, vb, var, xa, xb, ra, capA, capB, capR, S, rm, rf, ru, roff);
                }
                wave_sync();
                rm = __shfl(rm, 0);
                rf = __shfl(rf, 0);
                ru = __shfl(ru, 0);
                roff = __shfl(roff, 0);
                const int32_t *src = ra + roff;
                for (int64_t x = lane; x <= rm; x += 64) dst[x] = src[x];
                out = dst;
                first_positions(src, rm);
            } else {
                int32_t *xa = A.xs + k * 2 * (capA + capB), *xb = xa + 2 * capA;
                if (lane == 0) asm_build(va, vb, var, xa, xb, dst, capA, capB, capR, S, rm, rf, ru, roff);
                wave_sync();
                rm = __shfl(rm, 0);
                rf = __shfl(rf, 0);
                ru = __shfl(ru, 0);
                roff = __shfl(roff, 0);
                out = dst + roff;
                first_positions(out, rm);
            }
            if (lane == 0) {
                O.off[t] = out - A.arena;
                O.mask[t] = (int32_t)rm;
                O.fill[t] = (int32_t)rf;
                O.used[t] = (int32_t)ru;
            }
            if (lane < K) O.bits[t * K + lane] = A.rbits[(uint64_t)p * K + lane];
        }
        wave_sync();   // the wave's scratch is rewritten by its next clause
    }
    firstpos_flush(A, lfp);
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
    // grow to >= bytes; keep the first `keep` bytes (stream-ordered copy); `fill`
    // (>= 0) initialises the whole new buffer first
    int need(size_t bytes, hipStream_t s = nullptr, size_t keep = 0, int fill = -1) {
        if (bytes <= cap) return SATMI_OK;
        const size_t want = std::max<size_t>(bytes + bytes / 2, 256);
        void *np = nullptr;
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && want > free_b) {
            set_error("satmi_dp_host: out of device memory (" + std::to_string(want >> 20) + " MiB wanted, " +
                      std::to_string(free_b >> 20) + " MiB free); bound the elimination with clause_limit");
            return SATMI_ERR_NOMEM;
        }
        SATMI_HIP(hipMalloc(&np, want));
        if (fill >= 0) SATMI_HIP(hipMemsetAsync(np, fill, want, s));
        if (p && keep) SATMI_HIP(hipMemcpyAsync(np, p, std::min(keep, cap), hipMemcpyDeviceToDevice, s));
        if (p) {
            SATMI_HIP(hipStreamSynchronize(s));   // the old buffer is no longer read
            (void)hipFree(p);
        }
        p = np;
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

struct Gen {   // one generation's per-clause arrays
    Buf off, mask, fill, used, bits;
    int reserve(int64_t n, int K, hipStream_t s, int64_t keep_n) {
        n = std::max<int64_t>(n, 1);
        DP_TRY(off.need(8 * (size_t)n, s, 8 * (size_t)keep_n));
        DP_TRY(mask.need(4 * (size_t)n, s, 4 * (size_t)keep_n));
        DP_TRY(fill.need(4 * (size_t)n, s, 4 * (size_t)keep_n));
        DP_TRY(used.need(4 * (size_t)n, s, 4 * (size_t)keep_n));
        DP_TRY(bits.need(8 * (size_t)n * K, s, 8 * (size_t)keep_n * K));
        return SATMI_OK;
    }
    ClauseList view() const {
        return {off.as<int64_t>(), mask.as<int32_t>(), fill.as<int32_t>(), used.as<int32_t>(), bits.as<uint64_t>()};
    }
};

// Work and device time of the last satmi_dp_host call, for bench.py's roofline.
struct DpStats {
    int64_t steps = 0, tests = 0, new_clauses = 0, launches = 0;
    double device_ms = 0.0;
    int words = 0;
};
thread_local DpStats g_dp_stats;   // the calling thread's last call

// The captured step batch of a workspace (see satmi_dp_host).
struct DpGraph {
    hipGraphExec_t exec = nullptr;
    DpArgs args;
    int batch = 0;
    DpGraph() { std::memset(&args, 0, sizeof(args)); }
    void reset() {
        if (exec) (void)hipGraphExecDestroy(exec);
        exec = nullptr;
        batch = 0;
    }
};

// Device buffers of one solve, kept between calls (grow-only) in a process-wide
// pool: a call takes a free workspace (or makes one) and returns it when done,
// so concurrent calls from any number of threads each own one and the number
// of workspaces is the peak number of concurrent calls.
struct DpWork {
    Buf d_off, d_lits, d_v2d, d_d2v, state, firstpos, order, popscratch, trace;
    Buf plist, nlist, rlist, rbits, ntbits, table, uslot, dropped, hit, surv, klist, keptbits, xs, arena;
    Buf rkeys, skeys, ustage, stripes;
    Gen g[2];
    int64_t ncl_cap = 0, pair_cap = 0, arena_cap = 0, xs_cap = 0;
    uint64_t tslots = 0;
    int K = 0;
    int32_t epoch = 0;
    DpArgs hint_args;             // the last completed call's arguments and step slots used
    int hint_slots = 0;
    std::vector<hipEvent_t> ev;   // filter timing: one pair per step, read once per call
    hipStream_t stream = nullptr;
    DpState *pin = nullptr;       // pinned host copy of the state
    int dev = 0;
    DpGraph graph;
    ~DpWork() {   // only a workspace that failed mid-call (or a trim) destroys one, after its stream drained
        graph.reset();
        for (hipEvent_t e : ev) (void)hipEventDestroy(e);
        if (stream) (void)hipStreamDestroy(stream);
        if (pin) (void)hipHostFree(pin);
    }
};

struct DpPool {
    std::mutex mu;
    std::vector<DpWork *> free_list;
};
DpPool &dp_pool() {
    static DpPool *p = new DpPool;   // never destroyed: no hipFree after the runtime's teardown
    return *p;
}
DpWork *dp_acquire(int dev) {
    DpPool &P = dp_pool();
    {
        std::lock_guard<std::mutex> g(P.mu);
        for (size_t i = 0; i < P.free_list.size(); ++i)
            if (P.free_list[i]->dev == dev) {
                DpWork *w = P.free_list[i];
                P.free_list.erase(P.free_list.begin() + (long)i);
                return w;
            }
    }
    DpWork *w = new DpWork;
    w->dev = dev;
    if (hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc((void **)&w->pin, sizeof(DpState), hipHostMallocDefault) != hipSuccess) {
        delete w;
        return nullptr;
    }
    return w;
}
void dp_release(DpWork *w) {
    DpPool &P = dp_pool();
    std::lock_guard<std::mutex> g(P.mu);
    P.free_list.push_back(w);
}
// A call's hold on a workspace: returned to the pool after a call that
// completed; destroyed after a call that failed part-way (its device state --
// epoch stamps, the hash table -- may not be clean).
struct DpLease {
    DpWork *w;
    bool ok = false;
    ~DpLease() {
        if (!w) return;
        if (ok) {
            dp_release(w);
        } else {
            (void)hipStreamSynchronize(w->stream);
            delete w;
        }
    }
};

// grow the pair-sized buffers (contents are per-step scratch; the stamp
// arrays start at 0, the table EMPTY, the kept bitmap clear)
int grow_pairs(DpWork &W, int64_t npairs, int K) {
    if (npairs <= W.pair_cap && W.K == K && W.tslots) return SATMI_OK;
    const int64_t cap = std::max<int64_t>(std::max<int64_t>(npairs + npairs / 2, 1 << 16), W.pair_cap);
    if (cap >= (1ll << 31)) {
        set_error("satmi_dp_host: more than 2^31 resolvent pairs in one step");
        return SATMI_ERR_TOO_LARGE;
    }
    hipStream_t s = W.stream;
    DP_TRY(W.rbits.need(8 * (size_t)cap * K, s));
    DP_TRY(W.ntbits.need(8 * (size_t)((cap + 63) / 64 + 1), s));
    DP_TRY(W.uslot.need(4 * (size_t)cap, s));
    DP_TRY(W.surv.need(4 * (size_t)cap, s));
    DP_TRY(W.klist.need(4 * (size_t)cap, s));
    DP_TRY(W.ustage.need(4 * (size_t)DP_STRIPES * cap, s));
    DP_TRY(W.skeys.need(8 * (size_t)cap * K, s));
    DP_TRY(W.dropped.need(4 * (size_t)cap, s, 0, 0));
    DP_TRY(W.hit.need(4 * (size_t)cap, s, 0, 0));
    DP_TRY(W.keptbits.need(4 * (size_t)((cap + 31) / 32 + 1), s, 0, 0));
    uint64_t ts = 1024;
    while (ts < 2 * (uint64_t)cap) ts <<= 1;
    DP_TRY(W.table.need(8 * (size_t)ts, s, 0, 0xFF));
    // a buffer that did not move keeps its contents: the stamps stay below
    // the next epoch, every step leaves the bitmap and the table clear (slots
    // past the old table size were never used)
    uint64_t pw = 1024;
    while (pw * 2 <= W.table.cap / 8) pw <<= 1;
    W.tslots = pw;
    W.pair_cap = std::min<int64_t>((int64_t)(W.rbits.cap / (8 * (size_t)K)), (int64_t)(W.tslots / 2));
    W.pair_cap = std::min<int64_t>(W.pair_cap, (int64_t)(W.uslot.cap / 4));
    W.pair_cap = std::min<int64_t>(W.pair_cap, (int64_t)(W.ustage.cap / (4 * (size_t)DP_STRIPES)));
    W.pair_cap = std::min<int64_t>(W.pair_cap, (int64_t)(W.skeys.cap / (8 * (size_t)K)));
    W.pair_cap = std::min<int64_t>(W.pair_cap, (1ll << 31) - 1);
    W.K = K;
    return SATMI_OK;
}

int grow_ncl(DpWork &W, int64_t n, int K, int cur, int64_t keep_n) {
    if (n <= W.ncl_cap && W.K == K) return SATMI_OK;
    hipStream_t s = W.stream;
    const int64_t cap = std::max<int64_t>(n + n / 2, 1024);
    DP_TRY(W.g[cur].reserve(cap, K, s, keep_n));
    DP_TRY(W.g[cur ^ 1].reserve(cap, K, s, 0));
    DP_TRY(W.plist.need(8 * (size_t)cap, s));
    DP_TRY(W.nlist.need(8 * (size_t)cap, s));
    DP_TRY(W.rlist.need(8 * (size_t)cap, s));
    DP_TRY(W.rkeys.need(8 * (size_t)cap * K, s));
    int64_t c = INT64_MAX;
    for (int g = 0; g < 2; ++g) {
        c = std::min<int64_t>(c, (int64_t)(W.g[g].off.cap / 8));
        c = std::min<int64_t>(c, (int64_t)(W.g[g].mask.cap / 4));
        c = std::min<int64_t>(c, (int64_t)(W.g[g].fill.cap / 4));
        c = std::min<int64_t>(c, (int64_t)(W.g[g].used.cap / 4));
        c = std::min<int64_t>(c, (int64_t)(W.g[g].bits.cap / (8 * (size_t)K)));
    }
    c = std::min<int64_t>(c, (int64_t)(W.plist.cap / 8));
    c = std::min<int64_t>(c, (int64_t)(W.nlist.cap / 8));
    c = std::min<int64_t>(c, (int64_t)(W.rlist.cap / 8));
    c = std::min<int64_t>(c, (int64_t)(W.rkeys.cap / (8 * (size_t)K)));
    W.ncl_cap = c;
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
    g_dp_stats = DpStats{};
    if (V == 0) {   // no variables: `while variables` never runs -- True (REF.py:130)
        *h_result = 1;
        return SATMI_OK;
    }
    const int Wd = (V + 63) / 64;
    const int K = 2 * Wd;
    g_dp_stats.words = K;
    int dev_id = 0;
    SATMI_HIP(hipGetDevice(&dev_id));
    DpLease lease{dp_acquire(dev_id)};
    if (!lease.w) {
        set_error("satmi_dp_host: hipStreamCreate failed");
        return SATMI_ERR_HIP;
    }
    DpWork &Wk = *lease.w;
    hipStream_t s = Wk.stream;
    if (Wk.K != K) {   // key width changed: every K-sized buffer is re-laid out
        Wk.ncl_cap = 0;
        Wk.pair_cap = 0;
    }
    const int64_t cap0 = cap_for(maxlen);
    DP_TRY(Wk.d_off.need(4 * (size_t)(nclauses + 1), s));
    DP_TRY(Wk.d_lits.need(4 * (size_t)std::max<int64_t>(Ltot, 1), s));
    DP_TRY(Wk.d_v2d.need(4 * (size_t)(maxvar + 1), s));
    DP_TRY(Wk.d_d2v.need(4 * (size_t)V, s));
    DP_TRY(Wk.state.need(sizeof(DpState), s));
    DP_TRY(Wk.firstpos.need(8 * (size_t)V, s));
    DP_TRY(Wk.order.need(4 * (size_t)V, s));
    const int64_t popcap = cap_for(V);
    DP_TRY(Wk.popscratch.need(4 * (size_t)2 * popcap, s));
    DP_TRY(Wk.trace.need(4 * (size_t)(V + 1), s));
    DP_TRY(Wk.stripes.need(8 * 3 * DP_STRIPES, s, 0, 0));
    DP_TRY(grow_ncl(Wk, std::max<int64_t>(nclauses, 1), K, 0, 0));
    DP_TRY(grow_pairs(Wk, 1, K));
    const int64_t arena0 = (int64_t)nclauses * 2 * cap0;
    DP_TRY(Wk.arena.need(4 * (size_t)std::max<int64_t>(arena0 * 4, 1 << 16), s));
    Wk.arena_cap = (int64_t)(Wk.arena.cap / 4);
    DP_TRY(Wk.xs.need(4 * (size_t)(1 << 16), s));
    Wk.xs_cap = (int64_t)(Wk.xs.cap / 4);

    if (nclauses > 0) {
        SATMI_HIP(hipMemcpyAsync(Wk.d_off.p, h_clause_off, 4 * (size_t)(nclauses + 1), hipMemcpyHostToDevice, s));
        if (Ltot) SATMI_HIP(hipMemcpyAsync(Wk.d_lits.p, h_lits, 4 * (size_t)Ltot, hipMemcpyHostToDevice, s));
    }
    SATMI_HIP(hipMemcpyAsync(Wk.d_v2d.p, var2dense.data(), 4 * (size_t)(maxvar + 1), hipMemcpyHostToDevice, s));
    SATMI_HIP(hipMemcpyAsync(Wk.d_d2v.p, dense2var.data(), 4 * (size_t)V, hipMemcpyHostToDevice, s));
    SATMI_HIP(hipMemsetAsync(Wk.firstpos.p, 0xFF, 8 * (size_t)V, s));
    DpState &st = *Wk.pin;
    st = DpState{};
    st.ncl = nclauses;
    st.arena_top = arena0;
    st.first_empty = DP_EMPTY;
    st.epoch = Wk.epoch;
    SATMI_HIP(hipMemcpyAsync(Wk.state.p, Wk.pin, sizeof(DpState), hipMemcpyHostToDevice, s));

    double hz = 1e8;
    (void)satmi_wallclock_hz(&hz);
    const bool record = h_rec_lits && h_rec_clause_off && h_rec_step_off;
    const char *inl_env = std::getenv("SATMI_DP_INLINE");
    const bool inline_on = inl_env && inl_env[0] == '1';
    const auto args = [&]() {
        DpArgs a;
        std::memset(&a, 0, sizeof(a));   // padding too: a batch's graph is keyed by these bytes
        a.st = Wk.state.as<DpState>();
        a.g[0] = Wk.g[0].view();
        a.g[1] = Wk.g[1].view();
        a.arena = Wk.arena.as<int32_t>();
        a.arena_cap = Wk.arena_cap;
        a.v2d = Wk.d_v2d.as<int32_t>();
        a.d2v = Wk.d_d2v.as<int32_t>();
        a.V = V;
        a.W = Wd;
        a.K = K;
        a.firstpos = Wk.firstpos.as<unsigned long long>();
        a.order = Wk.order.as<int32_t>();
        a.popscratch = Wk.popscratch.as<int32_t>();
        a.popcap = popcap;
        a.plist = Wk.plist.as<int64_t>();
        a.nlist = Wk.nlist.as<int64_t>();
        a.rlist = Wk.rlist.as<int64_t>();
        a.ncl_cap = Wk.ncl_cap;
        a.rbits = Wk.rbits.as<uint64_t>();
        a.ntbits = Wk.ntbits.as<uint64_t>();
        a.pair_cap = Wk.pair_cap;
        a.table = Wk.table.as<uint64_t>();
        a.tmask = Wk.tslots - 1;
        a.uslot = Wk.uslot.as<uint32_t>();
        a.dropped = Wk.dropped.as<int32_t>();
        a.hit = Wk.hit.as<int32_t>();
        a.surv = Wk.surv.as<uint32_t>();
        a.klist = Wk.klist.as<uint32_t>();
        a.rkeys = Wk.rkeys.as<uint64_t>();
        a.skeys = Wk.skeys.as<uint64_t>();
        a.stripes = Wk.stripes.as<unsigned long long>();
        a.ustage = Wk.ustage.as<uint32_t>();
        a.keptbits = Wk.keptbits.as<uint32_t>();
        a.xs = Wk.xs.as<int32_t>();
        a.xs_cap = Wk.xs_cap;
        a.trace = Wk.trace.as<int32_t>();
        a.trace_cap = V + 1;
        a.step_limit = step_limit;
        a.clause_limit = clause_limit;
        a.limit_ticks = time_limit_s > 0 ? (uint64_t)std::max(1.0, time_limit_s * hz) : 0;
        // inline steps (opt-in); recording reads the clause list after every
        // step: one step per slot
        a.inline_steps = !inline_on ? 0 : record ? 1 : (1 << 30);
        return a;
    };
    DpArgs A = args();
    if (nclauses > 0) {
        hipLaunchKernelGGL(dp_encode_kernel, dim3(grid_for(nclauses)), dim3(256), 0, s, A, nclauses,
                           Wk.d_off.as<int32_t>(), Wk.d_lits.as<int32_t>(), cap0);
        SATMI_HIP(hipGetLastError());
    }
    // device time of the elimination steps: one event pair per batch
    size_t nev = 0;
    const auto next_events = [&]() -> hipEvent_t * {
        if (2 * nev + 2 > Wk.ev.size()) {
            hipEvent_t a = nullptr, b = nullptr;
            if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return nullptr;
            Wk.ev.push_back(a);
            Wk.ev.push_back(b);
        }
        return &Wk.ev[2 * nev++];
    };
    // one elimination step: DP_LAUNCHES_PER_STEP launches, sizes on the device
    const auto enqueue_step = [&](const DpArgs &a) -> int {
        const int gp = (int)std::min<int64_t>(DP_GRID_PAIRS, (a.pair_cap + 255) / 256);
        const int gc = (int)std::min<int64_t>(DP_GRID_ASM, (a.ncl_cap + ASM_WAVES - 1) / ASM_WAVES);
        if (a.inline_steps > 0) hipLaunchKernelGGL(dp_pop_split_kernel<true>, dim3(1), dim3(POP_THREADS), 0, s, a);
        else hipLaunchKernelGGL(dp_pop_split_kernel<false>, dim3(1), dim3(POP_THREADS), 0, s, a);
        hipLaunchKernelGGL(dp_pairs_kernel, dim3(gp), dim3(256), 0, s, a);
        hipLaunchKernelGGL(dp_hash_kernel, dim3(gp), dim3(256), 0, s, a);
        const dim3 gt((unsigned)std::min<int64_t>(DP_GRID_TEST, std::max<int64_t>(64, a.pair_cap / 256)));
        switch (a.K) {
            case 2: hipLaunchKernelGGL(dp_remtest_kernel<2>, gt, dim3(TEST_TILE), 0, s, a); break;
            case 4: hipLaunchKernelGGL(dp_remtest_kernel<4>, gt, dim3(TEST_TILE), 0, s, a); break;
            case 6: hipLaunchKernelGGL(dp_remtest_kernel<6>, gt, dim3(TEST_TILE), 0, s, a); break;
            case 8: hipLaunchKernelGGL(dp_remtest_kernel<8>, gt, dim3(TEST_TILE), 0, s, a); break;
            default: hipLaunchKernelGGL(dp_remtest_kernel<0>, gt, dim3(TEST_TILE), 0, s, a);
        }
        hipLaunchKernelGGL(dp_survlist_kernel, dim3(gp), dim3(256), 0, s, a);
        switch (a.K) {
            case 2: hipLaunchKernelGGL(dp_survtest_kernel<2>, gt, dim3(TEST_TILE), 0, s, a); break;
            case 4: hipLaunchKernelGGL(dp_survtest_kernel<4>, gt, dim3(TEST_TILE), 0, s, a); break;
            case 6: hipLaunchKernelGGL(dp_survtest_kernel<6>, gt, dim3(TEST_TILE), 0, s, a); break;
            case 8: hipLaunchKernelGGL(dp_survtest_kernel<8>, gt, dim3(TEST_TILE), 0, s, a); break;
            default: hipLaunchKernelGGL(dp_survtest_kernel<0>, gt, dim3(TEST_TILE), 0, s, a);
        }
        hipLaunchKernelGGL(dp_kept_kernel, dim3(1), dim3(POP_THREADS), 0, s, a);
        hipLaunchKernelGGL(dp_assemble_kernel, dim3(gc), dim3(64 * ASM_WAVES), 0, s, a);
        SATMI_HIP(hipGetLastError());
        return SATMI_OK;
    };
    int64_t rec_clauses = 0, rec_lits = 0;
    int recorded_steps = 0;
    std::vector<int64_t> h_off;
    std::vector<int32_t> h_mask, h_arena;
    int enqueued = 0;   // steps enqueued since the last resume
    bool first_batch = true;
    for (;;) {
        // at most V steps eliminate a variable, then one pop finds the set empty;
        // a slot may run many steps inline, so a call with the arguments of the
        // last one starts with as many slots as that one used (the next batch,
        // if any, with the full count)
        const bool hinted = first_batch && Wk.hint_slots > 0 && std::memcmp(&Wk.hint_args, &A, sizeof(DpArgs)) == 0;
        const int batch = record ? 1 : hinted ? std::min(Wk.hint_slots, V + 1) : std::min(64, V + 1);
        first_batch = false;
        hipEvent_t *ev = next_events();
        if (!ev) {
            set_error("satmi_dp_host: hipEventCreate failed");
            return SATMI_ERR_HIP;
        }
        SATMI_HIP(hipEventRecord(ev[0], s));
        // A batch is ~10 launches per step whose arguments depend only on the
        // workspace and the call's limits: the second time the same batch is
        // enqueued it is captured into a HIP graph, and from then on replayed
        // with one launch (the steps' sizes live on the device either way).
        DpGraph &G = Wk.graph;
        const bool same = G.batch == batch && std::memcmp(&G.args, &A, sizeof(DpArgs)) == 0;
        if (!record && same && G.exec) {
            SATMI_HIP(hipGraphLaunch(G.exec, s));
        } else if (!record && same) {
            hipGraph_t graph = nullptr;
            SATMI_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            int rc = SATMI_OK;
            for (int k = 0; k < batch && rc == SATMI_OK; ++k) rc = enqueue_step(A);
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
        } else {
            if (!record) {   // remember the batch: captured if it comes again
                G.reset();
                G.args = A;
                G.batch = batch;
            }
            for (int k = 0; k < batch; ++k) DP_TRY(enqueue_step(A));
        }
        SATMI_HIP(hipEventRecord(ev[1], s));
        enqueued += batch;
        g_dp_stats.launches += (int64_t)batch * DP_LAUNCHES_PER_STEP;
        SATMI_HIP(hipMemcpyAsync(Wk.pin, Wk.state.p, sizeof(DpState), hipMemcpyDeviceToHost, s));
        SATMI_HIP(hipStreamSynchronize(s));
        if (st.set_ovf) {
            set_error("satmi_dp_host: set model table overflow");
            return SATMI_ERR_TOO_LARGE;
        }
        if (st.overflow) {   // grow what ran out, then run the step again
            const int cur = st.cur;
            if (st.overflow & OVF_PAIRS) DP_TRY(grow_pairs(Wk, st.need[0], K));
            if (st.overflow & OVF_NCL) DP_TRY(grow_ncl(Wk, st.need[1], K, cur, st.ncl));
            if (st.overflow & OVF_ARENA) {
                DP_TRY(Wk.arena.need(4 * (size_t)st.need[2], s, 4 * (size_t)st.arena_top));
                Wk.arena_cap = (int64_t)(Wk.arena.cap / 4);
            }
            if (st.overflow & OVF_XS) {
                DP_TRY(Wk.xs.need(4 * (size_t)st.need[3], s));
                Wk.xs_cap = (int64_t)(Wk.xs.cap / 4);
            }
            st.overflow = 0;
            st.done = 0;
            SATMI_HIP(hipMemcpyAsync(Wk.state.p, Wk.pin, sizeof(DpState), hipMemcpyHostToDevice, s));
            A = args();
            SATMI_HIP(hipMemsetAsync(Wk.firstpos.p, 0xFF, 8 * (size_t)V, s));
            hipLaunchKernelGGL(dp_firstpos_kernel, dim3(grid_for(std::max<int64_t>(st.ncl, 1))), dim3(256), 0, s, A);
            SATMI_HIP(hipGetLastError());
            enqueued = 0;
            continue;
        }
        if (record && st.pending && st.steps > recorded_steps && st.steps < rec_step_cap) {
            // the clause list after this step, each clause in its set iteration order
            const int64_t n2 = st.ncl2;
            const int nxt = st.cur ^ 1;
            h_off.resize((size_t)std::max<int64_t>(n2, 1));
            h_mask.resize((size_t)std::max<int64_t>(n2, 1));
            h_arena.resize((size_t)std::max<int64_t>(st.arena_top, 1));
            if (n2 > 0) {
                SATMI_HIP(hipMemcpyAsync(h_off.data(), Wk.g[nxt].off.p, 8 * (size_t)n2, hipMemcpyDeviceToHost, s));
                SATMI_HIP(hipMemcpyAsync(h_mask.data(), Wk.g[nxt].mask.p, 4 * (size_t)n2, hipMemcpyDeviceToHost, s));
                SATMI_HIP(hipMemcpyAsync(h_arena.data(), Wk.arena.p, 4 * (size_t)st.arena_top, hipMemcpyDeviceToHost,
                                         s));
                SATMI_HIP(hipStreamSynchronize(s));
            }
            for (int64_t c = 0; c < n2 && rec_clauses + 1 < rec_clause_cap; ++c) {
                for (int64_t i = 0; i <= h_mask[c]; ++i) {
                    const int32_t k = h_arena[h_off[c] + i];
                    if (k != PY_EMPTY && k != PY_DUMMY && rec_lits < rec_lit_cap) h_rec_lits[rec_lits++] = k;
                }
                h_rec_clause_off[++rec_clauses] = rec_lits;
            }
            h_rec_step_off[st.steps] = rec_clauses;
            recorded_steps = st.steps;
        }
        if (st.done) break;
        if (enqueued > V + 1) {   // cannot happen: every step eliminates a variable
            set_error("satmi_dp_host: elimination did not terminate");
            return SATMI_ERR_HIP;
        }
    }
    Wk.epoch = st.epoch + 1;
    if (std::getenv("SATMI_DP_PHASES")) {   // diagnostics: dp_pop_split_kernel's phase clocks (ticks of hz)
        std::fprintf(stderr, "dp phases us: pop+split %.1f pairs %.1f dedup %.1f remtest %.1f survtest %.1f "
                             "kept %.1f assemble %.1f | slots %d inline steps %lld of %d\n",
                     st.ph[0] * 1e6 / hz, st.ph[1] * 1e6 / hz, st.ph[2] * 1e6 / hz, st.ph[3] * 1e6 / hz,
                     st.ph[4] * 1e6 / hz, st.ph[5] * 1e6 / hz, st.ph[6] * 1e6 / hz, st.slots,
                     (long long)st.inl_steps, st.steps);
    }
    if (!record) {   // the slots this call used: the next call's first batch
        Wk.hint_args = A;
        Wk.hint_slots = std::max(1, st.slots);
    }
    const int steps = st.steps;
    if (h_trace_vars && steps > 0) {
        std::vector<int32_t> tr((size_t)steps);
        SATMI_HIP(hipMemcpyAsync(tr.data(), Wk.trace.p, 4 * (size_t)steps, hipMemcpyDeviceToHost, s));
        SATMI_HIP(hipStreamSynchronize(s));
        for (int k = 0; k < steps && k < trace_cap; ++k) h_trace_vars[k] = tr[(size_t)k];
    }
    g_dp_stats.steps = steps;
    g_dp_stats.tests = st.tests;
    g_dp_stats.new_clauses = st.new_total;
    for (size_t i = 0; i < nev; ++i) {   // the stream has drained
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, Wk.ev[2 * i], Wk.ev[2 * i + 1]) == hipSuccess) g_dp_stats.device_ms += ms;
    }
    *h_result = st.result;
    *h_steps = steps;
    lease.ok = true;
    return SATMI_OK;
}

extern "C" int satmi_dp_last_stats(int64_t *steps, int64_t *subset_tests, int64_t *new_clauses,
                                   int64_t *launches, int *words, double *device_ms) {
    if (steps) *steps = g_dp_stats.steps;
    if (subset_tests) *subset_tests = g_dp_stats.tests;
    if (new_clauses) *new_clauses = g_dp_stats.new_clauses;
    if (launches) *launches = g_dp_stats.launches;
    if (words) *words = g_dp_stats.words;
    if (device_ms) *device_ms = g_dp_stats.device_ms;
    return SATMI_OK;
}

// Free every idle workspace of this solver (device buffers, streams, pinned
// words); calls in flight keep theirs.  The next call allocates afresh.
extern "C" int satmi_dp_trim(void) {
    std::vector<DpWork *> idle;
    {
        auto &P = dp_pool();
        std::lock_guard<std::mutex> g(P.mu);
        idle.swap(P.free_list);
    }
    for (DpWork *w : idle) {
        (void)hipStreamSynchronize(w->stream);
        delete w;
    }
    return SATMI_OK;
}
