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
//   * sort-based dedup: stable merge sort of the candidate indices by key,
//     keep the first of every run that is absent from `seen` (binary search in
//     the sorted `seen` array), scan + scatter, then rank-merge into `seen`;
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
template <bool WRITE>
__global__ void __launch_bounds__(256) res_pairs_kernel(const uint64_t *keys, int W, int64_t jlo, int64_t npairs,
                                                        unsigned long long *count, int *empty_found,
                                                        uint64_t *cand, int64_t cand_cap) {
    const int K = 2 * W;
    const int ln = lane_id();
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t base = tri(jlo);
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
            const int64_t slot = (int64_t)slot0 + __popcll(m & lanemask_lt());
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

// flag[t] = sorted candidate t is the first of its run and not in seen
__global__ void res_unique_kernel(KeyView cand, const int64_t *perm, int64_t n, KeyView seen, int64_t nseen,
                                  int64_t *flag) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t *x = cand.at(perm[t]);
        bool keep = t == 0 || key_cmp(cand.at(perm[t - 1]), x, cand.K) != 0;
        if (keep && nseen > 0) {
            const int64_t r = rank_in<false>(seen, nullptr, 0, nseen, x);
            if (r < nseen && key_cmp(seen.at(r), x, seen.K) == 0) keep = false;
        }
        flag[t] = keep ? 1 : 0;
    }
}

__global__ void res_scatter_kernel(KeyView cand, const int64_t *perm, const int64_t *flag, const int64_t *pos,
                                   int64_t n, uint64_t *out) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
        if (!flag[t]) continue;
        const uint64_t *x = cand.at(perm[t]);
        uint64_t *o = out + pos[t] * cand.K;
        for (int w = 0; w < cand.K; ++w) o[w] = x[w];
    }
}

// merge two sorted, disjoint key arrays A (na) and B (nb) into out
__global__ void res_merge_kernel(KeyView A, int64_t na, KeyView B, int64_t nb, uint64_t *out) {
    const int K = A.K;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < na + nb; t += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t *x;
        int64_t pos;
        if (t < na) {
            x = A.at(t);
            pos = t + rank_in<false>(B, nullptr, 0, nb, x);
        } else {
            x = B.at(t - na);
            pos = (t - na) + rank_in<false>(A, nullptr, 0, na, x);
        }
        for (int w = 0; w < K; ++w) out[pos * K + w] = x[w];
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

// Sort + dedup `n` candidate keys against the sorted `seen` (nseen); writes the
// new sorted keys to out_new and returns their count through *nnew.
struct Dedup {
    DevBuf perm_a, perm_b, flag, pos, tiles, grand;
    int run(const uint64_t *cand, int64_t n, const uint64_t *seen, int64_t nseen, int K, DevBuf &out_new,
            int64_t *nnew, hipStream_t s) {
        *nnew = 0;
        if (n == 0) return SATMI_OK;
        SATMI_TRY(perm_a.reserve(8 * n));
        SATMI_TRY(perm_b.reserve(8 * n));
        SATMI_TRY(flag.reserve(8 * n));
        SATMI_TRY(pos.reserve(8 * n));
        SATMI_TRY(tiles.reserve(8 * ((n + SCAN_TILE - 1) / SCAN_TILE + 1)));
        SATMI_TRY(grand.reserve(8));
        KeyView kc{cand, K}, ks{seen, K};
        int64_t *perm = nullptr;
        SATMI_TRY(sort_indices(kc, n, perm_a.as<int64_t>(), perm_b.as<int64_t>(), &perm, s));
        hipLaunchKernelGGL(res_unique_kernel, dim3(grid_for(n)), dim3(PRIM_BLOCK), 0, s, kc, perm, n, ks, nseen,
                           flag.as<int64_t>());
        SATMI_TRY(exclusive_scan(flag.as<int64_t>(), pos.as<int64_t>(), n, tiles.as<int64_t>(),
                                 grand.as<int64_t>(), s));
        SATMI_HIP(hipMemcpyAsync(nnew, grand.p, 8, hipMemcpyDeviceToHost, s));
        SATMI_HIP(hipStreamSynchronize(s));
        if (*nnew == 0) return SATMI_OK;
        SATMI_TRY(out_new.reserve(8 * (size_t)*nnew * K));
        hipLaunchKernelGGL(res_scatter_kernel, dim3(grid_for(n)), dim3(PRIM_BLOCK), 0, s, kc, perm,
                           flag.as<int64_t>(), pos.as<int64_t>(), n, out_new.as<uint64_t>());
        SATMI_HIP(hipGetLastError());
        return SATMI_OK;
    }
};

}  // namespace

}  // namespace satmi

using namespace satmi;

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
    hipStream_t s = nullptr;

    DevBuf d_off, d_lits, d_map, clauses, seen, seen2, cand, newk, counters;
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
    // seen = {frozenset(c) for c in clauses}  (REF.py:65): sorted unique input keys
    Dedup dd;
    int64_t nseen = 0;
    SATMI_TRY(dd.run(clauses.as<uint64_t>(), ncl, nullptr, 0, K, seen, &nseen, s));

    int64_t jlo = 0, rec_clauses = 0, rec_lits = 0;
    int passes = 0;
    std::vector<uint64_t> hkeys;
    for (;;) {
        if (max_passes > 0 && passes >= max_passes) break;
        if (time_limit_s > 0 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count() > time_limit_s)
            break;
        const int64_t npairs = (ncl * (ncl - 1) - jlo * (jlo - 1)) / 2;
        struct {
            unsigned long long count;
            int empty;
            int pad;
        } hc{0, 0, 0};
        SATMI_HIP(hipMemsetAsync(counters.p, 0, 16, s));
        unsigned long long *d_count = counters.as<unsigned long long>();
        int *d_empty = (int *)(counters.as<char>() + 8);
        const int grid = grid_for(npairs);
        if (npairs > 0) {
            hipLaunchKernelGGL(res_pairs_kernel<false>, dim3(grid), dim3(256), 0, s, clauses.as<uint64_t>(), W, jlo,
                               npairs, d_count, d_empty, nullptr, (int64_t)0);
            SATMI_HIP(hipGetLastError());
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
            // the pass's working set: candidate keys + four int64 arrays of the
            // sort/dedup; refuse (SATMI_ERR_NOMEM) rather than oversubscribe HBM
            const double need = (double)ncand * (8.0 * K + 32.0) + 8.0 * (double)(nseen + ncand) * K;
            size_t free_b = 0, total_b = 0;
            SATMI_HIP(hipMemGetInfo(&free_b, &total_b));
            if (need > 0.8 * (double)free_b) {
                set_error("satmi_resolution_host: pass " + std::to_string(passes + 1) + " has " +
                          std::to_string(ncand) + " candidate resolvents, needing " +
                          std::to_string(need / 1e9) + " GB of device memory (" + std::to_string(free_b / 1e9) +
                          " GB free); set clause_limit / max_passes");
                return SATMI_ERR_NOMEM;
            }
            SATMI_TRY(cand.reserve(8 * (size_t)ncand * K));
            SATMI_HIP(hipMemsetAsync(counters.p, 0, 16, s));
            hipLaunchKernelGGL(res_pairs_kernel<true>, dim3(grid), dim3(256), 0, s, clauses.as<uint64_t>(), W, jlo,
                               npairs, d_count, d_empty, cand.as<uint64_t>(), ncand);
            SATMI_HIP(hipGetLastError());
            SATMI_TRY(dd.run(cand.as<uint64_t>(), ncand, seen.as<uint64_t>(), nseen, K, newk, &nnew, s));
        }
        if (nnew == 0) {   // no new clauses can be derived (REF.py:91-92)
            *h_result = 1;
            break;
        }
        // record the pass (REF.py:94 `seen.update(new_clauses)`)
        if (h_pass_new && passes < pass_cap) h_pass_new[passes] = nnew;
        if (h_rec_lits && h_rec_clause_off && h_rec_pass_off && passes + 1 < rec_pass_cap) {
            hkeys.resize((size_t)nnew * K);
            SATMI_HIP(hipMemcpyAsync(hkeys.data(), newk.p, 8 * (size_t)nnew * K, hipMemcpyDeviceToHost, s));
            SATMI_HIP(hipStreamSynchronize(s));
            std::vector<int32_t> cl;
            for (int64_t c = 0; c < nnew && rec_clauses + 1 < rec_clause_cap; ++c) {
                cl.clear();
                const uint64_t *k = hkeys.data() + c * K;
                for (int d = 0; d < V; ++d) {
                    if ((k[d >> 6] >> (d & 63)) & 1ull) cl.push_back(dense2var[d]);
                    if ((k[W + (d >> 6)] >> (d & 63)) & 1ull) cl.push_back(-dense2var[d]);
                }
                std::sort(cl.begin(), cl.end());
                if (rec_lits + (int64_t)cl.size() > rec_lit_cap) break;
                std::copy(cl.begin(), cl.end(), h_rec_lits + rec_lits);
                rec_lits += (int64_t)cl.size();
                h_rec_clause_off[++rec_clauses] = rec_lits;
            }
            h_rec_pass_off[passes + 1] = rec_clauses;
        }
        ++passes;
        // clauses.extend(new) and seen |= new
        const int64_t ncl2 = ncl + nnew;
        if ((size_t)ncl2 * K * 8 > clauses.cap) {
            DevBuf grown;
            SATMI_TRY(grown.reserve(8 * (size_t)ncl2 * K * 2));
            SATMI_HIP(hipMemcpyAsync(grown.p, clauses.p, 8 * (size_t)ncl * K, hipMemcpyDeviceToDevice, s));
            std::swap(grown.p, clauses.p);
            std::swap(grown.cap, clauses.cap);
        }
        SATMI_HIP(hipMemcpyAsync(clauses.as<uint64_t>() + ncl * K, newk.p, 8 * (size_t)nnew * K,
                                 hipMemcpyDeviceToDevice, s));
        SATMI_TRY(seen2.reserve(8 * (size_t)(nseen + nnew) * K));
        hipLaunchKernelGGL(res_merge_kernel, dim3(grid_for(nseen + nnew)), dim3(PRIM_BLOCK), 0, s,
                           KeyView{seen.as<uint64_t>(), K}, nseen, KeyView{newk.as<uint64_t>(), K}, nnew,
                           seen2.as<uint64_t>());
        SATMI_HIP(hipGetLastError());
        std::swap(seen.p, seen2.p);
        std::swap(seen.cap, seen2.cap);
        nseen += nnew;
        jlo = ncl;
        ncl = ncl2;
        if (clause_limit > 0 && ncl > clause_limit) break;
    }
    SATMI_HIP(hipStreamSynchronize(s));
    *h_passes = passes;
    return SATMI_OK;
}
