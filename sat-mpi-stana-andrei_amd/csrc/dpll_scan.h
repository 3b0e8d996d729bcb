// dpll_scan.h -- launch interface of the clause-scan DPLL kernel (dpll_scan.hip),
// the SOUND-mode fast path behind satmi_dpll_batch_device (dpll.hip dispatches).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>

namespace satmi {

constexpr int SPLIT_HELPERS_PER_CU = 1;   // measured: 1 best with two pipelined streams (4: -6 %, 8: -48 % at the N=8 share)
// nodes a search visits before it may donate: short searches (most of
// configs[1]) would only ship overhead to the helpers
constexpr int SPLIT_WARMUP_NODES = 256;

struct ScanLaunch {
    int num_instances;
    const int32_t *inst_clause_begin, *clause_lit_begin, *lits, *inst_nvars;
    int max_vars, max_clauses, max_lits, max_clause_len;
    int64_t max_solutions, node_limit;
    uint64_t time_limit_ticks;
    int sol_cap, sol_stride;
    int32_t *status;
    int64_t *counters;
    int32_t *sol_len, *sol_lits, *root_len, *root_lits;
    uint32_t *work_counter;
    int num_cus;
    hipStream_t stream;
    bool inc = false;   // incremental propagation (occurrence lists) instead of full clause scans
    // incremental kernel: returns >= bytes of device scratch for the occurrence lists,
    // valid for this launch on `stream` (nullptr on failure)
    std::function<uint16_t *(size_t)> occ_alloc;
    // branch splitting of the launch's tail (dpll_scan.hip, "Splitting the tail"):
    // split_alloc returns >= bytes of device scratch valid for this launch on
    // `stream` and the launch's tag for the slot states (distinct per launch on
    // the stream), nullptr on failure
    bool split = false;
    bool split_always = false;   // split any eligible launch (else only 1 <= instances per resident wave <= 8)
    int split_helpers_per_cu = SPLIT_HELPERS_PER_CU;   // waves per CU that stay as helpers once the queue drains
    int split_warmup = SPLIT_WARMUP_NODES;   // nodes of a search before its first donation
    std::function<void *(size_t, uint32_t *)> split_alloc;
};

// Can the scan kernel take a batch of this shape (SOUND mode, no caller
// assignment)?  Fills *lds_bytes with the per-wave LDS it would use.
bool dpll_scan_eligible(int max_vars, int max_clauses, int max_lits, int max_clause_len, bool inc,
                        uint32_t *lds_bytes);

// Waves of the scan kernel resident per CU for this shape (LDS and registers),
// and the LDS bytes per wave of that launch (dynamic image + static literal states).
int dpll_scan_resident(int max_vars, int max_clauses, int max_clause_len, bool inc, int *waves_per_cu,
                       uint32_t *lds_per_wave = nullptr);

// Bytes of the splitting scratch head, and its statistics decoded from a host
// copy of it: [donations, tickets, claims, reclaims, helpers, handoffs, done].
constexpr int SPLIT_HEAD_BYTES = 512;
void dpll_split_decode(const void *head, int64_t out[7]);
int64_t dpll_split_busy(const void *head);   // wave ticks the launch's waves spent searching

// Launch on L.stream (asynchronous).  The caller has checked eligibility and
// zeroed *L.work_counter on the stream.
int dpll_scan_launch(const ScanLaunch &L);

}  // namespace satmi
