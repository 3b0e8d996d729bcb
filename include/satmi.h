/*
 * satmi.h -- C ABI of the MI355X-native clause-set solving path.
 *
 * The reference (andreistana05/SAT-MPI-Stana-Andrei) is one Python script,
 * "comparatie intre algoritmii de rezolvare a seturilor de clauze.py" (REF.py).
 * Its solver entry points are plain Python functions over `List[List[int]]`
 * (REF.py:11-14); the drop-in mirror of those functions lives in
 * sat-mpi-stana-andrei_amd/satmi/solvers.py and calls the entry points below
 * through ctypes (INTEGRATION.md shows the binding).  All pointers are plain
 * C pointers; "d_" pointers are HIP device pointers, "h_" pointers host memory.
 * Every function returns SATMI_OK (0) or a negative error; satmi_last_error()
 * describes the last failure of the calling thread.
 *
 * Formula layout (CSR, the "flat literal/offset arrays in HBM" of the design):
 *   instance b owns clauses  [inst_clause_begin[b], inst_clause_begin[b+1])
 *   clause   c owns literals [clause_lit_begin[c],  clause_lit_begin[c+1])
 *   literals are DIMACS ints (v or -v, v >= 1), exactly the ints of REF.py's
 *   Clause = List[int]; inst_nvars[b] = largest variable index of instance b.
 */
#ifndef SATMI_H
#define SATMI_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SATMI_ABI_VERSION 2

/* return codes */
#define SATMI_OK 0
#define SATMI_ERR_ARG (-1)
#define SATMI_ERR_HIP (-2)
#define SATMI_ERR_TOO_LARGE (-3)
#define SATMI_ERR_NOMEM (-4)

/* per-instance DPLL status (d_status[b]) */
#define SATMI_DPLL_EXHAUSTED 0      /* search tree fully explored                 */
#define SATMI_DPLL_STOPPED 1        /* stopped after max_solutions solutions      */
#define SATMI_DPLL_NODE_LIMIT 2     /* node_limit calls reached                   */
#define SATMI_DPLL_TIMEOUT 3        /* time_limit_s reached (REF.py:17, :417-437)  */
#define SATMI_DPLL_TOO_LARGE 4      /* instance exceeds the launch's LDS layout   */

/* DPLL modes */
#define SATMI_MODE_REF 0    /* dpll_optimized exactly as REF.py:133-214             */
#define SATMI_MODE_SOUND 1  /* same procedure, decisions applied as unit clauses   */

/* counters per instance, d_counters[b*SATMI_NCOUNTERS + k] */
#define SATMI_NCOUNTERS 8
#define SATMI_CTR_NODES 0        /* dpll_optimized calls                         */
#define SATMI_CTR_DECISIONS 1    /* branch assignments (REF.py:212)              */
#define SATMI_CTR_UNIT_PROPS 2   /* unit-propagation assignments (REF.py:154)    */
#define SATMI_CTR_PURE 3         /* pure-literal assignments (REF.py:189)        */
#define SATMI_CTR_CONFLICTS 4    /* unit_propagate returned None (REF.py:168)    */
#define SATMI_CTR_SOLUTIONS 5    /* solutions found (len of REF.py's result)     */
#define SATMI_CTR_ROUNDS 6       /* unit-propagation rounds (clause scans)       */
#define SATMI_CTR_TICKS 7        /* wall-clock ticks the wave spent on the instance (100 MHz s_memrealtime) */

int satmi_abi_version(void);
const char *satmi_last_error(void);
int satmi_device_count(int *count);
int satmi_set_device(int device);
int satmi_synchronize(void);

/* Device memory helpers, so a host program needs no other HIP binding. */
int satmi_malloc(void **d_ptr, uint64_t bytes);
int satmi_free(void *d_ptr);
int satmi_memcpy_h2d(void *d_dst, const void *h_src, uint64_t bytes, void *stream);
int satmi_memcpy_d2h(void *h_dst, const void *d_src, uint64_t bytes, void *stream);
int satmi_stream_synchronize(void *stream);

/*
 * Batched DPLL: one wavefront per instance.  Replaces dpll_optimized
 * (REF.py:133-214) for a batch of formulas.
 *   mode           SATMI_MODE_REF | SATMI_MODE_SOUND
 *   max_solutions  stop after this many solutions (0 = enumerate all, as REF.py)
 *   node_limit     stop after this many dpll calls (0 = none)
 *   time_limit_s   per-instance wall-clock limit (<= 0 = none)
 *   max_vars/max_clauses/max_lits   maxima over the batch (size the LDS layout)
 *   max_clause_len longest clause of the batch, with every clause non-empty;
 *                  0 = unknown.  SOUND mode without a caller assignment and
 *                  1 <= max_clause_len <= 5, max_vars <= 2047 runs the
 *                  clause-scan kernel (same results; see satmi_dpll_set_kernel);
 *                  an instance that breaks the promise gets SATMI_DPLL_TOO_LARGE
 *   d_init_begin/d_init_lits        optional caller assignment (REF.py:133's
 *                  `assignment`), as signed literals in dict order; may be NULL
 *   sol_cap        solutions stored per instance; sol_stride >= max assignment size
 *   outputs: d_status[B], d_counters[B*8], d_sol_len[B*sol_cap],
 *            d_sol_lits[B*sol_cap*sol_stride] (signed literals in the
 *            assignment dict's insertion order), d_root_len[B],
 *            d_root_lits[B*sol_stride] (the caller's dict after the root's
 *            unit_propagate, REF.py:167, which mutates it in place)
 *   stream         hipStream_t (NULL = default stream); the call is asynchronous
 */
int satmi_dpll_batch_device(int num_instances, const int32_t *d_inst_clause_begin,
                            const int32_t *d_clause_lit_begin, const int32_t *d_lits,
                            const int32_t *d_inst_nvars, int max_vars, int max_clauses, int max_lits,
                            int max_clause_len, const int32_t *d_init_begin, const int32_t *d_init_lits,
                            int mode, int64_t max_solutions, int64_t node_limit, double time_limit_s,
                            int sol_cap, int sol_stride,
                            int32_t *d_status, int64_t *d_counters, int32_t *d_sol_len,
                            int32_t *d_sol_lits, int32_t *d_root_len, int32_t *d_root_lits,
                            void *stream);

/* Same, from host arrays (allocates, copies, runs, copies back; synchronous). */
int satmi_dpll_batch_host(int num_instances, const int32_t *h_inst_clause_begin,
                          const int32_t *h_clause_lit_begin, const int32_t *h_lits,
                          const int32_t *h_inst_nvars,
                          const int32_t *h_init_begin, const int32_t *h_init_lits,
                          int mode, int64_t max_solutions, int64_t node_limit, double time_limit_s,
                          int sol_cap, int sol_stride,
                          int32_t *h_status, int64_t *h_counters, int32_t *h_sol_len,
                          int32_t *h_sol_lits, int32_t *h_root_len, int32_t *h_root_lits);

/*
 * Resolution saturation, replaces resolution_solver (REF.py:63-95) for one
 * clause set (CSR host arrays: clause c = lits[clause_off[c] .. clause_off[c+1])).
 * Clauses are variable bitsets in HBM; each pass resolves all pairs on the GPU
 * (tautologies filtered), dedups through a hash table over every clause key.
 * Thread-safe: a call takes a device workspace (buffers + its own HIP stream)
 * from a process-wide pool and returns it, so calls from several threads overlap.
 *   max_passes / clause_limit / time_limit_s   <= 0: unlimited
 *   *result   1 = True (no new clause derivable), 0 = False (empty resolvent),
 *             -1 = a limit stopped the saturation
 *   *passes   completed passes that added clauses; pass_new[p] = clauses added
 *   optional record (all three non-NULL): clauses new in pass p are
 *   rec_pass_off[p] .. rec_pass_off[p+1] in rec_clause_off / rec_lits, each
 *   clause as ascending literals.
 */
int satmi_resolution_host(int nclauses, const int32_t *h_clause_off, const int32_t *h_lits,
                          int64_t max_passes, int64_t clause_limit, double time_limit_s,
                          int32_t *h_result, int32_t *h_passes, int64_t *h_pass_new, int pass_cap,
                          int32_t *h_rec_lits, int64_t rec_lit_cap, int64_t *h_rec_clause_off,
                          int64_t rec_clause_cap, int64_t *h_rec_pass_off, int rec_pass_cap);

/* Work of the last satmi_resolution_host call: pairs resolved, candidate
 * resolvents generated, and the device time of its pair and claim (hash dedup)
 * launches (HIP events on its stream), for rooflines. */
int satmi_resolution_last_stats(int64_t *pairs, int64_t *candidates, double *pair_ms, double *claim_ms);

/* The live shader clock (Hz) of the last satmi_resolution_host call's fused
 * pass kernels (at most 31 variables): shader cycles (s_memtime) over
 * device-clock ticks (s_memrealtime) summed over one block in 64 of every
 * pass, so an issue roofline prices the pipes at the clock the kernel ran
 * at.  0 when no pass kernel ran (the general path beyond 31 variables). */
int satmi_resolution_last_clock(double *shader_hz);

/* Test knob: the first append slot (default 0) of the pair kernel's candidates
 * (more than 31 variables) or of a pass's new clauses (at most 31), so a small
 * pass exercises the slot arithmetic past 2^31 / 2^32. */
int satmi_resolution_debug_slot_base(int64_t base);

/* Test knob: cap of the candidate buffer of the > 31-variable path in bytes
 * (0 = the default 1 GiB), so a small pass takes the re-run-at-the-counted-size
 * path. */
int satmi_resolution_debug_cand_bytes(int64_t bytes);

/*
 * Davis-Putnam elimination, replaces davis_putnam_solver (REF.py:98-130) for one
 * clause set.  Variables are eliminated in the reference's order (CPython's
 * `set.pop()` on the variable set, modelled on the device), resolvents are
 * generated, tautology-filtered and subsumption-filtered on the GPU.
 *   step_limit / clause_limit / time_limit_s   <= 0: unlimited
 *   *result   1 = True, 0 = False (empty resolvent), -1 = a limit stopped it
 *   trace_vars[k] = variable eliminated at step k; *steps = steps run
 *   optional record (all three non-NULL): the clause list after completed step
 *   s is rec_step_off[s-1] .. rec_step_off[s] in rec_clause_off / rec_lits,
 *   every clause in its Python set iteration order; rec_step_off[s] is left
 *   untouched for a step that ended the elimination.
 * Thread-safe: a call takes a device workspace (buffers kept between calls,
 * its own HIP stream) from a process-wide pool and returns it, so solves from
 * several threads overlap and memory is bounded by the peak concurrency.
 */
int satmi_dp_host(int nclauses, const int32_t *h_clause_off, const int32_t *h_lits, int64_t step_limit,
                  int64_t clause_limit, double time_limit_s, int32_t *h_result, int32_t *h_trace_vars,
                  int trace_cap, int32_t *h_steps, int32_t *h_rec_lits, int64_t rec_lit_cap,
                  int64_t *h_rec_clause_off, int64_t rec_clause_cap, int64_t *h_rec_step_off, int rec_step_cap);

/* The floor of a chain of dependent kernel launches replayed from a HIP graph
 * on this device: `launches` one-block kernels captured in order on one
 * stream, the graph replayed `reps` times; *us_per_launch = the time per
 * launch.  The Davis-Putnam roofline (a solve is a chain of ~280 dependent
 * launches) prices its launches/s against this measured floor. */
int satmi_launch_chain_floor(int launches, int reps, double *us_per_launch);

/* Work of the calling thread's last satmi_dp_host call: elimination steps,
 * subset tests performed by the unique_new filter (REF.py:122-125), new
 * (non-tautological) resolvents, kernel launches enqueued for the steps, key
 * words per clause, and the device time of the step batches (HIP events on its
 * stream), for rooflines. */
int satmi_dp_last_stats(int64_t *steps, int64_t *subset_tests, int64_t *new_clauses, int64_t *launches,
                        int *words, double *device_ms);

/* Free the idle device workspaces that satmi_dp_host / satmi_resolution_host
 * keep between calls (buffers only grow while kept); calls in flight keep theirs. */
int satmi_dp_trim(void);
int satmi_resolution_trim(void);

/*
 * CDCL, replaces CDCLSolver / cdcl_solve (REF.py:217-384) for a batch of
 * formulas (CSR host arrays as satmi_dpll_batch_host), one wavefront per
 * instance.  The reference's solve loop has no bound of its own (its caller
 * kills it after 60 s): an instance stops after max_iter loop iterations (<= 0:
 * none), at time_limit_s (<= 0: none) or when its arena (sized for learn_cap
 * learned clauses; <= 0: max_iter, else 65536) is full.
 *   h_status[b]   SATMI_CDCL_SAT / _UNSAT (the reference's (True, model) /
 *                 (False, None)), _LIMIT (a bound stopped it), _ERROR (the
 *                 reference raises: KeyError in analyze_conflict), _FULL
 *   h_assign      [B x assign_stride] the assignment dict as signed literals in
 *                 its insertion order (h_assign_len[b] of them): the model for
 *                 _SAT, else the live dict where the run stopped
 *   h_stats       [B x SATMI_CDCL_NSTATS] iterations, conflicts analysed,
 *                 decisions, learned clauses, formula length, watch-list keys,
 *                 decision level, set-table slots used
 *   h_var_inc[b]  the solver's var_inc at the end
 */
#define SATMI_CDCL_UNSAT 0
#define SATMI_CDCL_SAT 1
#define SATMI_CDCL_LIMIT (-1)
#define SATMI_CDCL_ERROR (-2)
#define SATMI_CDCL_FULL (-3)
#define SATMI_CDCL_NSTATS 8
int satmi_cdcl_batch_host(int num_instances, const int32_t *h_inst_clause_begin, const int32_t *h_clause_lit_begin,
                          const int32_t *h_lits, int64_t max_iter, int64_t learn_cap, double time_limit_s,
                          int32_t *h_status, int32_t *h_assign_len, int32_t *h_assign, int assign_stride,
                          int64_t *h_stats, double *h_var_inc);

/* The calling thread's last satmi_cdcl_batch_host launch: its span on the
 * device wall clock (first wave start to last wave end), the busy wave-time
 * (sum over waves of the time spent solving formulas) and the resident waves;
 * busy / (resident x span) is the launch's wave utilisation. */
int satmi_cdcl_last_stats(double *span_s, double *busy_wave_s, int *resident_waves);

/* Device-side span of the last DPLL launch on `stream`: enqueues (on that
 * stream, after the launch) a copy of two uint64 s_memrealtime ticks into
 * d_span: [0] = ~(first wave's start), [1] = last wave's end, so the launch
 * took (d_span[1] - ~d_span[0]) / satmi_wallclock_hz() seconds -- the kernel's
 * own duration even when launches on two streams overlap. */
int satmi_dpll_launch_span(void *stream, uint64_t *d_span);
int satmi_wallclock_hz(double *hz);

/* LDS bytes one wavefront needs for an instance of this size (0 = unsupported). */
uint64_t satmi_dpll_lds_bytes(int max_vars, int max_clauses, int max_lits);

/* Same for the clause-scan kernel (0 = the shape is not eligible for it). */
uint64_t satmi_dpll_scan_lds_bytes(int max_vars, int max_clauses, int max_lits, int max_clause_len);

/* Which DPLL kernel satmi_dpll_batch_* use (process-wide; default AUTO):
 *   AUTO     the incremental clause kernel where eligible, else the general kernel
 *            (its wide HBM-arena form when the batch exceeds the LDS layout)
 *   GENERAL  always the general (occurrence-list, clause-counter) kernel
 *   SCAN     the clause-scan kernel, every propagation round a full clause scan;
 *            an ineligible call fails with SATMI_ERR_ARG
 *   INC      the clause kernel with incremental rounds (only the clauses that lost
 *            a literal are read); an ineligible call fails with SATMI_ERR_ARG
 *   WIDE     the general kernel in its wide form (see SATMI_KERNEL_WIDE)
 * All give identical statuses, counters and models. */
#define SATMI_KERNEL_AUTO 0
#define SATMI_KERNEL_GENERAL 1
#define SATMI_KERNEL_SCAN 2
#define SATMI_KERNEL_INC 3
#define SATMI_KERNEL_WIDE 4   /* the general kernel with its image in a per-wave HBM arena (32-bit
                                 indices); AUTO takes it for batches beyond the LDS layout */
int satmi_dpll_set_kernel(int policy);

/* Branch splitting in the clause kernels (process-wide; default on): once a
 * launch's instance queue drains, idle wavefronts take over the False branches
 * of open decisions of the searches still running (a search checks for idle
 * wavefronts every 16 nodes); the donor takes the helper's result when its
 * backtracking reaches the branch.  Statuses, counters and models are those of
 * the unsplit search (branches a sequential search would not have visited are
 * cancelled and count nothing).  Applies to SOUND-mode launches with
 * max_solutions == 1, no node limit and no time limit.
 *   enable          0 off; 1 auto (default): launches with at least one and
 *                   at most 8 instances per resident wavefront; 2 every
 *                   eligible launch
 *   helpers_per_cu  wavefronts per CU that stay as helpers once the queue
 *                   drains (0 = default 1); the others exit, freeing their CU
 *                   slots for a launch queued on another stream */
int satmi_dpll_set_split(int enable, int helpers_per_cu);

/* Nodes (recursive calls) a search visits before it may donate a branch
 * (process-wide; < 0 = default 256, 0 = from its first donation check).  Short
 * searches never split: their subtrees cost a helper more to restage than to
 * search. */
int satmi_dpll_set_split_warmup(int nodes);

/* Branch-splitting statistics of the last DPLL launch on `stream` (waits for
 * the stream): out[0..6] = donations, helper tickets, subtrees run by helpers,
 * donations taken back by their donors, waves that registered as helpers,
 * searches handed to a helper (a donor that reaches a branch its helper is
 * still searching passes it the rest of its search instead of waiting; until
 * r06 this entry was the donors' waiting ticks), root instances finished.  All zero
 * (out[6] = 0) when that launch did not split. */
int satmi_dpll_split_stats(void *stream, int64_t *out);

/* Wave ticks (satmi_wallclock_hz) that the waves of the last DPLL launch on
 * `stream` spent inside searches, summed over the launch's waves, if that
 * launch split (else 0; waits for the stream).  Divided by the launch's waves
 * and its span (satmi_dpll_launch_span) it is the launch's wave utilisation,
 * measured per wave -- independent of how a split search's rows collect their
 * helpers' ticks. */
int satmi_dpll_split_busy(void *stream, int64_t *busy_ticks);

/* The launch satmi_dpll_batch_device would make for this batch shape under the
 * current policy: *kernel = SATMI_KERNEL_SCAN or SATMI_KERNEL_GENERAL, LDS
 * bytes per wavefront, and wavefronts resident per CU (LDS and registers). */
int satmi_dpll_plan(int max_vars, int max_clauses, int max_lits, int max_clause_len, int mode, int has_init,
                    int *kernel, uint64_t *lds_bytes_per_wave, int *waves_per_cu);

#ifdef __cplusplus
}
#endif
#endif
