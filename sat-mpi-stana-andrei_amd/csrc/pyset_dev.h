// pyset_dev.h -- device model of CPython 3.10 `set` tables for int keys.
//
// davis_putnam_solver (REF.py:98-130) chooses the variable to eliminate with
// `variables.pop()` on `{abs(lit) for clause in clauses for lit in clause}`.
// Which variable that is depends on CPython's open-addressing layout of that
// set, which depends on the order the clause sets iterate, which depends on
// how each clause set was built: `set(list)` (REF.py:99), `pc - {var}`,
// `nc - {-var}` and their union `|` (REF.py:114).  To eliminate variables in
// the reference's order -- and so produce its intermediate clause lists -- a
// clause carries its table image: slots of int32 keys (0 = empty, INT32_MIN =
// dummy), mask, fill and used.  The operations below follow
// Objects/setobject.c of CPython 3.10: set_add_entry (9 linear probes, then
// perturbed probing), set_insert_clean, set_table_resize (new size = smallest
// power of two above 4*used, dummies dropped), set_merge (its resize rule,
// table-copy and insert-clean fast paths), set_difference (copy-and-discard
// when len(a) >> 2 > len(b)), set_lookkey / set_discard_entry and set_pop.
// int hash: hash(k) = k, except hash(-1) == -2.
//
// Everything is inlined, so a caller whose tables are all in LDS gets ds_*
// accesses.  A table is scanned PY_BATCH slots at a time (the slots read
// together, then processed): the chain of one set operation is a series of
// dependent round trips, and a scan slot's read does not depend on the adds
// before it (it reads another table), so batching takes most scan reads off
// the chain.  Table sizes are powers of two >= PY_MINSIZE = PY_BATCH.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace satmi {

constexpr int32_t PY_EMPTY = 0;
constexpr int32_t PY_DUMMY = INT32_MIN;
constexpr int PY_MINSIZE = 8;
constexpr int PY_LINEAR_PROBES = 9;
constexpr int PY_PERTURB_SHIFT = 5;
constexpr int PY_BATCH = 8;

__host__ __device__ __forceinline__ int64_t py_hash(int32_t k) { return k == -1 ? -2 : (int64_t)k; }

// A set under construction: table `t` of mask+1 slots, and a spare buffer of
// the same capacity that a resize rebuilds into.  `cap` bounds both.
struct DSet {
    int32_t *t;
    int32_t *spare;
    int64_t mask, fill, used;
    int64_t cap;
    bool overflow;
};

// read-only view of a stored table image
struct DView {
    const int32_t *t;
    int64_t mask, fill, used;
};

__device__ __forceinline__ void dset_init(DSet &s, int32_t *a, int32_t *b, int64_t cap) {
    s.t = a;
    s.spare = b;
    s.cap = cap;
    s.mask = PY_MINSIZE - 1;
    s.fill = s.used = 0;
    s.overflow = cap < PY_MINSIZE;
    for (int i = 0; i < PY_MINSIZE && i < cap; ++i) a[i] = PY_EMPTY;
}

__device__ __forceinline__ DView dset_view(const DSet &s) { return {s.t, s.mask, s.fill, s.used}; }

// The table size of a fresh set after n distinct adds (no deletions, so fill
// == used): set_add_entry resizes when fill * 5 >= mask * 3, to the smallest
// power of two > used * 4 (used * 2 past 50,000).  When every element is a
// small int below that size, each sits at its own slot (distinct home slots
// never collide), so the table is the elements in increasing order whatever
// the insertion order -- and a fresh set's pop() returns the smallest.
__host__ __device__ __forceinline__ int64_t py_size_after(int64_t n) {
    int64_t mask = PY_MINSIZE - 1;
    for (;;) {
        const int64_t thr = (mask * 3 + 4) / 5;   // the fill that triggers the next resize
        if (n < thr) return mask + 1;
        const int64_t minused = thr > 50000 ? thr * 2 : thr * 4;
        int64_t ns = PY_MINSIZE;
        while (ns <= minused) ns <<= 1;
        mask = ns - 1;
    }
}

__device__ __forceinline__ void py_insert_clean(int32_t *table, uint64_t mask, int32_t key) {
    const int64_t h = py_hash(key);
    uint64_t perturb = (uint64_t)h;
    uint64_t i = (uint64_t)h & mask;
    for (;;) {
        if (table[i] == PY_EMPTY) {
            table[i] = key;
            return;
        }
        if (i + PY_LINEAR_PROBES <= mask) {
            for (int j = 1; j <= PY_LINEAR_PROBES; ++j) {
                if (table[i + j] == PY_EMPTY) {
                    table[i + j] = key;
                    return;
                }
            }
        }
        perturb >>= PY_PERTURB_SHIFT;
        i = (i * 5 + 1 + perturb) & mask;
    }
}

// set_table_resize(so, minused)
__device__ __forceinline__ void py_resize(DSet &s, int64_t minused) {
    int64_t newsize = PY_MINSIZE;
    while (newsize <= minused) newsize <<= 1;
    if (newsize == PY_MINSIZE && s.mask == PY_MINSIZE - 1 && s.fill == s.used) return;   // small table, no dummies
    if (newsize > s.cap) {
        s.overflow = true;
        return;
    }
    int32_t *nt = s.spare;
    for (int64_t i = 0; i < newsize; ++i) nt[i] = PY_EMPTY;
    for (int64_t i0 = 0; i0 <= s.mask; i0 += PY_BATCH) {
        int32_t kb[PY_BATCH];
#pragma unroll
        for (int j = 0; j < PY_BATCH; ++j) kb[j] = s.t[i0 + j];
#pragma unroll
        for (int j = 0; j < PY_BATCH; ++j)
            if (kb[j] != PY_EMPTY && kb[j] != PY_DUMMY) py_insert_clean(nt, (uint64_t)(newsize - 1), kb[j]);
    }
    s.spare = s.t;
    s.t = nt;
    s.mask = newsize - 1;
    s.fill = s.used;
}

// set_add_entry(so, key, hash)
__device__ __forceinline__ void py_add(DSet &s, int32_t key) {
    if (s.overflow) return;
    const int64_t h = py_hash(key);
    const uint64_t mask = (uint64_t)s.mask;
    uint64_t i = (uint64_t)h & mask;
    int64_t slot = (int64_t)i;
    if (s.t[i] != PY_EMPTY) {
        int64_t freeslot = -1;
        uint64_t perturb = (uint64_t)h;
        for (;;) {
            int32_t k = s.t[i];
            if (k == key) return;                               // found_active
            if (k == PY_DUMMY) freeslot = (int64_t)i;
            bool hit_empty = false;
            if (i + PY_LINEAR_PROBES <= mask) {
                for (int j = 1; j <= PY_LINEAR_PROBES; ++j) {
                    k = s.t[i + j];
                    if (k == PY_EMPTY) {
                        slot = (int64_t)(i + j);
                        hit_empty = true;
                        break;
                    }
                    if (k == key) return;
                    if (k == PY_DUMMY) freeslot = (int64_t)(i + j);
                }
            }
            if (!hit_empty) {
                perturb >>= PY_PERTURB_SHIFT;
                i = (i * 5 + 1 + perturb) & mask;
                if (s.t[i] != PY_EMPTY) continue;
                slot = (int64_t)i;
            }
            // found_unused_or_dummy
            if (freeslot >= 0) {
                s.used++;
                s.t[freeslot] = key;
                return;
            }
            break;
        }
    }
    // found_unused
    s.fill++;
    s.used++;
    s.t[slot] = key;
    if ((uint64_t)s.fill * 5 < mask * 3) return;
    py_resize(s, s.used > 50000 ? s.used * 2 : s.used * 4);
}

// set_lookkey: slot of key or -1
__device__ __forceinline__ int64_t py_find(const DView &s, int32_t key) {
    const int64_t h = py_hash(key);
    const uint64_t mask = (uint64_t)s.mask;
    uint64_t perturb = (uint64_t)h;
    uint64_t i = (uint64_t)h & mask;
    for (;;) {
        const int probes = (i + PY_LINEAR_PROBES <= mask) ? PY_LINEAR_PROBES : 0;
        for (int j = 0; j <= probes; ++j) {
            const int32_t k = s.t[i + j];
            if (k == PY_EMPTY) return -1;
            if (k == key) return (int64_t)(i + j);
        }
        perturb >>= PY_PERTURB_SHIFT;
        i = (i * 5 + 1 + perturb) & mask;
    }
}

// set_merge(so, other)
__device__ __forceinline__ void py_merge(DSet &s, const DView &o) {
    if (s.overflow || o.used == 0) return;
    if ((s.fill + o.used) * 5 >= s.mask * 3) {
        py_resize(s, (s.used + o.used) * 2);
        if (s.overflow) return;
    }
    if (s.fill == 0 && s.mask == o.mask && o.fill == o.used) {   // empty target, same size, no dummies: copy
        for (int64_t i0 = 0; i0 <= o.mask; i0 += PY_BATCH) {
            int32_t kb[PY_BATCH];
#pragma unroll
            for (int j = 0; j < PY_BATCH; ++j) kb[j] = o.t[i0 + j];
#pragma unroll
            for (int j = 0; j < PY_BATCH; ++j) s.t[i0 + j] = kb[j];
        }
        s.fill = o.fill;
        s.used = o.used;
        return;
    }
    if (s.fill == 0) {   // empty target: insert_clean
        s.fill = o.used;
        s.used = o.used;
        for (int64_t i0 = 0; i0 <= o.mask; i0 += PY_BATCH) {
            int32_t kb[PY_BATCH];
#pragma unroll
            for (int j = 0; j < PY_BATCH; ++j) kb[j] = o.t[i0 + j];
#pragma unroll
            for (int j = 0; j < PY_BATCH; ++j)
                if (kb[j] != PY_EMPTY && kb[j] != PY_DUMMY) py_insert_clean(s.t, (uint64_t)s.mask, kb[j]);
        }
        return;
    }
    for (int64_t i0 = 0; i0 <= o.mask; i0 += PY_BATCH) {
        int32_t kb[PY_BATCH];
#pragma unroll
        for (int j = 0; j < PY_BATCH; ++j) kb[j] = o.t[i0 + j];
#pragma unroll
        for (int j = 0; j < PY_BATCH; ++j)
            if (kb[j] != PY_EMPTY && kb[j] != PY_DUMMY) py_add(s, kb[j]);
    }
}

// dst = a - {key}   (set_difference with a one-element right operand)
__device__ __forceinline__ void py_difference1(DSet &dst, const DView &a, int32_t key) {
    if ((a.used >> 2) > 1) {   // set_copy_and_difference: copy, then discard -> dummy
        py_merge(dst, a);
        if (dst.overflow) return;
        const int64_t at = py_find(dset_view(dst), key);
        if (at >= 0) {
            dst.t[at] = PY_DUMMY;
            dst.used--;
        }
        return;
    }
    for (int64_t i0 = 0; i0 <= a.mask; i0 += PY_BATCH) {
        int32_t kb[PY_BATCH];
#pragma unroll
        for (int j = 0; j < PY_BATCH; ++j) kb[j] = a.t[i0 + j];
#pragma unroll
        for (int j = 0; j < PY_BATCH; ++j)
            if (kb[j] != PY_EMPTY && kb[j] != PY_DUMMY && kb[j] != key) py_add(dst, kb[j]);
    }
}

// ---- Wave-cooperative forms, for tables in LDS.  Every lane of a wavefront
// calls them with the same arguments and keeps the same DSet fields.  A probe
// run (slot i, and the PY_LINEAR_PROBES after it when they fit) is read at
// once, one lane per slot, and settled by ballots in probe order -- the result
// of the serial probe loop above, in one LDS round trip per run instead of one
// per slot; table clears, copies and scans run across the lanes.  (A wave's
// LDS accesses complete in order, so a write by one lane is seen by the next
// read of any lane of the same wave.)

// lanes of the probe run at slot i
__device__ __forceinline__ uint64_t wpy_run(uint64_t i, uint64_t mask) {
    return (i + PY_LINEAR_PROBES <= mask) ? ((1ull << (PY_LINEAR_PROBES + 1)) - 1ull) : 1ull;
}

__device__ __forceinline__ void wpy_clear(int32_t *t, int64_t n) {
    for (int64_t x = __lane_id(); x < n; x += 64) t[x] = PY_EMPTY;
}

__device__ __forceinline__ void wpy_insert_clean(int32_t *table, uint64_t mask, int32_t key) {
    const uint32_t lane = __lane_id();
    const int64_t h = py_hash(key);
    uint64_t perturb = (uint64_t)h;
    uint64_t i = (uint64_t)h & mask;
    for (;;) {
        const bool in = (wpy_run(i, mask) >> lane) & 1ull;
        const int32_t k = in ? table[i + lane] : 1;
        const uint64_t em = __ballot(in && k == PY_EMPTY);
        if (em) {
            const uint32_t f = (uint32_t)__builtin_ctzll(em);
            if (lane == f) table[i + f] = key;
            return;
        }
        perturb >>= PY_PERTURB_SHIFT;
        i = (i * 5 + 1 + perturb) & mask;
    }
}

__device__ __forceinline__ void wpy_resize(DSet &s, int64_t minused) {
    int64_t newsize = PY_MINSIZE;
    while (newsize <= minused) newsize <<= 1;
    if (newsize == PY_MINSIZE && s.mask == PY_MINSIZE - 1 && s.fill == s.used) return;   // small table, no dummies
    if (newsize > s.cap) {
        s.overflow = true;
        return;
    }
    int32_t *nt = s.spare;
    wpy_clear(nt, newsize);
    const uint32_t lane = __lane_id();
    for (int64_t x0 = 0; x0 <= s.mask; x0 += 64) {   // old members in slot order
        const int32_t k = x0 + lane <= s.mask ? s.t[x0 + lane] : PY_EMPTY;
        uint64_t live = __ballot(k != PY_EMPTY && k != PY_DUMMY);
        while (live) {
            const int b = __builtin_ctzll(live);
            live &= live - 1;
            wpy_insert_clean(nt, (uint64_t)(newsize - 1), __builtin_amdgcn_readlane(k, b));
        }
    }
    s.spare = s.t;
    s.t = nt;
    s.mask = newsize - 1;
    s.fill = s.used;
}

// set_add_entry, wave-cooperative (see py_add: the LAST dummy before the first
// empty slot is reused)
__device__ __forceinline__ void wpy_add(DSet &s, int32_t key) {
    if (s.overflow) return;
    const uint32_t lane = __lane_id();
    const int64_t h = py_hash(key);
    const uint64_t mask = (uint64_t)s.mask;
    uint64_t i = (uint64_t)h & mask;
    uint64_t perturb = (uint64_t)h;
    int64_t freeslot = -1, slot;
    for (;;) {
        const bool in = (wpy_run(i, mask) >> lane) & 1ull;
        const int32_t k = in ? s.t[i + lane] : 1;
        const uint64_t em = __ballot(in && k == PY_EMPTY);
        const uint64_t km = __ballot(in && k == key);
        const uint64_t dm = __ballot(in && k == PY_DUMMY);
        const uint64_t stop = em | km;
        if (stop) {
            const int f = __builtin_ctzll(stop);
            if ((km >> f) & 1ull) return;                                   // found_active
            const uint64_t before = dm & ((1ull << f) - 1ull);
            if (before) freeslot = (int64_t)(i + 63 - __builtin_clzll(before));
            slot = (int64_t)(i + f);
            break;
        }
        if (dm) freeslot = (int64_t)(i + 63 - __builtin_clzll(dm));
        perturb >>= PY_PERTURB_SHIFT;
        i = (i * 5 + 1 + perturb) & mask;
    }
    if (freeslot >= 0) {   // found_unused_or_dummy: a dummy was probed first
        s.used++;
        if (lane == 0) s.t[freeslot] = key;
        return;
    }
    s.fill++;   // found_unused
    s.used++;
    if (lane == 0) s.t[slot] = key;
    if ((uint64_t)s.fill * 5 < mask * 3) return;
    wpy_resize(s, s.used > 50000 ? s.used * 2 : s.used * 4);
}

__device__ __forceinline__ int64_t wpy_find(const DView &s, int32_t key) {
    const uint32_t lane = __lane_id();
    const int64_t h = py_hash(key);
    const uint64_t mask = (uint64_t)s.mask;
    uint64_t perturb = (uint64_t)h;
    uint64_t i = (uint64_t)h & mask;
    for (;;) {
        const bool in = (wpy_run(i, mask) >> lane) & 1ull;
        const int32_t k = in ? s.t[i + lane] : 1;
        const uint64_t em = __ballot(in && k == PY_EMPTY);
        const uint64_t km = __ballot(in && k == key);
        const uint64_t stop = em | km;
        if (stop) {
            const int f = __builtin_ctzll(stop);
            return ((km >> f) & 1ull) ? (int64_t)(i + f) : -1;
        }
        perturb >>= PY_PERTURB_SHIFT;
        i = (i * 5 + 1 + perturb) & mask;
    }
}

__device__ __forceinline__ void wdset_init(DSet &s, int32_t *a, int32_t *b, int64_t cap) {
    s.t = a;
    s.spare = b;
    s.cap = cap;
    s.mask = PY_MINSIZE - 1;
    s.fill = s.used = 0;
    s.overflow = cap < PY_MINSIZE;
    wpy_clear(a, cap < PY_MINSIZE ? cap : PY_MINSIZE);
}

// set_merge, wave-cooperative
__device__ __forceinline__ void wpy_merge(DSet &s, const DView &o) {
    if (s.overflow || o.used == 0) return;
    if ((s.fill + o.used) * 5 >= s.mask * 3) {
        wpy_resize(s, (s.used + o.used) * 2);
        if (s.overflow) return;
    }
    const uint32_t lane = __lane_id();
    if (s.fill == 0 && s.mask == o.mask && o.fill == o.used) {   // empty target, same size, no dummies: copy
        for (int64_t x = lane; x <= o.mask; x += 64) s.t[x] = o.t[x];
        s.fill = o.fill;
        s.used = o.used;
        return;
    }
    const bool clean = s.fill == 0;   // empty target: insert_clean
    if (clean) {
        s.fill = o.used;
        s.used = o.used;
    }
    for (int64_t x0 = 0; x0 <= o.mask; x0 += 64) {   // o's members in slot order
        const int32_t k = x0 + lane <= o.mask ? o.t[x0 + lane] : PY_EMPTY;
        uint64_t live = __ballot(k != PY_EMPTY && k != PY_DUMMY);
        while (live) {
            const int b = __builtin_ctzll(live);
            live &= live - 1;
            const int32_t key = __builtin_amdgcn_readlane(k, b);
            if (clean)
                wpy_insert_clean(s.t, (uint64_t)s.mask, key);
            else
                wpy_add(s, key);
        }
    }
}

// dst = a - {key}, wave-cooperative
__device__ __forceinline__ void wpy_difference1(DSet &dst, const DView &a, int32_t key) {
    if ((a.used >> 2) > 1) {   // set_copy_and_difference: copy, then discard -> dummy
        wpy_merge(dst, a);
        if (dst.overflow) return;
        const int64_t at = wpy_find(dset_view(dst), key);
        if (at >= 0) {
            if (__lane_id() == 0) dst.t[at] = PY_DUMMY;
            dst.used--;
        }
        return;
    }
    const uint32_t lane = __lane_id();
    for (int64_t x0 = 0; x0 <= a.mask; x0 += 64) {
        const int32_t k = x0 + lane <= a.mask ? a.t[x0 + lane] : PY_EMPTY;
        uint64_t live = __ballot(k != PY_EMPTY && k != PY_DUMMY && k != key);
        while (live) {
            const int b = __builtin_ctzll(live);
            live &= live - 1;
            wpy_add(dst, __builtin_amdgcn_readlane(k, b));
        }
    }
}

}  // namespace satmi
