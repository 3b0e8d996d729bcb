// dpll_scan_access.h -- the hot LDS accesses of the clause-scan kernel by kind
// (included inside dpll_scan.hip's namespace, after SLds).
//
// Product builds: plain accesses, and the hooks dup_assign_store / dup_count
// compile to nothing.  Attribution builds only (`make variant
// VFLAGS=-DSATMI_DUP_<KIND>`): every LDS access of one kind is issued a second
// time with an effect-free operand (OR / ADD of an opaque zero, MIN of all
// ones, MAX of 0), so the search is unchanged and the rise of
// SQ_LDS_BANK_CONFLICT over the plain build is that kind's conflict cycles
// (profiles/r03/attr/).  Kinds: GATHER (literal-state byte gathers), CNT
// (counting-pass atomics), TS (snapshot stamp atomics), CLS (touched-clause
// word reads of the incremental rounds), ASSIGN (the batch assignment's stamp
// reads and state stores).
#pragma once

#if defined(SATMI_DUP_GATHER) || defined(SATMI_DUP_TS) || defined(SATMI_DUP_CLS) || defined(SATMI_DUP_ASSIGN) || \
    defined(SATMI_DUP_CNT)
__device__ __forceinline__ uint32_t opaque_zero() {
    uint32_t z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}
#endif

template <int K, typename C>
__device__ __forceinline__ uint32_t lv_get(const SLds<K, C> &S, uint32_t code) {
    uint32_t x = S.lv[code];
#ifdef SATMI_DUP_GATHER
    x |= (uint32_t)((const volatile uint8_t *)S.lv)[code] & opaque_zero();
#endif
    return x;
}

template <int K, typename C>
__device__ __forceinline__ void ts_stamp(const SLds<K, C> &S, uint32_t v, uint32_t st) {
    atomicMax(&S.ts[v], st);
#ifdef SATMI_DUP_TS
    atomicMax(&S.ts[v], st & opaque_zero());
#endif
}

template <int K, typename C>
__device__ __forceinline__ typename Pack<K>::W cls_at(const SLds<K, C> &S, uint32_t c) {
    typename Pack<K>::W w = S.cls[c];
#ifdef SATMI_DUP_CLS
    w |= ((const volatile typename Pack<K>::W *)S.cls)[c] & (typename Pack<K>::W)opaque_zero();
#endif
    return w;
}

// the stamp read of the batch assignment (propagate)
template <int K, typename C>
__device__ __forceinline__ uint32_t ts_first(const SLds<K, C> &S, uint32_t v) {
#ifdef SATMI_DUP_ASSIGN
    return S.ts[v] | (((const volatile uint32_t *)S.ts)[v] & opaque_zero());
#else
    return S.ts[v];
#endif
}

// the batch assignment's duplicated state store (attribution only)
template <int K, typename C>
__device__ __forceinline__ void dup_assign_store(const SLds<K, C> &S, bool first, uint32_t code) {
#ifdef SATMI_DUP_ASSIGN
    const uint32_t cd = first ? code : CODE_DUMMY;
    *(volatile uint16_t *)(S.lv + (cd & ~1u)) = (uint16_t)((cd & 1u) ? (LV_TRUE << 8) : LV_TRUE);
#else
    (void)S;
    (void)first;
    (void)code;
#endif
}

// the counting pass's duplicated atomic (attribution only), at the address
// cnt_inc uses: with packed counters (K = 3, 16-bit codes) a variable's two
// codes share the word cnt[code >> 1]
template <int K, typename C>
__device__ __forceinline__ void dup_count(const SLds<K, C> &S, uint32_t code) {
#ifdef SATMI_DUP_CNT
    atomicAdd(&S.cnt[(sizeof(C) == 2 && K == 3) ? (code >> 1) : code], opaque_zero());
#else
    (void)S;
    (void)code;
#endif
}
