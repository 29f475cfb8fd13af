// knn_i8_dev.h -- device helpers of the int8 MFMA kernel (knn_i8.hip,
// k_dist_topk_i8), also included by the round-6 16x16x64 experiment
// (tools/probe/knn_i8x.hip): register-list insertion, min/max trees,
// LDS-DMA issue, the launch's block table in LDS.
#pragma once
#include "knn_device.h"

typedef int knn_v16i __attribute__((ext_vector_type(16)));
typedef int knn_v8i __attribute__((ext_vector_type(8)));

#define I8_INF 0x7fffffff        // empty list slot / no bound

// i8_norm_pos / i8_norm_word (the byte block's norm words): knn_device.h
__device__ __forceinline__ int i8_max3(int a, int b, int c)
{
    int r;
    asm("v_max3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ unsigned i8_min3u(unsigned a, unsigned b, unsigned c)
{
    unsigned r;
    asm("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// max of 32 values (a pair of m-blocks' accumulators): 16 v_max3
__device__ __forceinline__ int i8_max32(const int *v)
{
    int m[11];
#pragma unroll
    for (int y = 0; y < 10; y++) m[y] = i8_max3(v[3 * y], v[3 * y + 1], v[3 * y + 2]);
    m[10] = v[30] > v[31] ? v[30] : v[31];
    const int a = i8_max3(m[0], m[1], m[2]), b = i8_max3(m[3], m[4], m[5]);
    const int c = i8_max3(m[6], m[7], m[8]), d = i8_max3(m[9], m[10], a);
    return i8_max3(b, c, d);
}
// the largest of the 32 values below vm, or `none` if there is none: the
// unsigned minimum of vm - 1 - v.  Values below vm map to [0, span) and the
// rest to [2^32 - span, 2^32) with span < 2^31 (the lane's values span less
// than 2^31, above), so the two never mix
__device__ __forceinline__ int i8_next(const int *v, int vm, int none)
{
    const unsigned c = (unsigned)vm - 1u;
    unsigned m[11];
#pragma unroll
    for (int y = 0; y < 10; y++) m[y] = i8_min3u(c - (unsigned)v[3 * y], c - (unsigned)v[3 * y + 1],
                                                 c - (unsigned)v[3 * y + 2]);
    {
        const unsigned a = c - (unsigned)v[30], b = c - (unsigned)v[31];
        m[10] = a < b ? a : b;
    }
    const unsigned a = i8_min3u(m[0], m[1], m[2]), b = i8_min3u(m[3], m[4], m[5]);
    const unsigned cc = i8_min3u(m[6], m[7], m[8]), d = i8_min3u(m[9], m[10], a);
    const unsigned u = i8_min3u(b, cc, d);
    return (int)u < 0 ? none : (int)(c - u);
}

// Insert (d, id) into the ascending register list L (after equal keys: the
// lane's candidates arrive in row order, so ties keep the lower index,
// SURVEY F1); d >= L[KL-1] is a no-op.  Keys: L'[e] = med3(L[e-1], L[e], d)
// (one v_med3_i32, since L[e-1] <= L[e]); ids move where d < L[e-1].
__device__ __forceinline__ int i8_med3(int a, int b, int c)
{
    int r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
template <int KL>
__device__ __forceinline__ void i8_insert(int (&L)[KL], int (&I)[KL], int d, int id)
{
    // masks as (d - L) >> 31 (keys are >= 0, no overflow) and ids through
    // v_bfi: no v_cmp -> v_cndmask lane-mask hazard (2 wait states each)
    int m_hi = (d - L[KL - 1]) >> 31;   // -1 iff d < L[KL-1]
#pragma unroll
    for (int e = KL - 1; e > 0; e--) {
        const int m_lo = (d - L[e - 1]) >> 31;
        L[e] = i8_med3(L[e - 1], L[e], d);
        const int in = (m_hi & id) | (~m_hi & I[e]);
        I[e] = (m_lo & I[e - 1]) | (~m_lo & in);
        m_hi = m_lo;
    }
    L[0] = d < L[0] ? d : L[0];
    I[0] = (m_hi & id) | (~m_hi & I[0]);
}

// four LDS-DMA pieces (1 KiB each, consecutive LDS) under one M0 setup
__device__ __forceinline__ void bglds16x4(knn_v4i rsrc, unsigned v0, unsigned v1, unsigned v2, unsigned v3,
                                          unsigned lds_dst)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %6\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %2, %1, 0 offen lds\n\t"
                 "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %3, %1, 0 offen lds\n\t"
                 "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %4, %1, 0 offen lds\n\t"
                 "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %5, %1, 0 offen lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "s"(rsrc), "v"(v0), "v"(v1), "v"(v2), "v"(v3), "s"(__builtin_amdgcn_readfirstlane(lds_dst))
                 : "memory", "scc");
}

__device__ __forceinline__ void bglds16x2(knn_v4i rsrc, unsigned v0, unsigned v1, unsigned lds_dst)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %2, %1, 0 offen lds\n\t"
                 "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %3, %1, 0 offen lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "s"(rsrc), "v"(v0), "v"(v1), "s"(__builtin_amdgcn_readfirstlane(lds_dst))
                 : "memory", "scc");
}

// the same two pieces at byte offset soff (soffset: a chunk's offset inside
// its tile rows, so one descriptor serves the tile)
__device__ __forceinline__ void bglds16x2s(knn_v4i rsrc, unsigned v0, unsigned v1, unsigned soff, unsigned lds_dst)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %2, %1, %5 offen lds\n\t"
                 "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %3, %1, %5 offen lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "s"(rsrc), "v"(v0), "v"(v1), "s"(__builtin_amdgcn_readfirstlane(lds_dst)),
                   "s"(__builtin_amdgcn_readfirstlane(soff))
                 : "memory", "scc");
}

// one piece from the lanes of `lanes` only (exec set and restored inside
// the asm: no divergent region for the compiler to structure around the
// loop's live registers -- as a C++ branch at PF2's static norm-piece site it
// pushed the 25-K-step kernel into 242 VGPRs of spills)
__device__ __forceinline__ void bglds16m(knn_v4i rsrc, unsigned voff, unsigned lds_dst, unsigned long long lanes)
{
    unsigned keep;
    unsigned long long ex;
    asm volatile("s_mov_b64 %1, exec\n\ts_mov_b64 exec, %5\n\t"
                 "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %2, %3, 0 offen lds\n\ts_mov_b32 m0, %0\n\t"
                 "s_mov_b64 exec, %1"
                 : "=&s"(keep), "=&s"(ex)
                 : "v"(voff), "s"(rsrc), "s"(__builtin_amdgcn_readfirstlane(lds_dst)), "s"(lanes)
                 : "memory");
}

// buffer descriptor of a wave-uniform base, pinned to SGPRs (the base comes
// from the LDS block table through readfirstlane; under register pressure
// the allocator otherwise left the descriptor in VGPRs)
__device__ __forceinline__ knn_v4i i8_rsrc(const void *base)
{
    const knn_v4i r = knn_rsrc(base);
    return (knn_v4i){__builtin_amdgcn_readfirstlane(r.x), __builtin_amdgcn_readfirstlane(r.y), r.z, r.w};
}

// Block table of the launch in LDS (written once by thread 0 from the
// kernel argument with static indices, so the argument is never indexed
// dynamically and its SGPRs die after the copy).  Lookups happen once a
// block (wave-uniform LDS reads, made scalar by readfirstlane).
struct i8_tab_lds {
    unsigned long long ptr[KNN_I8_MAXBLK];
    unsigned long long nptr[KNN_I8_MAXBLK];
    long long base[KNN_I8_MAXBLK];
    int nc[KNN_I8_MAXBLK];
    int t0[KNN_I8_MAXBLK + 1];
    int nblk;
};
__device__ __forceinline__ int i8_rfl(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ long long i8_rfl64(long long v)
{
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)((unsigned long long)v >> 32));
    return (long long)(((unsigned long long)hi << 32) | lo);
}
// block of global tile t (t inside the launch's tiles)
// Block-table words of a taken block switch (the staging cursor's and the
// epilogue's): read through asm, so the compiler cannot hoist them out of
// the rarely taken branch.  Hoisted, the reads ran at every stage, and the
// lgkmcnt(0) their readfirstlane needs drained the A-fragment reads issued
// just before them.
__device__ __forceinline__ long long i8_tab64(const LDS_AS void *p)
{
    long long v;
    asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((unsigned)(size_t)p) : "memory");
    return i8_rfl64(v);
}
__device__ __forceinline__ int i8_tab32(const LDS_AS void *p)
{
    int v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((unsigned)(size_t)p) : "memory");
    return i8_rfl(v);
}
__device__ __forceinline__ int i8_blk_of(const LDS_AS i8_tab_lds *tab, int t)
{
    int b = 0;
    const int nb = i8_rfl(tab->nblk);
    for (int j = 1; j < nb; j++) b += t >= i8_rfl(tab->t0[j]) ? 1 : 0;
    return b;
}

