// knn_order.hip -- a cache-friendly query order for the GEMM-mode merge.
//
// k_merge re-ranks every candidate inside a query's certificate window by
// the reference's exact S (knn-serial.c:78-85), which reads the candidate's
// element row: ~k rows of n_pad elements a query, at random.  For a corpus
// larger than the 256 MB Infinity Cache (GIST-shaped 500K x 960 fp32: 1.9 GB,
// ~190 GB of row reads a merge) those reads come from HBM.  Queries that are
// near each other share most of their candidates, so merging them together
// serves the rows from L2 / the Infinity Cache.  The order is found from the
// distance kernel's partial lists alone: each query's list heads (its nearest
// candidate in every lane list) are edges of a near-neighbour graph; a few
// rounds of min-label propagation with pointer jumping label its connected
// pieces (clusters of the data), and a radix sort of (label, query) gives
// the merge's query permutation.  The merge's results do not depend on it.
#include "knn_device.h"
#include <hipcub/hipcub.hpp>

// labels start at the query itself; the graph's edges (the list heads
// that are queries of this search, as query indices, -1 otherwise) are
// gathered once into ORD_E words a query, so the rounds read 4 bytes an
// edge from a compact array instead of a 64-byte line of the lists
#define ORD_E 8
__global__ __launch_bounds__(256) void k_order_init(const int *__restrict__ part_i, int nl, int kl, int nq, int nq_pad,
                                                    int lpq, long long q_base, int *__restrict__ lab,
                                                    int *__restrict__ iota, int *__restrict__ edges)
{
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= nq) return;
    lab[q] = q;
    iota[q] = q;
    // ORD_E heads spread over the lists (every list when nl <= ORD_E)
#pragma unroll
    for (int e = 0; e < ORD_E; e++) {
        int cq = -1;
        if (e < nl) {
            const int j = (int)((long long)e * nl / ORD_E);
            const int s = j / lpq, g = j - s * lpq;
            const int c = part_i[(((size_t)s * nq_pad + q) * lpq + g) * kl];
            const long long d = (long long)c - q_base;
            cq = (c >= 0 && d >= 0 && d < nq) ? (int)d : -1;
        }
        edges[(size_t)e * nq + q] = cq;
    }
}

// one round: lab[q] = min(lab[q], lab of its edges, lab[lab[q]]) -- labels
// only fall and every thread writes its own query, so concurrent updates
// only speed it up
__global__ __launch_bounds__(256) void k_order_prop(const int *__restrict__ edges, int nq, int *__restrict__ lab)
{
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= nq) return;
    int m = lab[q];
#pragma unroll
    for (int e = 0; e < ORD_E; e++) {
        const int c = edges[(size_t)e * nq + q];
        if (c >= 0) {
            const int lc = lab[c];
            m = lc < m ? lc : m;
        }
    }
    const int lm = lab[m];
    m = lm < m ? lm : m;
    lab[q] = m;
}

// the work buffer: the sort's temporary storage, then the edge array
extern "C" size_t knn_order_tmp_bytes(int nq)
{
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const int *)nullptr, (int *)nullptr, (const int *)nullptr,
                                       (int *)nullptr, nq, 0, 32);
    return (bytes + 255) / 256 * 256 + (size_t)ORD_E * nq * sizeof(int);
}

// perm[0..nq): the queries grouped by label (work buffers lab, keys, iota of
// nq ints, tmp of knn_order_tmp_bytes(nq))
extern "C" int knn_launch_order(const int *part_i, int nsplit, int lpq, int kl, int nq, int nq_pad, long long q_base,
                                int rounds, int *lab, int *keys, int *iota, int *perm, void *tmp, size_t tmp_bytes,
                                void *stream)
{
    if (nq <= 0 || nsplit <= 0 || lpq <= 0 || kl <= 0) return KNN_ERR_INVALID;
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((unsigned)((nq + 255) / 256));
    size_t sb = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sb, (const int *)nullptr, (int *)nullptr, (const int *)nullptr,
                                             (int *)nullptr, nq, 0, 32);
    sb = (sb + 255) / 256 * 256;
    if (sb + (size_t)ORD_E * nq * sizeof(int) > tmp_bytes) return KNN_ERR_INVALID;
    int *edges = (int *)((char *)tmp + sb);
    hipLaunchKernelGGL(k_order_init, grid, dim3(256), 0, s, part_i, nsplit * lpq, kl, nq, nq_pad, lpq, q_base, lab,
                       iota, edges);
    for (int r = 0; r < rounds; r++) hipLaunchKernelGGL(k_order_prop, grid, dim3(256), 0, s, edges, nq, lab);
    int bits = 1;
    while (bits < 31 && (1 << bits) < nq) bits++;
    size_t tb = sb;
    if (hipcub::DeviceRadixSort::SortPairs(tmp, tb, lab, keys, iota, perm, nq, 0, bits, s) != hipSuccess)
        return KNN_ERR_HIP;
    return hipGetLastError() == hipSuccess ? KNN_OK : KNN_ERR_HIP;
}
