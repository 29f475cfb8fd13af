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

__global__ __launch_bounds__(256) void k_order_init(int *__restrict__ lab, int *__restrict__ iota, int nq)
{
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q < nq) {
        lab[q] = q;
        iota[q] = q;
    }
}

// one round: lab[q] = min(lab[q], lab of every list head that is a query
// of this search, lab[lab[q]]) -- labels only fall, every thread writes its
// own query, so concurrent rounds of other threads only speed it up
__global__ __launch_bounds__(256) void k_order_prop(const int *__restrict__ part_i, int nl, int kl, int nq,
                                                    int nq_pad, int lpq, long long q_base, int *__restrict__ lab)
{
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= nq) return;
    int m = lab[q];
    for (int j = 0; j < nl; j++) {
        const int s = j / lpq, g = j - s * lpq;
        const int c = part_i[(((size_t)s * nq_pad + q) * lpq + g) * kl];
        const long long cq = (long long)c - q_base;
        if (c >= 0 && cq >= 0 && cq < nq) {
            const int lc = lab[cq];
            m = lc < m ? lc : m;
        }
    }
    const int lm = lab[m];
    m = lm < m ? lm : m;
    lab[q] = m;
}

extern "C" size_t knn_order_tmp_bytes(int nq)
{
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const int *)nullptr, (int *)nullptr, (const int *)nullptr,
                                       (int *)nullptr, nq, 0, 32);
    return bytes;
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
    hipLaunchKernelGGL(k_order_init, grid, dim3(256), 0, s, lab, iota, nq);
    for (int r = 0; r < rounds; r++)
        hipLaunchKernelGGL(k_order_prop, grid, dim3(256), 0, s, part_i, nsplit * lpq, kl, nq, nq_pad, lpq, q_base,
                           lab);
    int bits = 1;
    while (bits < 31 && (1 << bits) < nq) bits++;
    size_t tb = tmp_bytes;
    if (hipcub::DeviceRadixSort::SortPairs(tmp, tb, lab, keys, iota, perm, nq, 0, bits, s) != hipSuccess)
        return KNN_ERR_HIP;
    return hipGetLastError() == hipSuccess ? KNN_OK : KNN_ERR_HIP;
}
