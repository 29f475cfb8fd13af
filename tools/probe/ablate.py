#!/usr/bin/env python3
"""Ablated copies of k_dist_topk_i8 for kbench8 (diagnostic; the product
source carries no hooks).  The patches target the one-deep chunk loop;
since round 6 the 8..25-K-step half-tile kernels (MNIST) run the two-deep
PF2 loop, which these patterns do not touch -- re-derive them before
ablating an MNIST-shaped launch.  Each variant is the product file with textual
patches applied, compiled into tools/probe/abl/libkbench8_<name>.so; time it
with  KB8_SO=tools/probe/abl/libkbench8_<name>.so python tools/probe/kbench8.py

  noepi        the per-tile epilogue replaced by an XOR sink of the
               accumulators (kept live; no survivor code compiled in)
  noepi_nodma  ... and no LDS-DMA staging (fragments read stale LDS)
  noepi_nodma_nobar  ... and no per-chunk barrier
  nodma        epilogue kept, staging removed (garbage keys: timing only)
  noepi_halfdma  one of each wave's two pieces a chunk (timing only)
  noepi_nowait   pieces issued, never waited for (racy: timing only)
  stamp        the product kernel plus per-workgroup wall-clock stamps
               (s_memrealtime at start, first chunk ready, loop done, end)
  tri          each query block scans only the tiles from its own rows on
               (the upper triangle of the self-join; its splits share that
               range): half the MFMA work (timing only, results partial)
  tricol       tri plus a column-direction filter in the epilogue (per-row
               thresholds from LDS against 2 acc - |q'|^2, ballot, no
               emission): the estimate of a symmetric kernel (timing only)
  sym          the self-join's symmetric launch (tools/probe/ksym.hip): an
               extra argument block; sy_mode 1 restricts each query block to
               the tiles from its own rows on (the first sy_qa blocks: from
               row 128 sy_qa on, row direction only) and adds the column
               direction on the tiles past the block's own: per-row
               thresholds w = lim - |r'|^2 staged as the (unused, long-row)
               init words, survivors appended to a per-workgroup region
  stagA_D / stagB_D  the product kernel with the first round's second-slot
               (A: blockIdx 256..511; B: odd XCD-local ids) workgroups
               started D x 1024 cycles late (an epilogue stagger between
               the two workgroups of a CU; timing only)
  count        the product kernel plus per-wave event counters (one vector
               atomic a wave and event, lane 0): groups past the init-word
               filter (all groups where it is off), groups whose exact keys
               were built, groups with exact survivors, extraction rounds,
               list merges (kbench8.py prints them per launch)
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "..", "..", "mpi-knn_amd", "csrc", "knn_i8.hip")

SINK = ("""            { int sk = 0;
#pragma unroll
              for (int bb = 0; bb < MB; bb++)
#pragma unroll
                for (int i = 0; i < 16; i++) sk ^= acc[0][bb][i];
              if (sk == 0x12345678) part_T[0] = 1.0; }
""")


COUNT_HDR = """__device__ unsigned long long kb8_cnt[8];
#define KB8_COUNT 1
#define KB8C(i) do { if ((threadIdx.x & 63) == 0) { unsigned long long one_ = 1ull; \\
    asm volatile("global_atomic_add_x2 %0, %1, off" :: "v"(&kb8_cnt[i]), "v"(one_) : "memory"); } } while (0)
"""


STAMP_HDR = """__device__ unsigned long long kb8_stamp[4 * 16384];
#define KB8_STAMP 1
#define KB8S(i) do { if (threadIdx.x == 0 && blockIdx.x < 16384) \\
    kb8_stamp[4 * blockIdx.x + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)
"""


def patch(s, name):
    if name.startswith("stag"):
        # stagA_D: the first round's second-slot workgroups (blockIdx 256..511:
        # breadth-first dispatch puts them beside 0..255 on the 256 CUs) start
        # D x 1024 cycles late, so the two workgroups of a CU -- and every
        # later pair, which inherits the offset through the freed slots --
        # reach their epilogues at different times; stagB_D: the odd
        # XCD-local workgroups of the first round instead (depth-first
        # placement: b and b + 8 on one CU).  Timing only; results unchanged.
        kind, d = name[4], int(name.split("_")[1])
        cond = ("(blockIdx.x >= 256u && blockIdx.x < 512u)" if kind == "A"
                else "(blockIdx.x < 512u && ((blockIdx.x >> 3) & 1u))")
        old = "    const int qb = blockIdx.x % nqb, split = blockIdx.x / nqb;\n"
        assert s.count(old) == 1
        s = s.replace(old, old + "    if (%s) { for (int z_ = 0; z_ < %d; z_++) __builtin_amdgcn_s_sleep(16); }\n" % (cond, d))
        return s
    if name == "stamp":
        # per-workgroup wall clock (100 MHz): start, first chunk ready, loop
        # done, end -- kbench8.py prints the spans of the last timed launch
        s = STAMP_HDR + s
        for old, new in (
                ("    const int qb = blockIdx.x % nqb, split = blockIdx.x / nqb;\n",
                 "    const int qb = blockIdx.x % nqb, split = blockIdx.x / nqb;\n    KB8S(0);\n"),
                ("        rdA(0, 0, acur);\n", "        KB8S(1);\n        rdA(0, 0, acur);\n"),
                ("        asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");   // no LDS-DMA left in flight\n",
                 "        asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");   // no LDS-DMA left in flight\n        KB8S(2);\n"),
                ("            atomicMin(qthr + myq[g], (unsigned long long)__double_as_longlong((double)thr[g]));\n    }\n    }\n}\n",
                 "            atomicMin(qthr + myq[g], (unsigned long long)__double_as_longlong((double)thr[g]));\n    }\n    }\n    KB8S(3);\n}\n")):
            assert s.count(old) == 1, old
            s = s.replace(old, new)
        return s
    if name == "count":
        s = COUNT_HDR + s
        for old, new in (
                ("            // exact keys of the group (slot words from the norm ring)\n",
                 "            KB8C(0);\n            // exact keys of the group (slot words from the norm ring)\n"),
                ("            int T = thr_v(g);\n            int vm = i8_max32(v);\n",
                 "            KB8C(1);\n            int T = thr_v(g);\n            int vm = i8_max32(v);\n"),
                ("            if (__ballot(vm >= T) == 0ull) continue;\n",
                 "            if (__ballot(vm >= T) == 0ull) continue;\n            KB8C(2);\n"),
                ("            do {\n                if (vm >= T) {\n",
                 "            do {\n                KB8C(3);\n                if (vm >= T) {\n"),
                ("        cnt[g] = 0;\n        refresh(g);\n",
                 "        cnt[g] = 0;\n        KB8C(4);\n        refresh(g);\n")):
            assert old in s, old
            s = s.replace(old, new)
        return s
    if name.startswith("tri"):
        old = ("    const int tb = ntiles / nsplit, tr = ntiles - tb * nsplit;\n"
               "    const int t_lo = split * tb + (split < tr ? split : tr);\n"
               "    const int t_hi = t_lo + tb + (split < tr ? 1 : 0);\n")
        assert s.count(old) == 1
        s = s.replace(old, "    const int tq0_ = (qb * QB) / TR, nt2_ = ntiles - tq0_;\n"
                           "    const int tb = nt2_ / nsplit, tr = nt2_ - tb * nsplit;\n"
                           "    const int t_lo = tq0_ + split * tb + (split < tr ? split : tr);\n"
                           "    const int t_hi = t_lo + tb + (split < tr ? 1 : 0);\n")
    if name == "tricol":
        old = "            int T = thr_v(g);\n            int vm = i8_max32(v);\n"
        assert s.count(old) == 1
        s = s.replace(old, """            {   // column direction: row r's threshold |r'|^2 - lim_r (init-word slots)
                int cm = 0;
#pragma unroll
                for (int bb = 0; bb < 2; bb++)
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const knn_v4i t4 = *(const LDS_AS knn_v4i *)(cn + NSEG / 2 + nofs(4 * h + 8 * (MB * rh + 2 * pr + bb) + j));
#pragma unroll
                        for (int i = 0; i < 4; i++) cm |= (2 * a[16 * bb + 4 * j + i] - qn[g] >= t4[i]) ? 1 : 0;
                    }
                colsink ^= (unsigned)__ballot(cm);
            }
""" + old)
        old = "    long c_base = 0;\n"
        assert s.count(old) == 1
        s = s.replace(old, "    unsigned colsink = 0;\n" + old)
        old = "#pragma unroll\n    for (int g = 0; g < QG; g++) merge(g);\n"
        assert s.count(old) == 1
        s = s.replace(old, old + "    if (colsink == 0x9e3779b9u) part_T[0] = 2.0;\n")
    if name.startswith("sym"):
        for old, new in (
                ("    unsigned long long *__restrict__ qthr, int uj, unsigned long long *__restrict__ qsum)\n{\n",
                 "    unsigned long long *__restrict__ qthr, int uj, unsigned long long *__restrict__ qsum,\n"
                 "    int sy_mode, int sy_qa, unsigned *__restrict__ sy_wcnt, uint4 *__restrict__ sy_buf, int sy_wcap)\n{\n"),
                ("                       KL != KNN_I8_KL_L ? qsum : nullptr);\n",
                 "                       KL != KNN_I8_KL_L ? qsum : nullptr, 0, 0, nullptr, nullptr, 0);\n"),
                ("    __shared__ __attribute__((aligned(16))) char smem[LDSB];\n",
                 "    __shared__ __attribute__((aligned(16))) char smem[LDSB];\n    __shared__ unsigned sy_n;\n"),
                ("    const int tb = ntiles / nsplit, tr = ntiles - tb * nsplit;\n"
                 "    const int t_lo = split * tb + (split < tr ? split : tr);\n"
                 "    const int t_hi = t_lo + tb + (split < tr ? 1 : 0);\n",
                 "    const int sy_t0 = sy_mode ? (qb < sy_qa ? sy_qa * 128 / TR : qb * QB / TR) : 0;\n"
                 "    const int sy_ct0 = (sy_mode && qb >= sy_qa) ? (qb + 1) * QB / TR : 0x7fffffff;\n"
                 "    const int sy_nt = ntiles - sy_t0;\n"
                 "    const int tb = sy_nt / nsplit, tr = sy_nt - tb * nsplit;\n"
                 "    const int t_lo = sy_t0 + split * tb + (split < tr ? split : tr);\n"
                 "    const int t_hi = t_lo + tb + (split < tr ? 1 : 0);\n"),
                ("    __syncthreads();\n\n    // ---- staging ----",
                 "    if (threadIdx.x == 0) sy_n = 0;\n    __syncthreads();\n\n    // ---- staging ----"),
                ("            // exact keys of the group (slot words from the norm ring)\n",
                 """            if (WPW / 4 == 4 && !SHORT && t >= sy_ct0) {   // (wave-uniform: the ballots below see every lane)   // (the 64-row long-row kernel)
                // column direction: candidate = this lane's query for the
                // tile's rows as queries; w = lim_r - |r'|^2 (init-word slots):
                // d^2 <= lim_r <=> 2 acc + w >= |q'|^2
                const LDS_AS char *cnh = cn + h * NSEG;   // nofs(4h + 8m + j) = (h + 2m) NSEG + 16 j
                int cmax = (int)0x80000000;
#pragma unroll
                for (int bb = 0; bb < 2; bb++)
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const knn_v4i w4 = *(const LDS_AS knn_v4i *)(cnh + (NSEG / 2 + 2 * (MB * rh + 2 * pr + bb) * NSEG + 16 * j));
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            const int x = 16 * bb + 4 * j + i;
                            int c = (int)((unsigned)a[x] * 2u + (unsigned)w4[i]);
                            if (masked) c = a[x] == A_NONE ? (int)0x80000000 : c;
                            cmax = c > cmax ? c : cmax;
                        }
                    }
                if (myq[g] >= nq) cmax = (int)0x80000000;   // padding queries are nobody's candidates
                if (__ballot(cmax >= qn[g]) != 0ull) {
                    // the lane's survivors as a mask, one LDS atomic a wave
                    // (the wave's total), each lane's slots from a bit-sliced
                    // prefix of the counts
                    unsigned cm = 0;
#pragma unroll
                    for (int bb = 0; bb < 2; bb++)
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            const knn_v4i w4 = *(const LDS_AS knn_v4i *)(cnh + (NSEG / 2 + 2 * (MB * rh + 2 * pr + bb) * NSEG + 16 * j));
#pragma unroll
                            for (int i = 0; i < 4; i++) {
                                const int x = 16 * bb + 4 * j + i;
                                const int c = (int)((unsigned)a[x] * 2u + (unsigned)w4[i]);
                                const bool ok = c >= qn[g] && !(masked && a[x] == A_NONE);
                                cm |= ok ? (1u << x) : 0u;
                            }
                        }
                    if (myq[g] >= nq) cm = 0u;
                    const int cl = __popc(cm);
                    int pre = 0, tot = 0;
#pragma unroll
                    for (int b = 0; b < 6; b++) {
                        const unsigned long long mb_ = __ballot((cl >> b) & 1);
                        pre += (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mb_ >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mb_, 0u)) << b;
                        tot += __popcll(mb_) << b;
                    }
                    unsigned base = 0;
                    if (lane == 0) base = atomicAdd(&sy_n, (unsigned)tot);
                    int o = __builtin_amdgcn_readfirstlane((int)base) + pre;
                    uint4 *dst = sy_buf + (size_t)blockIdx.x * sy_wcap;
                    if (cm != 0u) {
#pragma unroll
                        for (int bb = 0; bb < 2; bb++)
#pragma unroll
                            for (int j = 0; j < 4; j++) {
                                if (((cm >> (16 * bb + 4 * j)) & 15u) == 0u) continue;
                                const knn_v4i k4 = *(const LDS_AS knn_v4i *)(cnh + (2 * (MB * rh + 2 * pr + bb) * NSEG + 16 * j));
#pragma unroll
                                for (int i = 0; i < 4; i++) {
                                    const int x = 16 * bb + 4 * j + i;
                                    if ((cm >> x) & 1u) {
                                        // (d^2 == 0, an exact duplicate: stored as 0, dropped by the scatter)
                                        const int d2 = qn[g] - (k4[i] >> 5) - 2 * a[x];
                                        if (o < sy_wcap)
                                            dst[o] = make_uint4((unsigned)(idb + 32 * (2 * pr + bb) + 8 * j + i),
                                                                (unsigned)(d2 > 0 ? d2 : 0), (unsigned)gq[g], 0u);
                                        o++;
                                    }
                                }
                            }
                    }
                }
            }
            // exact keys of the group (slot words from the norm ring)
"""),
                ("            atomicMin(qthr + myq[g], (unsigned long long)__double_as_longlong((double)thr[g]));\n    }\n    }\n}\n",
                 "            atomicMin(qthr + myq[g], (unsigned long long)__double_as_longlong((double)thr[g]));\n    }\n    }\n"
                 "    if (sy_mode) {\n        __syncthreads();\n        if (threadIdx.x == 0) sy_wcnt[blockIdx.x] = sy_n;\n    }\n}\n"),
                # (no cross-split summaries: their registers go to the column path)
                ("    constexpr bool SUM = REREAD && KL == KNN_I8_KL_S && QG == 1;\n",
                 "    constexpr bool SUM = false;\n"),
                # (long rows: the norm is the slot word's alone -- the init
                # words carry the column thresholds here)
                ("        qn[g] = i8_norm_of(qnorms[i8_norm_pos(lq[g])], qnorms[q_rows_pad + i8_norm_pos(lq[g])]);\n",
                 "        qn[g] = -(qnorms[i8_norm_pos(lq[g])] >> 5);\n")):
            assert s.count(old) == 1, old[:70]
            s = s.replace(old, new)
        if name == "sym_nostore":   # survivors counted, not stored (timing only)
            old = "                                        if (o < sy_wcap)\n"
            assert s.count(old) == 1
            s = s.replace(old, "                                        if (o < 0)\n")
        return s
    if "noepi" in name:
        old = "            epilogue(t, acc, x);\n"
        assert old in s
        s = s.replace(old, SINK)
    if "nodma" in name:
        for old in ("        if constexpr (PW == 4) bglds16x4(i8_rsrc(s_row + s_coff), voff[0], voff[1], voff[2], voff[3], dst);\n"
                    "        else bglds16x2(i8_rsrc(s_row + s_coff), voff[0], voff[1], dst);\n",):
            assert old in s
            s = s.replace(old, "        (void)dst;\n")
    if "halfdma" in name:
        old = "        else bglds16x2(i8_rsrc(s_row + s_coff), voff[0], voff[1], dst);\n"
        assert old in s
        s = s.replace(old, "        else bglds16(i8_rsrc(s_row + s_coff), voff[0], dst);\n")
        old = 'asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NCH == 1 ? PW + 1 : PW) * (NST - 3)) : "memory");'
        assert old in s
        s = s.replace(old, 'asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NCH == 1 ? PW / 2 + 1 : PW / 2) * (NST - 3)) : "memory");')
    if "nowait" in name:
        old = 'asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NCH == 1 ? PW + 1 : PW) * (NST - 3)) : "memory");'
        assert old in s
        s = s.replace(old, '')
    if "rr4s" in name:   # one-chunk tiles re-read the shared bound every 4th tile
        old = "(NCH == 1 || (t & 1) == 0)"
        assert old in s
        s = s.replace(old, "((t & 3) == 0)")
    if "nosum" in name:  # no cross-split summaries
        old = "constexpr bool SUM = REREAD && KL == KNN_I8_KL_S && QG == 1;"
        assert old in s
        s = s.replace(old, "constexpr bool SUM = false;")
    if "norr" in name:   # no shared-bound re-read (nor summaries)
        old = "constexpr bool REREAD = KL != KNN_I8_KL_L;"
        assert old in s
        s = s.replace(old, "constexpr bool REREAD = false;")
    if "filtonly" in name:   # the init-word filter only, never the keys (timing only)
        old = "                if (__ballot(i8_max32(a) >= thr_a(g)) == 0ull) continue;\n"
        assert old in s
        s = s.replace(old, old + "                if (a[0] != 0x7fffffff) continue;\n")
    if "nobar" in name:
        old = "                            __builtin_amdgcn_s_barrier();   // B(x + 1)\n"
        assert old in s
        s = s.replace(old, "")
    return s


def main():
    names = sys.argv[1:] or ["noepi", "noepi_nodma", "noepi_nodma_nobar", "nodma"]
    out = os.path.join(HERE, "abl")
    os.makedirs(out, exist_ok=True)
    src = open(SRC).read()
    for name in names:
        f = os.path.join(out, "knn_i8_%s.hip" % name)
        open(f, "w").write(patch(src, name))
        so = os.path.join(out, "libkbench8_%s.so" % name)
        harness = "ksym.hip" if name.startswith("sym") else "kbench8.hip"
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-I" + os.path.join(HERE, "..", "..", "include"),
               "-I" + os.path.join(HERE, "..", "..", "mpi-knn_amd", "csrc"),
               "-mllvm", "-disable-promote-alloca-to-lds", '-DKB8_SRC="%s"' % f, "-o", so,
               os.path.join(HERE, harness)]
        subprocess.check_call(cmd)
        print(so)


if __name__ == "__main__":
    main()
