"""mpiknn -- Python host mirror of libknn (include/knn.h) over ctypes.

The product is the C-ABI library ``mpi-knn_amd/lib/libknn.so`` (HIP kernels
for gfx950 + a C host engine).  This module only binds it: numpy arrays for
the host API, raw device pointers (e.g. ``torch.Tensor.data_ptr()``) for the
device-resident API used by the per-rank RCCL ring (``mpiknn.ring``) and by
bench.py.  There is no CPU fallback: if the library is missing, importing
this module raises.

Reference (yiapou13/mpi-knn): serial:L = knn-serial.c,
blk:L = mpi-knn-parallel_blocking.c, nb:L = mpi-knn-parallel_non_blocking.c.
"""
import atexit
import ctypes
import os
import sys
import weakref

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (KNN_LIB_PATH: another build of the same library, for A/B timing runs)
LIB_PATH = os.environ.get("KNN_LIB_PATH") or os.path.join(PKG_DIR, "lib", "libknn.so")

# knn_neighbour_t (blk:15-20): {double distance; int32 idx (1-based); int32 label}
NB_DTYPE = np.dtype([("distance", "<f8"), ("idx", "<i4"), ("label", "<i4")])

OK, ERR_INVALID, ERR_NOMEM, ERR_HIP, ERR_IO, ERR_FORMAT, ERR_UNSUPPORTED, ERR_NODEVICE, ERR_RCCL = range(9)
COLMAJOR, ROWMAJOR = 0, 1
F64, F32 = 0, 1
VOTE_SERIAL, VOTE_MPI, VOTE_MAJORITY = 0, 1, 2
MAX_K = 32          # KNN_MAX_K (fp64)
MAX_K_F32 = 128     # KNN_MAX_K_F32
META_DOUBLES = 8
STEP_LAG = 2        # KNN_STEP_LAG: a ring rotates STEP_LAG + 2 receive buffers
MODE_NAMES = {0: "int-exact", 1: "gemm+rerank", 2: "exact-scan"}

# every symbol include/knn.h declares (checked by tests/test_abi.py)
API_SYMBOLS = (
    "knn_strerror", "knn_load_mat", "knn_free", "knn_search", "knn_last_search_seconds",
    "knn_classify", "knn_block_bytes", "knn_block_meta_offset", "knn_block_pack",
    "knn_ctx_create", "knn_ctx_destroy", "knn_ctx_begin", "knn_ctx_step", "knn_ctx_end",
    "knn_ctx_rescan_step", "knn_ctx_rescan_end", "knn_search_packed", "knn_ctx_info",
    "knn_ctx_profile", "knn_block_bytes_dt", "knn_block_meta_offset_dt", "knn_block_pack_dt",
    "knn_ctx_create_dt", "knn_classify_device", "knn_search_mpi_compat",
    "knn_ctx_contraction_bits", "knn_wire_bytes", "knn_wire_ok", "knn_wire_pack",
    "knn_wire_unpack", "knn_shadow_bytes", "knn_shadow_norm_offset", "knn_shadow_pack", "knn_split_bytes", "knn_split_pack",
    "knn_ctx_shadow", "knn_ctx_step_shadow", "knn_ctx_begin_meta", "knn_ctx_shadow_bytes",
    "knn_ctx_shadow_pack", "knn_ctx_step_shadow_n", "knn_ctx_split", "knn_s8_block_bytes",
    "knn_s8_block_meta_offset", "knn_block_pack_s8", "knn_s8_spec_ok", "knn_ctx_begin_s8",
    "knn_ctx_attach_qblock", "knn_ctx_research_blocks", "knn_ctx_step_n", "knn_ctx_profile_merge",
    "knn_ctx_set_solo", "knn_ctx_search_meta",
)
DTYPES = {"f64": F64, "f32": F32, F64: F64, F32: F32}


class KnnError(RuntimeError):
    def __init__(self, status, what=""):
        self.status = status
        super().__init__("%s: %s (status %d)" % (what, strerror(status), status))


def _share_torch_runtime():
    """One HIP runtime per process.  PyTorch-ROCm ships its own
    libamdhip64/librccl with the same sonames as /opt/rocm's; if libknn
    pulled in the system copies first, torch would later load a second HIP
    runtime (no GPU found, heap corruption at exit).  Importing torch first
    (no device is touched) makes libknn bind to torch's copies; without
    torch the system ROCm libraries are used."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError("libknn not built: %s missing (run `make -C mpi-knn_amd` or "
                          "__graft_entry__.build())" % LIB_PATH)
    _share_torch_runtime()
    L = ctypes.CDLL(LIB_PATH)
    p, sz, i, d = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_double
    pp = ctypes.POINTER(ctypes.c_void_p)
    psz = ctypes.POINTER(ctypes.c_size_t)
    sig = {
        "knn_strerror": ([i], ctypes.c_char_p),
        "knn_load_mat": ([ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, pp, psz, psz, pp, psz], i),
        "knn_free": ([p], None),
        "knn_search": ([p, sz, sz, i, p, i, i, i, p], i),
        "knn_search_mpi_compat": ([p, sz, sz, i, p, i, i, p], i),
        "knn_last_search_seconds": ([], d),
        "knn_classify": ([p, sz, i, i, i, p, p, psz], i),
        "knn_block_bytes": ([sz, sz], sz),
        "knn_block_meta_offset": ([sz, sz], sz),
        "knn_block_pack": ([p, sz, sz, sz, p, sz, i, p], i),
        "knn_ctx_create": ([pp, i, sz, sz, sz, i], i),
        "knn_block_bytes_dt": ([sz, sz, i], sz),
        "knn_block_meta_offset_dt": ([sz, sz, i], sz),
        "knn_block_pack_dt": ([p, i, sz, sz, sz, p, i, sz, i, p], i),
        "knn_ctx_create_dt": ([pp, i, sz, sz, sz, i, i], i),
        "knn_ctx_destroy": ([p], i),
        "knn_classify_device": ([p, sz, i, i, i, p, sz, sz, p, p, p], i),
        "knn_ctx_begin": ([p, p, sz, sz, p, p], i),
        "knn_ctx_begin_meta": ([p, p, sz, sz, p, p, p], i),
        "knn_ctx_shadow_bytes": ([p, sz], sz),
        "knn_ctx_shadow_pack": ([p, p, p, sz, p], i),
        "knn_ctx_step": ([p, p, sz, sz, p], i),
        "knn_ctx_end": ([p, p, psz, p], i),
        "knn_ctx_rescan_step": ([p, p, sz, sz, p], i),
        "knn_ctx_rescan_end": ([p, p, p], i),
        "knn_search_packed": ([p, p, sz, p, p], i),
        "knn_ctx_info": ([p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)], i),
        "knn_ctx_contraction_bits": ([p], i),
        "knn_ctx_split": ([p], i),
        "knn_wire_bytes": ([sz, sz, i], sz),
        "knn_wire_ok": ([p], i),
        "knn_wire_pack": ([p, p, sz, sz, i, p], i),
        "knn_wire_unpack": ([p, p, sz, sz, i, p], i),
        "knn_shadow_bytes": ([sz, sz, i], sz),
        "knn_shadow_norm_offset": ([sz, sz], sz),
        "knn_shadow_pack": ([p, p, sz, sz, i, p], i),
        "knn_split_bytes": ([sz, sz], sz),
        "knn_split_pack": ([p, p, sz, sz, i, ctypes.c_double, p], i),
        "knn_ctx_shadow": ([p], i),
        "knn_ctx_step_shadow": ([p, p, sz, sz, p], i),
        "knn_ctx_step_shadow_n": ([p, i, pp, psz, psz, p], i),
        "knn_ctx_profile": ([p, i, ctypes.POINTER(d), ctypes.POINTER(d), ctypes.POINTER(i)], i),
        "knn_ctx_profile_merge": ([p, ctypes.POINTER(d), ctypes.POINTER(i), ctypes.POINTER(d)], i),
        "knn_ctx_set_solo": ([p, i], i),
        "knn_ctx_search_meta": ([p, ctypes.POINTER(d)], i),
        "knn_s8_block_bytes": ([sz, sz], sz),
        "knn_s8_block_meta_offset": ([sz, sz], sz),
        "knn_block_pack_s8": ([p, i, sz, sz, sz, p, i, sz, i, p], i),
        "knn_s8_spec_ok": ([p, sz, i], i),
        "knn_ctx_begin_s8": ([p, p, sz, sz, p, p, p], i),
        "knn_ctx_attach_qblock": ([p, p, sz], i),
        "knn_ctx_research_blocks": ([p, i, pp, psz, psz, p, psz, p], i),
        "knn_ctx_step_n": ([p, i, pp, psz, psz, p], i),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    return L


lib = _load()


def strerror(status):
    return lib.knn_strerror(status).decode()


def _check(rc, what):
    if rc != OK:
        raise KnnError(rc, what)


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


# ---------------------------------------------------------------- host API

def load_mat(path, xvar="train_X", lvar="train_labels"):
    """knn_load_mat (replaces matOpen/matGetVariable/mxGetPr, serial:40-52).

    Returns (X (m, n) float64 -- a C-ordered copy of the column-major data,
    labels (numel,) float64 or None)."""
    Xp, Lp = ctypes.c_void_p(), ctypes.c_void_p()
    m, n, nl = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
    rc = lib.knn_load_mat(path.encode(), xvar.encode(), lvar.encode() if lvar else None,
                          ctypes.byref(Xp), ctypes.byref(m), ctypes.byref(n),
                          ctypes.byref(Lp), ctypes.byref(nl))
    _check(rc, "knn_load_mat(%s)" % path)
    try:
        cnt = m.value * n.value
        flat = np.ctypeslib.as_array(ctypes.cast(Xp, ctypes.POINTER(ctypes.c_double)),
                                     shape=(max(cnt, 1),))[:cnt].copy()
        X = flat.reshape((n.value, m.value)).T.copy()  # column-major m x n
        labels = None
        if Lp.value:
            labels = np.ctypeslib.as_array(ctypes.cast(Lp, ctypes.POINTER(ctypes.c_double)),
                                           shape=(max(nl.value, 1),))[:nl.value].copy()
    finally:
        lib.knn_free(Xp)
        lib.knn_free(Lp)
    return X, labels


def search(X, k=30, ngpus=1, labels=None, layout="row", dtype="f64"):
    """knn_search: all-kNN with the reference's serial semantics.

    X: (m, n) float64.  layout="row" passes C order, "col" Fortran order (the
    .mat layout).  dtype "f64" (reference arithmetic) or "f32" (fp32 MFMA
    filter; exact kNN of the fp32-rounded points, include/knn.h).
    Returns (neighbours (m, k) NB_DTYPE, search seconds)."""
    X = np.asarray(X, dtype=np.float64)
    m, n = X.shape
    if layout == "col":
        buf, lay = np.asfortranarray(X), COLMAJOR
    else:
        buf, lay = np.ascontiguousarray(X), ROWMAJOR
    out = np.zeros((m, k), dtype=NB_DTYPE)
    lab = None if labels is None else np.ascontiguousarray(labels, dtype=np.float64)
    rc = lib.knn_search(_ptr(buf), m, n, lay, _ptr(lab), k, ngpus, DTYPES[dtype], _ptr(out))
    _check(rc, "knn_search")
    return out, lib.knn_last_search_seconds()


def search_mpi_compat(X, k=30, procs=2, labels=None, layout="row"):
    """knn_search_mpi_compat: the lists the reference MPI programs compute
    with `procs` ranks, bugs included (include/knn.h).  Returns
    (neighbours (procs*floor(m/procs), k) NB_DTYPE, search seconds)."""
    X = np.asarray(X, dtype=np.float64)
    m, n = X.shape
    if layout == "col":
        buf, lay = np.asfortranarray(X), COLMAJOR
    else:
        buf, lay = np.ascontiguousarray(X), ROWMAJOR
    R = m // procs if procs > 0 else 0
    out = np.zeros((max(procs * R, 1), k), dtype=NB_DTYPE)
    lab = None if labels is None else np.ascontiguousarray(labels, dtype=np.float64)
    rc = lib.knn_search_mpi_compat(_ptr(buf), m, n, lay, _ptr(lab), k, procs, _ptr(out))
    _check(rc, "knn_search_mpi_compat")
    return out[: procs * R], lib.knn_last_search_seconds()


def classify(nb, labels, nclasses=10, rule=VOTE_SERIAL):
    """knn_classify (serial:104-130 / blk:252-270).  Returns (pred, matches)."""
    nb = np.ascontiguousarray(nb)
    m, k = nb.shape
    lab = np.ascontiguousarray(labels, dtype=np.float64)
    pred = np.zeros(m, dtype=np.int32)
    matches = ctypes.c_size_t()
    rc = lib.knn_classify(_ptr(nb), m, k, nclasses, rule, _ptr(lab), _ptr(pred), ctypes.byref(matches))
    _check(rc, "knn_classify")
    return pred, matches.value


# ------------------------------------------------------ device-resident API

VOTE_MAX_CLASSES = 1024


def classify_device(d_nb, m, k, nclasses, rule, d_labels, nlabels, q_base=0, d_pred=None,
                    d_matches=None, stream=0):
    """knn_classify_device on device pointers (ints): fills the records'
    labels, writes m predictions to d_pred and the match count (uint64) to
    d_matches (both nullable)."""
    _check(lib.knn_classify_device(d_nb, m, k, nclasses, rule, d_labels, nlabels, q_base,
                                   d_pred or None, d_matches or None, stream or None),
           "knn_classify_device")

def block_bytes(cap, n, dtype="f64"):
    return lib.knn_block_bytes_dt(cap, n, DTYPES[dtype])


def block_meta_offset(cap, n, dtype="f64"):
    return lib.knn_block_meta_offset_dt(cap, n, DTYPES[dtype])


def wire_bytes(cap, n, dtype="f64"):
    return lib.knn_wire_bytes(cap, n, DTYPES[dtype])


def wire_ok(meta_host):
    """meta_host: the reduced block meta as a float64 numpy array."""
    m = np.ascontiguousarray(meta_host, dtype=np.float64)
    return bool(lib.knn_wire_ok(_ptr(m)))


def wire_pack(d_wire, d_block, cap, n, dtype="f64", stream=0):
    _check(lib.knn_wire_pack(d_wire, d_block, cap, n, DTYPES[dtype], stream or None), "knn_wire_pack")


def wire_unpack(d_block, d_wire, cap, n, dtype="f64", stream=0):
    _check(lib.knn_wire_unpack(d_block, d_wire, cap, n, DTYPES[dtype], stream or None),
           "knn_wire_unpack")


def shadow_bytes(cap, n, dtype="f64"):
    return lib.knn_shadow_bytes(cap, n, DTYPES[dtype])


def shadow_pack(d_sblock, d_block, cap, n, dtype="f64", stream=0):
    _check(lib.knn_shadow_pack(d_sblock, d_block, cap, n, DTYPES[dtype], stream or None),
           "knn_shadow_pack")


def split_bytes(cap, n):
    return lib.knn_split_bytes(cap, n)


def split_pack(d_dst, d_block, cap, n, dtype="f64", scale=1.0, stream=0):
    _check(lib.knn_split_pack(d_dst, d_block, cap, n, DTYPES[dtype], float(scale), stream or None),
           "knn_split_pack")


def block_pack(d_block, cap, rows, n, d_src, ld, layout, stream=0, dtype="f64", src_dtype="f64"):
    """knn_block_pack_dt on device pointers (ints).  layout COLMAJOR/ROWMAJOR;
    dtype = block element type, src_dtype = that of d_src."""
    _check(lib.knn_block_pack_dt(d_block, DTYPES[dtype], cap, rows, n, d_src, DTYPES[src_dtype],
                                 ld, layout, stream or None), "knn_block_pack_dt")


_live_contexts = weakref.WeakSet()


def s8_block_bytes(cap, n):
    return lib.knn_s8_block_bytes(cap, n)


def s8_block_meta_offset(cap, n):
    return lib.knn_s8_block_meta_offset(cap, n)


def block_pack_s8(d_sblock, cap, rows, n, d_src, ld, layout, stream=0, dtype="f64", src_dtype="f64"):
    """knn_block_pack_s8: the speculative byte block (x - 128) + meta straight
    from the source (valid for the search iff s8_spec_ok(reduced meta))."""
    _check(lib.knn_block_pack_s8(d_sblock, DTYPES[dtype], cap, rows, n, d_src, DTYPES[src_dtype], ld, layout,
                                 stream or None), "knn_block_pack_s8")


def s8_spec_ok(meta_host, n, dtype="f64"):
    m = np.ascontiguousarray(meta_host, dtype=np.float64)
    return bool(lib.knn_s8_spec_ok(_ptr(m), n, DTYPES[dtype]))


@atexit.register
def _close_all():
    # release device buffers while the HIP runtime is still up (its own
    # teardown runs after Python's atexit handlers)
    for c in list(_live_contexts):
        c.close()


class Context:
    """knn_ctx_t: running neighbour lists of nq queries on one device."""

    def __init__(self, device, nq, n, block_cap, k, dtype="f64"):
        self._h = ctypes.c_void_p()
        _check(lib.knn_ctx_create_dt(ctypes.byref(self._h), device, nq, n, block_cap, k,
                                     DTYPES[dtype]), "knn_ctx_create_dt")
        self.nq, self.n, self.block_cap, self.k, self.dtype = nq, n, block_cap, k, dtype
        _live_contexts.add(self)

    def close(self):
        if self._h:
            lib.knn_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        if not sys.is_finalizing():
            self.close()

    def begin(self, d_qblock, q_cap, q_base, d_meta, stream=0, h_meta=None):
        """knn_ctx_begin; with h_meta (host float64 copy of the reduced meta)
        knn_ctx_begin_meta, which needs no device read-back."""
        if h_meta is None:
            _check(lib.knn_ctx_begin(self._h, d_qblock, q_cap, q_base, d_meta, stream or None),
                   "knn_ctx_begin")
        else:
            hm = np.ascontiguousarray(h_meta, dtype=np.float64)
            _check(lib.knn_ctx_begin_meta(self._h, d_qblock, q_cap, q_base, d_meta, _ptr(hm),
                                          stream or None), "knn_ctx_begin_meta")

    def begin_s8(self, d_sblock, q_cap, q_base, d_meta, h_meta, stream=0):
        """knn_ctx_begin_s8: start from the query block's speculative byte block"""
        hm = np.ascontiguousarray(h_meta, dtype=np.float64)
        _check(lib.knn_ctx_begin_s8(self._h, d_sblock, q_cap, q_base, d_meta, _ptr(hm), stream or None),
               "knn_ctx_begin_s8")

    def attach_qblock(self, d_qblock, q_cap):
        _check(lib.knn_ctx_attach_qblock(self._h, d_qblock, q_cap), "knn_ctx_attach_qblock")

    def step(self, d_cblock, nc, c_base, stream=0):
        _check(lib.knn_ctx_step(self._h, d_cblock, nc, c_base, stream or None), "knn_ctx_step")

    def step_shadow(self, d_sblock, nc, c_base, stream=0):
        _check(lib.knn_ctx_step_shadow(self._h, d_sblock, nc, c_base, stream or None),
               "knn_ctx_step_shadow")

    def step_shadow_n(self, d_sblocks, ncs, c_bases, stream=0):
        """several resident shadow-form blocks in one step (int8 byte
        blocks: one fused distance launch per 8 blocks)"""
        nb = len(d_sblocks)
        ptrs = (ctypes.c_void_p * nb)(*d_sblocks)
        ncv = (ctypes.c_size_t * nb)(*ncs)
        cbv = (ctypes.c_size_t * nb)(*c_bases)
        _check(lib.knn_ctx_step_shadow_n(self._h, nb, ptrs, ncv, cbv, stream or None),
               "knn_ctx_step_shadow_n")

    def step_n(self, d_cblocks, ncs, c_bases, stream=0):
        """several resident element blocks in one step (split-filter
        searches: one fused distance launch and merge per 8 blocks)"""
        nb = len(d_cblocks)
        ptrs = (ctypes.c_void_p * nb)(*d_cblocks)
        ncv = (ctypes.c_size_t * nb)(*ncs)
        cbv = (ctypes.c_size_t * nb)(*c_bases)
        _check(lib.knn_ctx_step_n(self._h, nb, ptrs, ncv, cbv, stream or None), "knn_ctx_step_n")

    def research_blocks(self, d_sblocks, ncs, c_bases, d_out, stream=0):
        """A ring rank's int8 re-search of the queries end() left
        uncertified, against the byte blocks it holds (knn_ctx_research_blocks);
        returns the count the rescan pass still has to resolve."""
        nb = len(d_sblocks)
        ptrs = (ctypes.c_void_p * nb)(*d_sblocks)
        ncv = (ctypes.c_size_t * nb)(*ncs)
        cbv = (ctypes.c_size_t * nb)(*c_bases)
        u = ctypes.c_size_t(0)
        _check(lib.knn_ctx_research_blocks(self._h, nb, ptrs, ncv, cbv, d_out, ctypes.byref(u), stream or None),
               "knn_ctx_research_blocks")
        return u.value

    def shadow(self):
        """Shadow form of this search (after begin): 0 none, 1 fp16 shadow
        rows, 2 byte blocks of the int8 contraction."""
        return lib.knn_ctx_shadow(self._h)

    def shadow_bytes(self, cap):
        return lib.knn_ctx_shadow_bytes(self._h, cap)

    def shadow_pack(self, d_sblock, d_block, cap, stream=0):
        _check(lib.knn_ctx_shadow_pack(self._h, d_sblock, d_block, cap, stream or None),
               "knn_ctx_shadow_pack")

    def end(self, d_out, stream=0):
        u = ctypes.c_size_t()
        _check(lib.knn_ctx_end(self._h, d_out, ctypes.byref(u), stream or None), "knn_ctx_end")
        return u.value

    def rescan_step(self, d_cblock, nc, c_base, stream=0):
        _check(lib.knn_ctx_rescan_step(self._h, d_cblock, nc, c_base, stream or None),
               "knn_ctx_rescan_step")

    def rescan_end(self, d_out, stream=0):
        _check(lib.knn_ctx_rescan_end(self._h, d_out, stream or None), "knn_ctx_rescan_end")

    def search_packed(self, d_block, m, d_out, stream=0):
        _check(lib.knn_search_packed(self._h, d_block, m, d_out, stream or None),
               "knn_search_packed")

    def profile(self, enable=-1):
        """knn_ctx_profile: (dist_ms, merge_ms, launches); enable 1 resets+starts."""
        dm, mm, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        _check(lib.knn_ctx_profile(self._h, enable, ctypes.byref(dm), ctypes.byref(mm),
                                   ctypes.byref(n)), "knn_ctx_profile")
        return dm.value, mm.value, n.value

    def set_solo(self, on):
        """knn_ctx_set_solo: one-step searches (P = 1) on the caller's stream."""
        _check(lib.knn_ctx_set_solo(self._h, 1 if on else 0), "knn_ctx_set_solo")

    def search_meta(self):
        """knn_ctx_search_meta: the meta the last search's kernels read."""
        out = (ctypes.c_double * META_DOUBLES)()
        _check(lib.knn_ctx_search_meta(self._h, out), "knn_ctx_search_meta")
        return np.frombuffer(out, dtype=np.float64).copy()

    def profile_merge(self):
        """knn_ctx_profile_merge: (merge kernel ms, merge launches,
        algorithmic bytes) over the profiled steps."""
        mm, n, b = ctypes.c_double(), ctypes.c_int(), ctypes.c_double()
        _check(lib.knn_ctx_profile_merge(self._h, ctypes.byref(mm), ctypes.byref(n), ctypes.byref(b)),
               "knn_ctx_profile_merge")
        return mm.value, n.value, b.value

    def info(self):
        mode, splits = ctypes.c_int(), ctypes.c_int()
        _check(lib.knn_ctx_info(self._h, ctypes.byref(mode), ctypes.byref(splits)), "knn_ctx_info")
        return mode.value, splits.value

    def contraction_bits(self):
        """64 / 32, 16 (exact fp16 MFMA, or the split fp16 filter) or 8 (exact
        int8 MFMA) for this search."""
        return lib.knn_ctx_contraction_bits(self._h)

    def split(self):
        """1 when this search filters with the split fp16 contraction."""
        return lib.knn_ctx_split(self._h)
