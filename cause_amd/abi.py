"""ctypes binding of include/causeweave.h (libcauseweave.so).

This is the Python side of the drop-in boundary: the same C entry points a JVM
shim binds through Panama/JNA.  There is no fallback: if the
HIP library is missing or fails, calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
import re
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# (CW_LIB: another build of the same library, for A/B timing runs on one box)
LIB_PATH = os.environ.get("CW_LIB") or os.path.join(_HERE, "libcauseweave.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "causeweave.h")

CW_MEM_HOST, CW_MEM_DEVICE = 0, 1
STATUS_ROOT, STATUS_DUP, STATUS_ORPHAN, STATUS_NON_LAMPORT, STATUS_INTERNAL = 1, 2, 4, 8, 32
STATUS_MAP_KEY = 16
STATUS_WEFT = 64
STATUS_KEY_RANGE = 128
STATUS_UNWOVEN = 256  # reserved: never set since round 4 (include/causeweave.h)
NIL32 = 0xFFFFFFFF
K32_RESERVED = 0xFFFFFFF0     # K32 words from here up = the top 16 K64 values (CW_NIL, ...)


def narrow_k32(id_key, cause_key):
    """K64 packed keys -> the K32 words of cw_weave_lists_k32.  The top 16 K64
    values (nil, the non-id cause) map to the top 16 K32 words; every other key
    must be below K32_RESERVED (ValueError otherwise)."""
    out = []
    for a in (id_key, cause_key):
        a = np.ascontiguousarray(a, np.uint64)
        top = a >= np.uint64((1 << 64) - 16)
        rest = np.where(top, np.uint64(0), a)
        if rest.size and int(rest.max()) >= K32_RESERVED:
            raise ValueError("keys do not fit K32 (every id and cause below 2^32 - 16)")
        out.append(a.astype(np.uint32))     # the top 16 keep their low 32 bits
    return out[0], out[1]


class CwListBatch(C.Structure):
    _fields_ = [("n_docs", C.c_uint64), ("doc_offsets", C.POINTER(C.c_uint64)),
                ("id_key", C.c_void_p), ("cause_key", C.c_void_p), ("kind", C.c_void_p),
                ("key_bits", C.c_uint32), ("ts_shift", C.c_uint32), ("site_shift", C.c_uint32),
                ("site_bits", C.c_uint32)]


class CwListBatchK32(C.Structure):
    _fields_ = [("n_docs", C.c_uint64), ("doc_offsets", C.POINTER(C.c_uint64)),
                ("id_key", C.c_void_p), ("cause_key", C.c_void_p), ("kind", C.c_void_p),
                ("key_bits", C.c_uint32), ("ts_shift", C.c_uint32), ("site_shift", C.c_uint32),
                ("site_bits", C.c_uint32), ("perm16", C.c_uint32)]


class CwListBatchK128(C.Structure):
    _fields_ = [("n_docs", C.c_uint64), ("doc_offsets", C.POINTER(C.c_uint64)),
                ("id_key", C.c_void_p), ("cause_key", C.c_void_p), ("kind", C.c_void_p)]


class CwListResult(C.Structure):
    _fields_ = [("weave_perm", C.c_void_p), ("visible_bits", C.c_void_p),
                ("visible_count", C.c_void_p), ("max_ts", C.c_void_p), ("status", C.c_void_p),
                ("yarn_perm", C.c_void_p)]


class CwMapBatch(C.Structure):
    _fields_ = [("n_colls", C.c_uint64), ("coll_offsets", C.POINTER(C.c_uint64)),
                ("id_key", C.c_void_p), ("cause", C.c_void_p), ("cause_is_id", C.c_void_p),
                ("kind", C.c_void_p), ("key_bits", C.c_uint32), ("token_bits", C.c_uint32)]


class CwMapResult(C.Structure):
    _fields_ = [("cap_segs", C.c_uint64), ("n_segs", C.c_uint64), ("seg_offsets", C.c_void_p),
                ("seg_coll", C.c_void_p), ("seg_key", C.c_void_p), ("seg_active", C.c_void_p),
                ("seg_perm", C.c_void_p), ("status", C.c_void_p)]


class CwMergeBatch(C.Structure):
    _fields_ = [("a", CwListBatch), ("a_value", C.c_void_p), ("b", CwListBatch),
                ("b_value", C.c_void_p)]


class CwMergeResult(C.Structure):
    _fields_ = [("merged_offsets", C.POINTER(C.c_uint64)), ("merged_src", C.c_void_p),
                ("weave", CwListResult)]


class CwWeftBatch(C.Structure):
    _fields_ = [("nodes", CwListBatch), ("cut", C.POINTER(C.c_uint64))]


class CwWeftResult(C.Structure):
    _fields_ = [("kept_offsets", C.POINTER(C.c_uint64)), ("kept_src", C.c_void_p),
                ("weave", CwListResult)]


class CwRankedList(C.Structure):
    _fields_ = [("n", C.c_uint64), ("par", C.c_void_p), ("kind", C.c_void_p), ("val", C.c_void_p)]


class CwLinkedList(C.Structure):
    _fields_ = [("n", C.c_uint64), ("succ", C.c_void_p), ("thr", C.c_void_p), ("val", C.c_void_p)]


# the distributed tree's building blocks (include/causeweave.h, dist.hip):
# argument types after the context
_DIST_ARGS = {
    "check": "U64 U32 P P P", "eff": "U64 U32 P P P", "climb": "U64 U32 P P P U64 P",
    "pending": "P U64 P P", "gkey": "P P U64 P", "runs": "P P U64 U32 P P P P",
    "rkey": "P U64 P", "link": "P P U64 P U32 U64 P P P", "put": "P P U64 U32 U64 P",
    "thr": "P U64 U32 P", "succ": "P P P U64 U32 P",
    "rs_rulers": "P P U64 U32 U32 U32 P P P", "rs_walk": "P U64 P U32 P P U64 U32 P P P P P P",
    "rs_top": "P U64 U64 P P", "rs_pos": "P P P P U64 P P", "rs_emit": "P U64 U32 U64 P P P P",
}


class CwKernelStat(C.Structure):
    _fields_ = [("name", C.c_char * 48), ("launches", C.c_uint64), ("total_ms", C.c_double),
                ("bytes_alg", C.c_double)]


_LIB = None


class WeaveError(RuntimeError):
    pass


def header_functions():
    """Names of every function declared in include/causeweave.h."""
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(cw_\w+)\s*\(", src, re.M)))


def build_id() -> str:
    """The loaded library's build id (a hash of its sources, see Makefile)."""
    return lib().cw_build_id().decode()


def _share_torch_hip_runtime():
    """One HIP runtime per process.  PyTorch-ROCm ships its own libamdhip64
    (soname libamdhip64.so.7, NEEDED by torch as plain "libamdhip64.so"): when
    this library loaded /opt/rocm's copy first, a later `import torch` loads a
    second runtime, which then sees no GPU, and device pointers / streams could
    not be shared.  Loading torch's copy first (without importing torch) makes
    libcauseweave.so bind to it (same soname) and torch reuse it (same path).
    CW_HIP_RUNTIME=system keeps /opt/rocm's runtime."""
    if os.environ.get("CW_HIP_RUNTIME") == "system":
        return
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    path = os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so")
    if os.path.exists(path):
        C.CDLL(path, mode=C.RTLD_GLOBAL)


def lib():
    """Load libcauseweave.so (raises if it was not built)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise WeaveError(f"{LIB_PATH} is missing: build it (python -c "
                             "'import __graft_entry__ as g; g.build()' or `make`)")
        _share_torch_hip_runtime()
        L = C.CDLL(LIB_PATH)
        L.cw_abi_version.restype = C.c_int
        L.cw_build_id.restype = C.c_char_p
        L.cw_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
        L.cw_ctx_create.restype = C.c_int
        L.cw_ctx_destroy.argtypes = [C.c_void_p]
        L.cw_ctx_destroy.restype = None
        L.cw_last_error.argtypes = [C.c_void_p]
        L.cw_last_error.restype = C.c_char_p
        L.cw_ctx_set_stream.argtypes = [C.c_void_p, C.c_void_p]
        L.cw_ctx_set_async.argtypes = [C.c_void_p, C.c_int]
        L.cw_ctx_set_profiling.argtypes = [C.c_void_p, C.c_int]
        L.cw_ctx_set_profile_only.argtypes = [C.c_void_p, C.c_char_p]
        L.cw_get_kernel_stats.argtypes = [C.c_void_p, C.POINTER(CwKernelStat), C.c_int]
        L.cw_reset_kernel_stats.argtypes = [C.c_void_p]
        L.cw_get_counter.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_uint64)]
        L.cw_get_counter.restype = C.c_int
        L.cw_weave_lists.argtypes = [C.c_void_p, C.POINTER(CwListBatch), C.POINTER(CwListResult),
                                     C.c_int]
        L.cw_weave_lists.restype = C.c_int
        L.cw_weave_lists_k32.argtypes = [C.c_void_p, C.POINTER(CwListBatchK32),
                                         C.POINTER(CwListResult), C.c_int]
        L.cw_weave_lists_k32.restype = C.c_int
        L.cw_weave_lists_k128.argtypes = [C.c_void_p, C.POINTER(CwListBatchK128),
                                          C.POINTER(CwListResult), C.c_int]
        L.cw_weave_lists_k128.restype = C.c_int
        L.cw_weave_maps.argtypes = [C.c_void_p, C.POINTER(CwMapBatch), C.POINTER(CwMapResult),
                                    C.c_int]
        L.cw_weave_maps.restype = C.c_int
        L.cw_merge_lists.argtypes = [C.c_void_p, C.POINTER(CwMergeBatch),
                                     C.POINTER(CwMergeResult), C.c_int]
        L.cw_merge_lists.restype = C.c_int
        L.cw_weft_lists.argtypes = [C.c_void_p, C.POINTER(CwWeftBatch), C.POINTER(CwWeftResult),
                                    C.c_int]
        L.cw_weft_lists.restype = C.c_int
        P, U64, U32 = C.c_void_p, C.c_uint64, C.c_uint32
        L.cw_sort_keys.argtypes = [P, P, U64, U32, P, P]
        L.cw_lookup_keys.argtypes = [P, P, U64, P, U64, U32, P, P]
        L.cw_partition_keys.argtypes = [P, P, U64, P, U32, P, P]
        L.cw_partition_keys_dev.argtypes = [P, P, U64, P, U32, P, P]
        L.cw_gather.argtypes = [P, P, P, U64, U32, P]
        L.cw_scatter32.argtypes = [P, P, P, U64, P]
        L.cw_weave_ranked.argtypes = [P, C.POINTER(CwRankedList), C.POINTER(CwListResult)]
        L.cw_weave_linked.argtypes = [P, C.POINTER(CwLinkedList), C.POINTER(CwListResult)]
        L.cw_sort_keys32.argtypes = [P, P, U64, U32, P, P]
        L.cw_sort_keys32.restype = C.c_int
        for f in ("cw_sort_keys", "cw_lookup_keys", "cw_partition_keys", "cw_partition_keys_dev",
                  "cw_gather", "cw_scatter32",
                  "cw_weave_ranked", "cw_weave_linked"):
            getattr(L, f).restype = C.c_int
        for f, a in _DIST_ARGS.items():
            fn = getattr(L, "cw_dist_" + f)
            fn.argtypes = [P] + [{"P": P, "U64": U64, "U32": U32}[x] for x in a.split()]
            fn.restype = C.c_int
        _LIB = L
    return _LIB


@dataclass
class ListResult:
    weave_perm: np.ndarray     # uint32[N] doc-local input index per weave position
    visible_bits: np.ndarray   # uint32[(N+31)//32]
    visible_count: np.ndarray  # uint32[D]
    max_ts: np.ndarray         # uint64[D]
    status: np.ndarray         # uint32[D]
    yarn_perm: np.ndarray | None

    def visible(self) -> np.ndarray:
        """uint8[N]: 1 where the global weave position renders."""
        n = len(self.weave_perm)
        b = np.unpackbits(self.visible_bits.view(np.uint8), bitorder="little")
        return b[:n]


@dataclass
class MergeResult:
    """Union of two node bags per document and its weave (cw_merge_lists)."""
    offsets: np.ndarray      # uint64[D+1] merged documents
    src: np.ndarray          # uint32[M] merged nodes in id order: < na_d -> a, else b (- na_d)
    weave: ListResult        # weave_perm holds doc-local merged indices (into src)

    def weave_src(self) -> np.ndarray:
        """uint32[M]: source index (as in src) of every weave position."""
        out = np.empty_like(self.weave.weave_perm)
        for d in range(len(self.offsets) - 1):
            lo, hi = int(self.offsets[d]), int(self.offsets[d + 1])
            out[lo:hi] = self.src[lo:hi][self.weave.weave_perm[lo:hi]]
        return out


@dataclass
class MapResult:
    """Key weaves of a batch of maps, per collection in ascending key-token order."""
    seg_offsets: np.ndarray  # uint64[S+1] into seg_perm
    seg_coll: np.ndarray     # uint32[S]
    seg_key: np.ndarray      # uint64[S] key token
    seg_active: np.ndarray   # int64[S] collection-local input index, -1 = ::blank
    seg_perm: np.ndarray     # uint32[N+S] root (UINT32_MAX) then input indices, weave order
    status: np.ndarray       # uint32[n_colls]

    def key_weave(self, s):
        return self.seg_perm[int(self.seg_offsets[s]):int(self.seg_offsets[s + 1])]


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


class Weaver:
    """A weave context on one HIP device (cw_ctx)."""

    def __init__(self, device: int = 0):
        self._L = lib()
        h = C.c_void_p()
        rc = self._L.cw_ctx_create(device, C.byref(h))
        if rc != 0 or not h:
            raise WeaveError(f"cw_ctx_create(device={device}) failed: no usable HIP device")
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            self._L.cw_ctx_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            raise WeaveError(f"{what}: {self._L.cw_last_error(self._h).decode()}")

    def set_stream(self, stream_ptr):
        self._check(self._L.cw_ctx_set_stream(self._h, C.c_void_p(stream_ptr)), "set_stream")

    def set_async(self, on: bool):
        self._check(self._L.cw_ctx_set_async(self._h, int(on)), "set_async")

    def set_profiling(self, on: bool):
        self._check(self._L.cw_ctx_set_profiling(self._h, int(on)), "set_profiling")

    def set_profile_only(self, kernel: str | None):
        """Per-kernel events for this kernel stat name only (None: every kernel)."""
        self._check(self._L.cw_ctx_set_profile_only(self._h, kernel.encode() if kernel else None),
                    "set_profile_only")

    def kernel_stats(self):
        n = self._L.cw_get_kernel_stats(self._h, None, 0)
        arr = (CwKernelStat * max(n, 1))()
        self._L.cw_get_kernel_stats(self._h, arr, n)
        return {a.name.decode(): (a.launches, a.total_ms, a.bytes_alg) for a in arr[:n]}

    def reset_kernel_stats(self):
        self._L.cw_reset_kernel_stats(self._h)

    def counter(self, name: str) -> int:
        """A diagnostic counter of the last call (cw_get_counter; waits for the
        stream): "continued_sublists" = walk-slot overflows of the last HBM walk."""
        v = C.c_uint64(0)
        self._check(self._L.cw_get_counter(self._h, name.encode(), C.byref(v)), "get_counter")
        return int(v.value)

    @staticmethod
    def _batch(offsets, id_ptr, cause_ptr, kind_ptr, layout, key_bits=None):
        off = np.ascontiguousarray(offsets, np.uint64)
        b = CwListBatch()
        b.n_docs = len(off) - 1
        b.doc_offsets = off.ctypes.data_as(C.POINTER(C.c_uint64))
        b.id_key, b.cause_key, b.kind = id_ptr, cause_ptr, kind_ptr
        b.key_bits = layout.key_bits if key_bits is None else key_bits
        b.ts_shift = layout.ts_shift
        b.site_shift = layout.site_shift
        b.site_bits = layout.site_bits
        return b, off

    def weave_lists(self, offsets, id_key, cause_key, kind, layout, yarns=True,
                    key_bits=None) -> ListResult:
        """Host-memory call: numpy in, numpy out."""
        i = np.ascontiguousarray(id_key, np.uint64)
        c = np.ascontiguousarray(cause_key, np.uint64)
        k = np.ascontiguousarray(kind, np.uint8)
        off = np.ascontiguousarray(offsets, np.uint64)
        D, N = len(off) - 1, len(i)
        if int(off[-1]) != N:
            raise ValueError("offsets[-1] != number of nodes")
        b, off = self._batch(off, _ptr(i), _ptr(c), _ptr(k), layout, key_bits)
        out = ListResult(np.zeros(N, np.uint32), np.zeros((N + 31) // 32, np.uint32),
                         np.zeros(D, np.uint32), np.zeros(D, np.uint64), np.zeros(D, np.uint32),
                         np.zeros(N, np.uint32) if (yarns and layout.site_bits) else None)
        r = CwListResult(_ptr(out.weave_perm), _ptr(out.visible_bits), _ptr(out.visible_count),
                         _ptr(out.max_ts), _ptr(out.status), _ptr(out.yarn_perm))
        self._check(self._L.cw_weave_lists(self._h, C.byref(b), C.byref(r), CW_MEM_HOST),
                    "cw_weave_lists")
        return out

    def weave_lists_device(self, offsets, id_ptr, cause_ptr, kind_ptr, layout, out_ptrs,
                           key_bits=None):
        """Device-memory call: raw device pointers (e.g. torch tensor data_ptr()).
        out_ptrs: dict with weave_perm, visible_bits, visible_count, max_ts,
        status, yarn_perm (None allowed where the header allows NULL)."""
        b, off = self._batch(offsets, C.c_void_p(id_ptr), C.c_void_p(cause_ptr),
                             C.c_void_p(kind_ptr), layout, key_bits)
        g = lambda n: C.c_void_p(out_ptrs[n]) if out_ptrs.get(n) else None
        r = CwListResult(g("weave_perm"), g("visible_bits"), g("visible_count"), g("max_ts"),
                         g("status"), g("yarn_perm"))
        self._check(self._L.cw_weave_lists(self._h, C.byref(b), C.byref(r), CW_MEM_DEVICE),
                    "cw_weave_lists")

    def weave_lists_k32(self, offsets, id_key, cause_key, kind, layout, yarns=True,
                        key_bits=None) -> ListResult:
        """Host-memory call of cw_weave_lists_k32: id_key / cause_key are uint32
        (nil = NIL32, see narrow_k32)."""
        i = np.ascontiguousarray(id_key, np.uint32)
        c = np.ascontiguousarray(cause_key, np.uint32)
        k = np.ascontiguousarray(kind, np.uint8)
        off = np.ascontiguousarray(offsets, np.uint64)
        D, N = len(off) - 1, len(i)
        if int(off[-1]) != N or len(c) != N or len(k) != N:
            raise ValueError("offsets[-1] / id_key / cause_key / kind sizes differ")
        b, off = self._batch_k32(off, _ptr(i), _ptr(c), _ptr(k), layout, key_bits)
        out = ListResult(np.zeros(N, np.uint32), np.zeros((N + 31) // 32, np.uint32),
                         np.zeros(D, np.uint32), np.zeros(D, np.uint64), np.zeros(D, np.uint32),
                         np.zeros(N, np.uint32) if (yarns and layout.site_bits) else None)
        r = CwListResult(_ptr(out.weave_perm), _ptr(out.visible_bits), _ptr(out.visible_count),
                         _ptr(out.max_ts), _ptr(out.status), _ptr(out.yarn_perm))
        self._check(self._L.cw_weave_lists_k32(self._h, C.byref(b), C.byref(r), CW_MEM_HOST),
                    "cw_weave_lists_k32")
        return out

    @staticmethod
    def _batch_k32(offsets, id_ptr, cause_ptr, kind_ptr, layout, key_bits=None, perm16=False):
        off = np.ascontiguousarray(offsets, np.uint64)
        b = CwListBatchK32()
        b.n_docs = len(off) - 1
        b.doc_offsets = off.ctypes.data_as(C.POINTER(C.c_uint64))
        b.id_key, b.cause_key, b.kind = id_ptr, cause_ptr, kind_ptr
        b.key_bits = layout.key_bits if key_bits is None else key_bits
        b.ts_shift, b.site_shift, b.site_bits = layout.ts_shift, layout.site_shift, layout.site_bits
        b.perm16 = int(perm16)
        return b, off

    def weave_lists_k32_device(self, offsets, id_ptr, cause_ptr, kind_ptr, layout, out_ptrs,
                               key_bits=None, perm16=False):
        """Device-memory call of cw_weave_lists_k32 (u32 keys; out_ptrs as
        weave_lists_device; perm16: weave_perm is uint16 per node)."""
        b, off = self._batch_k32(offsets, C.c_void_p(id_ptr), C.c_void_p(cause_ptr),
                                 C.c_void_p(kind_ptr), layout, key_bits, perm16)
        g = lambda n: C.c_void_p(out_ptrs[n]) if out_ptrs.get(n) else None
        r = CwListResult(g("weave_perm"), g("visible_bits"), g("visible_count"), g("max_ts"),
                         g("status"), g("yarn_perm"))
        self._check(self._L.cw_weave_lists_k32(self._h, C.byref(b), C.byref(r), CW_MEM_DEVICE),
                    "cw_weave_lists_k32")

    @staticmethod
    def _batch_k128(offsets, id_ptr, cause_ptr, kind_ptr):
        off = np.ascontiguousarray(offsets, np.uint64)
        b = CwListBatchK128()
        b.n_docs = len(off) - 1
        b.doc_offsets = off.ctypes.data_as(C.POINTER(C.c_uint64))
        b.id_key, b.cause_key, b.kind = id_ptr, cause_ptr, kind_ptr
        return b, off

    def weave_lists_k128(self, offsets, id_key, cause_key, kind, yarns=True) -> ListResult:
        """Host-memory call of cw_weave_lists_k128: id_key / cause_key are
        uint64[N, 2] (hi = ts, lo = site_rank << 32 | tx; nil = (NIL, NIL))."""
        i = np.ascontiguousarray(id_key, np.uint64).reshape(-1, 2)
        c = np.ascontiguousarray(cause_key, np.uint64).reshape(-1, 2)
        k = np.ascontiguousarray(kind, np.uint8)
        off = np.ascontiguousarray(offsets, np.uint64)
        D, N = len(off) - 1, len(k)
        if int(off[-1]) != N or len(i) != N or len(c) != N:
            raise ValueError("offsets[-1] / id_key / cause_key / kind sizes differ")
        b, off = self._batch_k128(off, _ptr(i), _ptr(c), _ptr(k))
        out = ListResult(np.zeros(N, np.uint32), np.zeros((N + 31) // 32, np.uint32),
                         np.zeros(D, np.uint32), np.zeros(D, np.uint64), np.zeros(D, np.uint32),
                         np.zeros(N, np.uint32) if yarns else None)
        r = CwListResult(_ptr(out.weave_perm), _ptr(out.visible_bits), _ptr(out.visible_count),
                         _ptr(out.max_ts), _ptr(out.status), _ptr(out.yarn_perm))
        self._check(self._L.cw_weave_lists_k128(self._h, C.byref(b), C.byref(r), CW_MEM_HOST),
                    "cw_weave_lists_k128")
        return out

    def weave_lists_k128_device(self, offsets, id_ptr, cause_ptr, kind_ptr, out_ptrs):
        """Device-memory call of cw_weave_lists_k128 (out_ptrs as weave_lists_device)."""
        b, off = self._batch_k128(offsets, C.c_void_p(id_ptr), C.c_void_p(cause_ptr),
                                  C.c_void_p(kind_ptr))
        g = lambda n: C.c_void_p(out_ptrs[n]) if out_ptrs.get(n) else None
        r = CwListResult(g("weave_perm"), g("visible_bits"), g("visible_count"), g("max_ts"),
                         g("status"), g("yarn_perm"))
        self._check(self._L.cw_weave_lists_k128(self._h, C.byref(b), C.byref(r), CW_MEM_DEVICE),
                    "cw_weave_lists_k128")

    # --- building blocks of the distributed giant list (device pointers) ---------
    def sort_keys_device(self, keys_ptr, n, key_bits, keys_out_ptr, idx_out_ptr):
        self._check(self._L.cw_sort_keys(self._h, keys_ptr, n, key_bits, keys_out_ptr, idx_out_ptr),
                    "cw_sort_keys")

    def sort_keys(self, keys, key_bits=0):
        """Host arrays: (sorted keys, input index of each) through cw_sort_keys
        (device buffers from torch; the call is synchronous)."""
        import torch

        k = np.ascontiguousarray(keys, np.uint64)
        n = len(k)
        if n == 0:
            return k.copy(), np.zeros(0, np.uint32)
        dev = torch.device("cuda", self.device)
        kin = torch.from_numpy(k.view(np.int64)).to(dev)
        kout = torch.empty_like(kin)
        iout = torch.empty(n, dtype=torch.int32, device=dev)
        torch.cuda.synchronize(dev)
        self.sort_keys_device(kin.data_ptr(), n, key_bits, kout.data_ptr(), iout.data_ptr())
        return kout.cpu().numpy().view(np.uint64), iout.cpu().numpy().view(np.uint32)

    def lookup_keys_device(self, sorted_ptr, n, q_ptr, m, base, out_ptr, status_ptr=None):
        self._check(self._L.cw_lookup_keys(self._h, sorted_ptr, n, q_ptr, m, base, out_ptr,
                                           status_ptr), "cw_lookup_keys")

    def partition_keys_device(self, keys_ptr, m, split_ptr, n_split, perm_ptr) -> np.ndarray:
        counts = np.zeros(n_split + 1, np.uint64)
        self._check(self._L.cw_partition_keys(self._h, keys_ptr, m, split_ptr, n_split, perm_ptr,
                                              counts.ctypes.data), "cw_partition_keys")
        return counts

    def partition_keys_dev(self, keys_ptr, m, split_ptr, n_split, perm_ptr, counts_ptr):
        """cw_partition_keys with the n_split + 1 counts (u64) left in device memory."""
        self._check(self._L.cw_partition_keys_dev(self._h, keys_ptr, m, split_ptr, n_split, perm_ptr,
                                                  counts_ptr), "cw_partition_keys_dev")

    def gather_device(self, src_ptr, idx_ptr, m, elem_size, dst_ptr):
        self._check(self._L.cw_gather(self._h, src_ptr, idx_ptr, m, elem_size, dst_ptr), "cw_gather")

    def scatter32_device(self, src_ptr, idx_ptr, m, dst_ptr):
        self._check(self._L.cw_scatter32(self._h, src_ptr, idx_ptr, m, dst_ptr), "cw_scatter32")

    def weave_ranked_device(self, n, par_ptr, kind_ptr, val_ptr, out_ptrs):
        """out_ptrs: weave_perm, visible_bits (or None), visible_count, status."""
        lst = CwRankedList(n, par_ptr, kind_ptr, val_ptr)
        g = lambda k: C.c_void_p(out_ptrs[k]) if out_ptrs.get(k) else None
        r = CwListResult(g("weave_perm"), g("visible_bits"), g("visible_count"), None, g("status"),
                         None)
        self._check(self._L.cw_weave_ranked(self._h, C.byref(lst), C.byref(r)), "cw_weave_ranked")

    def sort_keys32_device(self, keys_ptr, n, key_bits, keys_out_ptr, idx_out_ptr):
        self._check(self._L.cw_sort_keys32(self._h, keys_ptr, n, key_bits, keys_out_ptr,
                                           idx_out_ptr), "cw_sort_keys32")

    def dist(self, name, *args):
        """cw_dist_<name>(ctx, *args): a building block of the distributed tree
        (device pointers as ints, sizes, bases)."""
        self._check(getattr(self._L, "cw_dist_" + name)(self._h, *args), "cw_dist_" + name)

    def weave_linked_device(self, n, succ_ptr, thr_ptr, val_ptr, out_ptrs):
        """cw_weave_linked: out_ptrs as weave_ranked_device."""
        lst = CwLinkedList(n, succ_ptr, thr_ptr, val_ptr)
        g = lambda k: C.c_void_p(out_ptrs[k]) if out_ptrs.get(k) else None
        r = CwListResult(g("weave_perm"), g("visible_bits"), g("visible_count"), None, g("status"),
                         None)
        self._check(self._L.cw_weave_linked(self._h, C.byref(lst), C.byref(r)), "cw_weave_linked")

    def merge_lists(self, a, b, layout, yarns=True) -> MergeResult:
        """Host-memory call of cw_merge_lists.  a, b: (offsets, id_key, cause_key,
        kind, value_token) per side, with the same number of documents."""
        def side(t):
            off, i, c, k, v = t
            off = np.ascontiguousarray(off, np.uint64)
            arrs = (np.ascontiguousarray(i, np.uint64), np.ascontiguousarray(c, np.uint64),
                    np.ascontiguousarray(k, np.uint8), np.ascontiguousarray(v, np.uint64))
            if int(off[-1]) != len(arrs[0]):
                raise ValueError("offsets[-1] != number of nodes")
            return off, arrs
        ao, (ai, ac, ak, av) = side(a)
        bo, (bi, bc, bk, bv) = side(b)
        if len(ao) != len(bo):
            raise ValueError("a and b must have the same number of documents")
        D, NC = len(ao) - 1, len(ai) + len(bi)
        ba, _ = self._batch(ao, _ptr(ai), _ptr(ac), _ptr(ak), layout)
        bb, _ = self._batch(bo, _ptr(bi), _ptr(bc), _ptr(bk), layout)
        mb = CwMergeBatch(ba, _ptr(av), bb, _ptr(bv))
        mo = np.zeros(D + 1, np.uint64)
        src = np.zeros(max(NC, 1), np.uint32)
        w = ListResult(np.zeros(max(NC, 1), np.uint32), np.zeros((NC + 31) // 32 + 1, np.uint32),
                       np.zeros(max(D, 1), np.uint32), np.zeros(max(D, 1), np.uint64),
                       np.zeros(max(D, 1), np.uint32),
                       np.zeros(max(NC, 1), np.uint32) if (yarns and layout.site_bits) else None)
        r = CwMergeResult(mo.ctypes.data_as(C.POINTER(C.c_uint64)), _ptr(src),
                          CwListResult(_ptr(w.weave_perm), _ptr(w.visible_bits),
                                       _ptr(w.visible_count), _ptr(w.max_ts), _ptr(w.status),
                                       _ptr(w.yarn_perm)))
        self._check(self._L.cw_merge_lists(self._h, C.byref(mb), C.byref(r), CW_MEM_HOST),
                    "cw_merge_lists")
        M = int(mo[-1])
        w = ListResult(w.weave_perm[:M], w.visible_bits[:(M + 31) // 32], w.visible_count[:D],
                       w.max_ts[:D], w.status[:D], None if w.yarn_perm is None else w.yarn_perm[:M])
        return MergeResult(mo, src[:M], w)

    def weft_lists(self, offsets, id_key, cause_key, kind, layout, cut, yarns=True) -> MergeResult:
        """Host-memory call of cw_weft_lists.  cut: uint64[D << site_bits] packed
        cut id per (document, site rank), 0 = site not named.  Returns the kept
        nodes (src = doc-local input index, input order) and their weave."""
        i = np.ascontiguousarray(id_key, np.uint64)
        c = np.ascontiguousarray(cause_key, np.uint64)
        k = np.ascontiguousarray(kind, np.uint8)
        off = np.ascontiguousarray(offsets, np.uint64)
        cut = np.ascontiguousarray(cut, np.uint64)
        D, N = len(off) - 1, len(i)
        if int(off[-1]) != N or len(cut) != D << layout.site_bits:
            raise ValueError("offsets / cut sizes")
        b, off = self._batch(off, _ptr(i), _ptr(c), _ptr(k), layout)
        wb = CwWeftBatch(b, cut.ctypes.data_as(C.POINTER(C.c_uint64)))
        ko = np.zeros(D + 1, np.uint64)
        cap = max(N + (D << layout.site_bits), 1)  # + one [id] node per named site
        src = np.zeros(cap, np.uint32)
        w = ListResult(np.zeros(cap, np.uint32), np.zeros((cap + 31) // 32 + 1, np.uint32),
                       np.zeros(max(D, 1), np.uint32), np.zeros(max(D, 1), np.uint64),
                       np.zeros(max(D, 1), np.uint32),
                       np.zeros(cap, np.uint32) if (yarns and layout.site_bits) else None)
        r = CwWeftResult(ko.ctypes.data_as(C.POINTER(C.c_uint64)), _ptr(src),
                         CwListResult(_ptr(w.weave_perm), _ptr(w.visible_bits),
                                      _ptr(w.visible_count), _ptr(w.max_ts), _ptr(w.status),
                                      _ptr(w.yarn_perm)))
        self._check(self._L.cw_weft_lists(self._h, C.byref(wb), C.byref(r), CW_MEM_HOST),
                    "cw_weft_lists")
        M = int(ko[-1])
        w = ListResult(w.weave_perm[:M], w.visible_bits[:(M + 31) // 32], w.visible_count[:D],
                       w.max_ts[:D], w.status[:D], None if w.yarn_perm is None else w.yarn_perm[:M])
        return MergeResult(ko, src[:M], w)

    def weave_maps_device(self, offsets, ptrs, token_bits, key_bits, out_ptrs, cap_segs) -> int:
        """Device-memory call of cw_weave_maps: ptrs = (id_key, cause, cause_is_id,
        kind) device pointers; out_ptrs: seg_offsets, seg_coll, seg_key,
        seg_active, seg_perm, status device pointers.  Returns n_segs."""
        off = np.ascontiguousarray(offsets, np.uint64)
        b = CwMapBatch()
        b.n_colls = len(off) - 1
        b.coll_offsets = off.ctypes.data_as(C.POINTER(C.c_uint64))
        b.id_key, b.cause, b.cause_is_id, b.kind = (C.c_void_p(p) for p in ptrs)
        b.key_bits = key_bits
        b.token_bits = token_bits
        g = lambda n: C.c_void_p(out_ptrs[n])
        r = CwMapResult(cap_segs, 0, g("seg_offsets"), g("seg_coll"), g("seg_key"),
                        g("seg_active"), g("seg_perm"), g("status"))
        self._check(self._L.cw_weave_maps(self._h, C.byref(b), C.byref(r), CW_MEM_DEVICE),
                    "cw_weave_maps")
        return int(r.n_segs)

    def weave_maps(self, offsets, id_key, cause, cause_is_id, kind, token_bits,
                   key_bits=0) -> MapResult:
        """Host-memory call of cw_weave_maps."""
        i = np.ascontiguousarray(id_key, np.uint64)
        c = np.ascontiguousarray(cause, np.uint64)
        ci = np.ascontiguousarray(cause_is_id, np.uint8)
        k = np.ascontiguousarray(kind, np.uint8)
        off = np.ascontiguousarray(offsets, np.uint64)
        D, N = len(off) - 1, len(i)
        if int(off[-1]) != N:
            raise ValueError("offsets[-1] != number of nodes")
        b = CwMapBatch()
        b.n_colls = D
        b.coll_offsets = off.ctypes.data_as(C.POINTER(C.c_uint64))
        b.id_key, b.cause, b.cause_is_id, b.kind = _ptr(i), _ptr(c), _ptr(ci), _ptr(k)
        b.key_bits = key_bits
        b.token_bits = token_bits
        cap = max(N, 1)
        out = MapResult(np.zeros(cap + 1, np.uint64), np.zeros(cap, np.uint32),
                        np.zeros(cap, np.uint64), np.zeros(cap, np.int64),
                        np.zeros(N + cap, np.uint32), np.zeros(max(D, 1), np.uint32))
        r = CwMapResult(cap, 0, _ptr(out.seg_offsets), _ptr(out.seg_coll), _ptr(out.seg_key),
                        _ptr(out.seg_active), _ptr(out.seg_perm), _ptr(out.status))
        self._check(self._L.cw_weave_maps(self._h, C.byref(b), C.byref(r), CW_MEM_HOST),
                    "cw_weave_maps")
        S = int(r.n_segs)
        return MapResult(out.seg_offsets[:S + 1], out.seg_coll[:S], out.seg_key[:S],
                         out.seg_active[:S], out.seg_perm[:N + S], out.status[:D])
