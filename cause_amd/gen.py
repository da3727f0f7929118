"""Synthetic workloads via libcauseweave_gen.so (input only).

``config1()`` -- one CausalList of 100,000 single-char inserts from 4 sites,
no hides (BASELINE.json configs[0]).
``config2(n_docs)`` -- independent CausalLists of 50,000 non-root nodes from
8 sites: 10% hides, 2% h.shows, 5% conj-style causes (BASELINE.json configs[1]).
``CONFIG4`` -- CausalMap collections of 100 nodes, keys Zipf(1.1) over 256
tokens, 8% key-level hides, 6% id-caused h.hide, 6% id-caused h.show
(BASELINE.json configs[3]).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from .pack import KeyLayout

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class CwgParams(C.Structure):
    _fields_ = [("nodes_per_doc", C.c_uint32), ("n_sites", C.c_uint32),
                ("p_hide", C.c_double), ("p_show", C.c_double), ("p_conj", C.c_double),
                ("p_chain", C.c_double), ("sync_every", C.c_uint32), ("seed", C.c_uint64),
                ("shuffle", C.c_int)]


class CwgMapParams(C.Structure):
    _fields_ = [("nodes_per_coll", C.c_uint32), ("n_sites", C.c_uint32), ("n_keys", C.c_uint32),
                ("zipf_s", C.c_double), ("p_hide", C.c_double), ("p_hhide", C.c_double),
                ("p_hshow", C.c_double), ("p_bad", C.c_double), ("sync_every", C.c_uint32),
                ("seed", C.c_uint64), ("shuffle", C.c_int)]


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libcauseweave_gen.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make`")
        L = C.CDLL(path)
        L.cwg_layout.argtypes = [C.POINTER(CwgParams), C.POINTER(C.c_uint32),
                                 C.POINTER(C.c_uint32)]
        L.cwg_layout.restype = None
        L.cwg_generate.argtypes = [C.POINTER(CwgParams), C.c_uint64, C.c_uint64, C.c_void_p,
                                   C.c_void_p, C.c_void_p, C.c_int]
        L.cwg_generate.restype = C.c_int
        L.cwg_generate32.argtypes = L.cwg_generate.argtypes
        L.cwg_generate32.restype = C.c_int
        L.cwg_map_layout.argtypes = [C.POINTER(CwgMapParams)] + [C.POINTER(C.c_uint32)] * 3
        L.cwg_map_layout.restype = None
        L.cwg_map_generate.argtypes = [C.POINTER(CwgMapParams), C.c_uint64, C.c_uint64] + \
            [C.c_void_p] * 4 + [C.c_int]
        L.cwg_map_generate.restype = C.c_int
        _LIB = L
    return _LIB


@dataclass(frozen=True)
class GenSpec:
    nodes_per_doc: int
    n_sites: int
    p_hide: float = 0.0
    p_show: float = 0.0
    p_conj: float = 0.0
    p_chain: float = 0.7
    sync_every: int = 16
    seed: int = 0xC0FFEE
    shuffle: bool = True

    def params(self) -> CwgParams:
        return CwgParams(self.nodes_per_doc, self.n_sites, self.p_hide, self.p_show, self.p_conj,
                         self.p_chain, self.sync_every, self.seed, int(self.shuffle))

    def layout(self) -> KeyLayout:
        tb, sb = C.c_uint32(), C.c_uint32()
        lib().cwg_layout(C.byref(self.params()), C.byref(tb), C.byref(sb))
        return KeyLayout(tb.value, sb.value, 0)

    @property
    def doc_size(self) -> int:
        return self.nodes_per_doc + 1


CONFIG1 = GenSpec(nodes_per_doc=100_000, n_sites=4, seed=0xC0FFEE ^ 1)
CONFIG2 = GenSpec(nodes_per_doc=50_000, n_sites=8, p_hide=0.10, p_show=0.02, p_conj=0.05,
                  seed=0xC0FFEE ^ 2)


def generate(spec: GenSpec, doc_begin: int, doc_end: int, nthreads: int | None = None, out=None,
             k32: bool = False):
    """-> (offsets u64[D+1], id_key u64[N], cause_key u64[N], kind u8[N]) for
    documents [doc_begin, doc_end) of ``spec``.  ``out`` may pass preallocated
    (id, cause, kind) arrays (e.g. pinned host memory).  k32: the same documents
    with u32 keys for cw_weave_lists_k32 (nil = 0xFFFFFFFF)."""
    D = doc_end - doc_begin
    n = spec.doc_size
    N = D * n
    kt = np.uint32 if k32 else np.uint64
    if out is None:
        idk, ck, kd = np.empty(N, kt), np.empty(N, kt), np.empty(N, np.uint8)
    else:
        idk, ck, kd = out
        if idk.dtype != kt or ck.dtype != kt:
            raise ValueError(f"out arrays must be {np.dtype(kt).name}")
    fn = lib().cwg_generate32 if k32 else lib().cwg_generate
    rc = fn(C.byref(spec.params()), doc_begin, doc_end,
                            idk.ctypes.data_as(C.c_void_p), ck.ctypes.data_as(C.c_void_p),
                            kd.ctypes.data_as(C.c_void_p), nthreads or min(os.cpu_count() or 1, 32))
    if rc != 0:
        raise RuntimeError("cwg_generate failed")
    off = np.arange(D + 1, dtype=np.uint64) * np.uint64(n)
    return off, idk, ck, kd


@dataclass(frozen=True)
class MapSpec:
    nodes_per_coll: int
    n_sites: int = 8
    n_keys: int = 256
    zipf_s: float = 1.1
    p_hide: float = 0.08
    p_hhide: float = 0.06
    p_hshow: float = 0.06
    p_bad: float = 0.0
    sync_every: int = 16
    seed: int = 0xC0FFEE ^ 4
    shuffle: bool = True

    def params(self) -> CwgMapParams:
        return CwgMapParams(self.nodes_per_coll, self.n_sites, self.n_keys, self.zipf_s,
                            self.p_hide, self.p_hhide, self.p_hshow, self.p_bad,
                            self.sync_every, self.seed, int(self.shuffle))

    def layout(self):
        """-> (KeyLayout of the ids, token_bits)."""
        tb, sb, kb = C.c_uint32(), C.c_uint32(), C.c_uint32()
        lib().cwg_map_layout(C.byref(self.params()), C.byref(tb), C.byref(sb), C.byref(kb))
        return KeyLayout(tb.value, sb.value, 0), kb.value


CONFIG4 = MapSpec(nodes_per_coll=100)


def generate_maps(spec: MapSpec, coll_begin: int, coll_end: int, nthreads: int | None = None):
    """-> (offsets u64[D+1], id_key u64[N], cause u64[N], cause_is_id u8[N], kind u8[N])."""
    D = coll_end - coll_begin
    n = spec.nodes_per_coll
    N = D * n
    idk, ck = np.empty(N, np.uint64), np.empty(N, np.uint64)
    ci, kd = np.empty(N, np.uint8), np.empty(N, np.uint8)
    rc = lib().cwg_map_generate(C.byref(spec.params()), coll_begin, coll_end,
                                idk.ctypes.data_as(C.c_void_p), ck.ctypes.data_as(C.c_void_p),
                                ci.ctypes.data_as(C.c_void_p), kd.ctypes.data_as(C.c_void_p),
                                nthreads or min(os.cpu_count() or 1, 32))
    if rc != 0:
        raise RuntimeError("cwg_map_generate failed")
    off = np.arange(D + 1, dtype=np.uint64) * np.uint64(n)
    return off, idk, ck, ci, kd
