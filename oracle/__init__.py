"""CPU oracle for Cause's weave -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this package, and only as the checker.  The product path (cause_amd/) must never
import it.

* ``oracle.causal_ref`` -- pure-Python restatement on real Clojure-shaped values
  (small cases).
* this module -- numpy/ctypes front end of ``liboracle.so`` (weave_oracle.c), the
  C restatement on packed 64-bit ids (any size).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

METHOD_LITERAL, METHOD_LINKED, METHOD_EFF, METHOD_GENERAL = 0, 1, 2, 3
NIL = (1 << 64) - 1  # OR_NIL (weave_oracle.h)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make oracle`")
        L = C.CDLL(path)
        u64p, u32p, u8p = (C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.POINTER(C.c_uint8))
        for name in ("or_list_fold_literal", "or_list_fold_linked", "or_list_eff_preorder",
                     "or_list_fold_general"):
            f = getattr(L, name)
            f.restype = C.c_uint32
            f.argtypes = [C.c_size_t, u64p, u64p, u8p, u32p]
        L.or_list_insert_sequence.restype = C.c_uint32
        L.or_list_insert_sequence.argtypes = [C.c_size_t, u64p, u64p, u8p, u32p, u32p]
        L.or_list_visible_literal.restype = None
        L.or_list_visible_literal.argtypes = [C.c_size_t, u64p, u64p, u8p, u32p, u8p]
        L.or_list_yarns.restype = None
        L.or_list_yarns.argtypes = [C.c_size_t, u64p, C.c_uint, C.c_uint64, u32p]
        L.or_batch_lists.restype = C.c_int
        L.or_batch_lists.argtypes = [C.c_size_t, u64p, u64p, u64p, u8p, C.c_int, C.c_int,
                                     u32p, u8p, u32p]
        L.or_map_fold_literal.restype = C.c_size_t
        L.or_map_fold_literal.argtypes = [C.c_size_t, u64p, u64p, u8p, u8p, C.c_uint64,
                                          u64p, u32p, u64p, C.POINTER(C.c_int64)]
        _LIB = L
    return _LIB


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def _arrs(id_key, cause_key, kind):
    return (np.ascontiguousarray(id_key, np.uint64), np.ascontiguousarray(cause_key, np.uint64),
            np.ascontiguousarray(kind, np.uint8))


def list_weave(id_key, cause_key, kind, method=METHOD_LITERAL):
    """One document -> (perm uint32[n], status)."""
    i, c, k = _arrs(id_key, cause_key, kind)
    n = len(i)
    out = np.zeros(n, np.uint32)
    f = {METHOD_LITERAL: lib().or_list_fold_literal, METHOD_LINKED: lib().or_list_fold_linked,
         METHOD_EFF: lib().or_list_eff_preorder, METHOD_GENERAL: lib().or_list_fold_general}[method]
    st = f(n, _p(i, C.c_uint64), _p(c, C.c_uint64), _p(k, C.c_uint8), _p(out, C.c_uint32))
    return out, int(st)


def list_insert_sequence(id_key, cause_key, kind, order):
    i, c, k = _arrs(id_key, cause_key, kind)
    o = np.ascontiguousarray(order, np.uint32)
    out = np.zeros(len(i), np.uint32)
    st = lib().or_list_insert_sequence(len(i), _p(i, C.c_uint64), _p(c, C.c_uint64),
                                       _p(k, C.c_uint8), _p(o, C.c_uint32), _p(out, C.c_uint32))
    return out, int(st)


def list_visible(id_key, cause_key, kind, perm):
    i, c, k = _arrs(id_key, cause_key, kind)
    p = np.ascontiguousarray(perm, np.uint32)
    vis = np.zeros(len(i), np.uint8)
    lib().or_list_visible_literal(len(i), _p(i, C.c_uint64), _p(c, C.c_uint64),
                                  _p(k, C.c_uint8), _p(p, C.c_uint32), _p(vis, C.c_uint8))
    return vis


def list_yarns(id_key, site_shift, site_mask):
    i = np.ascontiguousarray(id_key, np.uint64)
    out = np.zeros(len(i), np.uint32)
    lib().or_list_yarns(len(i), _p(i, C.c_uint64), site_shift, site_mask, _p(out, C.c_uint32))
    return out


def batch_lists(offsets, id_key, cause_key, kind, method=METHOD_LINKED, nthreads=None,
                with_vis=True):
    """Whole batch -> (perm uint32[N] doc-local, vis uint8[N] per weave position,
    status uint32[D])."""
    off = np.ascontiguousarray(offsets, np.uint64)
    i, c, k = _arrs(id_key, cause_key, kind)
    D, N = len(off) - 1, len(i)
    perm = np.zeros(N, np.uint32)
    vis = np.zeros(N, np.uint8) if with_vis else None
    st = np.zeros(D, np.uint32)
    nthreads = nthreads or os.cpu_count() or 1
    lib().or_batch_lists(D, _p(off, C.c_uint64), _p(i, C.c_uint64), _p(c, C.c_uint64),
                         _p(k, C.c_uint8), method, nthreads, _p(perm, C.c_uint32),
                         _p(vis, C.c_uint8) if vis is not None else None, _p(st, C.c_uint32))
    return perm, vis, st


MAP_TOKEN_BIT = 1 << 63


def map_causes(cause, cause_is_id):
    """The ABI's map causes (packed id, key token, nil: cause_is_id 1 / 0 / 2)
    in the form map_weave keys them by: ids as they are, tokens with bit 63 set
    (a keyword is never a vector), nil as OR_NIL."""
    c = np.asarray(cause, np.uint64)
    ci = np.asarray(cause_is_id)
    return np.where(ci == 1, c, np.where(ci == 2, np.uint64(NIL), c | np.uint64(MAP_TOKEN_BIT)))


def map_weave(id_key, cause, cause_is_id, kind, root_id):
    """One map collection -> (node_key u64[n], node_pos u32[n], seg_key u64[S],
    seg_active i64[S])."""
    i = np.ascontiguousarray(id_key, np.uint64)
    c = np.ascontiguousarray(cause, np.uint64)
    ci = np.ascontiguousarray(cause_is_id, np.uint8)
    k = np.ascontiguousarray(kind, np.uint8)
    n = len(i)
    nk = np.zeros(n, np.uint64)
    npos = np.zeros(n, np.uint32)
    sk = np.zeros(max(n, 1), np.uint64)
    sa = np.zeros(max(n, 1), np.int64)
    S = lib().or_map_fold_literal(n, _p(i, C.c_uint64), _p(c, C.c_uint64), _p(ci, C.c_uint8),
                                  _p(k, C.c_uint8), root_id, _p(nk, C.c_uint64),
                                  _p(npos, C.c_uint32), _p(sk, C.c_uint64),
                                  _p(sa, C.c_int64))
    return nk, npos, sk[:S], sa[:S]
