"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU oracle (oracle/libfgo.so).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg. See fgo.h for
what the oracle restates and how it is pinned (behaviour pins of the reference's own tests; no
numeric golden vectors exist in the reference).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libfgo.so")
NONE = 0xFFFFFFFF


def build():
    subprocess.run(["make", "-C", HERE, "-s"], check=True)


class Stats(C.Structure):
    _fields_ = [("v_inv", C.c_uint64), ("e_trav", C.c_uint64), ("e_match", C.c_uint64),
                ("n_flagged", C.c_uint64), ("wall_ns", C.c_uint64), ("threads", C.c_uint32),
                ("pad", C.c_uint32)]


_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)
_u8p = C.POINTER(C.c_uint8)
_O = C.c_void_p
_SIG = {
    "fgo_create": ([C.c_uint32], _O),
    "fgo_destroy": ([_O], None),
    "fgo_load_graph": ([_O, C.c_uint32, _u64p, _u32p, C.c_uint64, _u32p, _u32p, _u64p], C.c_int),
    "fgo_current": ([_O, C.c_uint32], C.c_uint32),
    "fgo_last": ([_O, C.c_uint32], C.c_uint32),
    "fgo_node_count": ([_O], C.c_uint32),
    "fgo_node_info": ([_O, C.c_uint32, _u32p, _u64p, _u32p], C.c_int),
    "fgo_dump_states": ([_O, _u64p, _u32p], None),
    "fgo_begin_compute": ([_O, C.c_uint32, C.c_uint64, C.c_int, _u32p, _u32p, C.POINTER(Stats)], C.c_int),
    "fgo_set_output": ([_O, C.c_uint32, C.POINTER(Stats)], C.c_int),
    "fgo_add_used": ([_O, C.c_uint32, C.c_uint32, C.POINTER(Stats)], C.c_uint32),
    "fgo_begin_compute_n": ([_O, C.c_uint32, _u32p, _u64p, _u8p, C.POINTER(Stats)], C.c_int),
    "fgo_set_output_n": ([_O, C.c_uint32, _u32p, C.POINTER(Stats)], C.c_uint32),
    "fgo_add_used_n": ([_O, C.c_uint32, _u32p, _u32p, _u32p, C.POINTER(Stats)], None),
    "fgo_invalidate_slots":([_O, C.c_uint32, _u32p, _u8p, C.c_uint32, C.POINTER(Stats)], C.c_int),
    "fgo_invalidate_nodes": ([_O, C.c_uint32, _u32p, _u8p, C.POINTER(Stats)], C.c_int),
    "fgo_invalidate_everything": ([_O, C.POINTER(Stats)], C.c_int),
    "fgo_prune": ([_O, _u64p, _u64p], C.c_int),
    "fgo_prune_range": ([_O, C.c_uint32, C.c_uint32, _u64p, _u64p], C.c_int),
    "fgo_inv_log": ([_O, _u32p, C.c_uint64], C.c_uint64),
    "fgo_clear_log": ([_O], None),
    "fgo_used_by": ([_O, C.c_uint32, _u32p, _u64p, C.c_uint64], C.c_uint64),
    "fgo_export_used_by": ([C.c_void_p, _u32p, _u32p, _u64p, C.c_uint64], C.c_uint64),
    "fgo_used_count": ([_O, C.c_uint32], C.c_uint32),
    "fgo_total_used_by": ([_O], C.c_uint64),
    "fgo_snapshot": ([_O], C.c_int),
    "fgo_restore": ([_O], C.c_int),
    "fgo_splitmix64": ([C.c_uint64], C.c_uint64),
    "fgo_version_of": ([C.c_uint64, C.c_uint32], C.c_uint64),
    "fgo_gen_layered": ([C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64, _u32p, _u32p], C.c_uint64),
    "fgo_gen_rmat": ([C.c_uint32, C.c_uint32, C.c_uint64, _u32p, _u32p], C.c_uint64),
    "fgo_gen_tags": ([C.c_uint64, _u32p, _u32p, C.c_uint64, C.c_uint32, C.c_uint64, _u64p], None),
    "fgo_gen_roots": ([C.c_uint32, C.c_uint32, C.c_uint64, _u32p, _u32p], C.c_uint32),
    "fgo_set_threads": ([C.c_uint32], None),
    "fgo_get_threads": ([], C.c_uint32),
}
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        l = C.CDLL(LIB)
        for k, (a, r) in _SIG.items():
            f = getattr(l, k)
            f.argtypes = a
            f.restype = r
        _lib = l
    return _lib


def _p(a, ct):
    return None if a is None else a.ctypes.data_as(C.POINTER(ct))


def u32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint32))


def u64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint64))


def set_threads(n: int):
    """Worker threads of the bulk operations (import, snapshot/restore, generators); results do not
    depend on it."""
    lib().fgo_set_threads(int(n))


# ---- workload generators (CPU definitions) ----
def version_of(seed: int, slot) -> np.ndarray:
    """Vectorised fgo_version_of: (splitmix64(seed ^ slot) & (2^55-1)) | 1."""
    x = (np.uint64(seed) ^ u64(slot)) + np.uint64(0x9E3779B97F4A7C15)
    with np.errstate(over="ignore"):
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    return (x & np.uint64((1 << 55) - 1)) | np.uint64(1)


def gen_layered(levels, width, fanout, seed):
    m = lib().fgo_gen_layered(levels, width, fanout, seed, None, None)
    s, d = np.zeros(m, np.uint32), np.zeros(m, np.uint32)
    m = lib().fgo_gen_layered(levels, width, fanout, seed, _p(s, C.c_uint32), _p(d, C.c_uint32))
    return s[:m], d[:m]


def gen_rmat(scale, edge_factor, seed):
    m = (edge_factor << scale)
    s, d = np.zeros(m, np.uint32), np.zeros(m, np.uint32)
    m = lib().fgo_gen_rmat(scale, edge_factor, seed, _p(s, C.c_uint32), _p(d, C.c_uint32))
    return s[:m].copy(), d[:m].copy()


def gen_tags(src, dst, ver_seed, stale_pct=0, stale_seed=0):
    src, dst = u32(src), u32(dst)
    t = np.zeros(len(src), np.uint64)
    lib().fgo_gen_tags(len(src), _p(src, C.c_uint32), _p(dst, C.c_uint32), ver_seed, stale_pct, stale_seed,
                       _p(t, C.c_uint64))
    return t


def gen_roots(n_roots, range_, seed, out_degree=None):
    r = np.zeros(n_roots, np.uint32)
    deg = None if out_degree is None else u32(out_degree)
    n = lib().fgo_gen_roots(n_roots, range_, seed, _p(deg, C.c_uint32), _p(r, C.c_uint32))
    return r[:n].copy()


class Oracle:
    """The reference object graph (Computed nodes + ComputedRegistry) restated on the CPU."""

    def __init__(self, n_slots: int):
        self.l = lib()
        self.n_slots = n_slots
        self.o = self.l.fgo_create(n_slots)

    def close(self):
        if self.o:
            self.l.fgo_destroy(self.o)
            self.o = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load_graph(self, versions, state_flags, src, dst, tags):
        v = u64(versions)
        f = None if state_flags is None else u32(state_flags)
        s, d, t = u32(src), u32(dst), u64(tags)
        rc = self.l.fgo_load_graph(self.o, len(v), _p(v, C.c_uint64), _p(f, C.c_uint32), len(s),
                                   _p(s, C.c_uint32), _p(d, C.c_uint32), _p(t, C.c_uint64))
        assert rc == 0, "fgo_load_graph failed"

    def current(self, slot):
        return self.l.fgo_current(self.o, slot)

    def last(self, slot):
        return self.l.fgo_last(self.o, slot)

    def node_info(self, h):
        s, v, f = C.c_uint32(), C.c_uint64(), C.c_uint32()
        assert self.l.fgo_node_info(self.o, h, C.byref(s), C.byref(v), C.byref(f)) == 0
        return s.value, v.value, f.value

    def dump_states(self):
        v = np.zeros(self.n_slots, np.uint64)
        f = np.zeros(self.n_slots, np.uint32)
        self.l.fgo_dump_states(self.o, _p(v, C.c_uint64), _p(f, C.c_uint32))
        return v, f

    def begin_compute(self, slot, version, has_delay=False, stats=None):
        n, d = C.c_uint32(), C.c_uint32()
        assert self.l.fgo_begin_compute(self.o, slot, version, int(has_delay), C.byref(n), C.byref(d),
                                        C.byref(stats) if stats is not None else None) == 0
        return n.value, d.value

    def set_output(self, h, stats=None):
        return self.l.fgo_set_output(self.o, h, C.byref(stats) if stats is not None else None)

    def add_used(self, dependant_h, used_h):
        return self.l.fgo_add_used(self.o, dependant_h, used_h, None)

    def begin_compute_slots(self, slots, versions, has_delay=None):
        s, v = u32(slots), u64(versions)
        d = None if has_delay is None else np.ascontiguousarray(np.asarray(has_delay, np.uint8))
        assert self.l.fgo_begin_compute_n(self.o, len(s), _p(s, C.c_uint32), _p(v, C.c_uint64), _p(d, C.c_uint8),
                                          None) == 0

    def set_output_slots(self, slots):
        s = u32(slots)
        return self.l.fgo_set_output_n(self.o, len(s), _p(s, C.c_uint32), None)

    def add_used_slots(self, dependant_slots, used_slots):
        d, u = u32(dependant_slots), u32(used_slots)
        out = np.zeros(len(d), np.uint32)
        self.l.fgo_add_used_n(self.o, len(d), _p(d, C.c_uint32), _p(u, C.c_uint32), _p(out, C.c_uint32), None)
        return out

    def invalidate_slots(self, slots, immediately=None, threads=1, stats=None):
        s = u32(slots)
        imm = None if immediately is None else np.ascontiguousarray(np.asarray(immediately, np.uint8))
        st = stats if stats is not None else Stats()
        self.l.fgo_invalidate_slots(self.o, len(s), _p(s, C.c_uint32), _p(imm, C.c_uint8), threads, C.byref(st))
        return st

    def invalidate_nodes(self, handles, immediately=None, stats=None):
        h = u32(handles)
        imm = None if immediately is None else np.ascontiguousarray(np.asarray(immediately, np.uint8))
        st = stats if stats is not None else Stats()
        self.l.fgo_invalidate_nodes(self.o, len(h), _p(h, C.c_uint32), _p(imm, C.c_uint8), C.byref(st))
        return st

    def invalidate_everything(self, stats=None):
        st = stats if stats is not None else Stats()
        self.l.fgo_invalidate_everything(self.o, C.byref(st))
        return st

    def prune(self):
        a, b = C.c_uint64(), C.c_uint64()
        self.l.fgo_prune(self.o, C.byref(a), C.byref(b))
        return a.value, b.value

    def prune_range(self, first, count):
        a, b = C.c_uint64(), C.c_uint64()
        self.l.fgo_prune_range(self.o, first, count, C.byref(a), C.byref(b))
        return a.value, b.value

    def inv_log(self):
        n = self.l.fgo_inv_log(self.o, None, 0)
        out = np.zeros(n, np.uint32)
        self.l.fgo_inv_log(self.o, _p(out, C.c_uint32), n)
        return out

    def clear_log(self):
        self.l.fgo_clear_log(self.o)

    def used_by(self, h):
        n = self.l.fgo_used_by(self.o, h, None, None, 0)
        d, t = np.zeros(n, np.uint32), np.zeros(n, np.uint64)
        self.l.fgo_used_by(self.o, h, _p(d, C.c_uint32), _p(t, C.c_uint64), n)
        return d, t

    def export_used_by(self):
        """(slot, dependant slot, tag) of every slot's most recent node's `_usedBy` entries."""
        n = self.l.fgo_export_used_by(self.o, None, None, None, 0)
        s, d, t = np.zeros(n, np.uint32), np.zeros(n, np.uint32), np.zeros(n, np.uint64)
        self.l.fgo_export_used_by(self.o, _p(s, C.c_uint32), _p(d, C.c_uint32), _p(t, C.c_uint64), n)
        return s, d, t

    def used_count(self, h):
        return self.l.fgo_used_count(self.o, h)

    def total_used_by(self):
        return self.l.fgo_total_used_by(self.o)

    def snapshot(self):
        assert self.l.fgo_snapshot(self.o) == 0

    def restore(self):
        assert self.l.fgo_restore(self.o) == 0
