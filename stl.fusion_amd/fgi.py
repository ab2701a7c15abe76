"""ctypes binding of the fgi C-ABI (include/fgi.h) — the MI355X cascading-invalidation engine.

This is plumbing for tests and the bench; the drop-in host layers are the C++ mirror in
``stl.fusion_amd/host/fusion.hpp`` and the C# ``[LibraryImport]`` stubs in INTEGRATION.md. The
library is the in-tree ``stl.fusion_amd/lib/libfgi.so``; there is no fallback: if it is missing,
or no GPU is present, every call raises.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# FGI_LIBRARY selects another in-tree build of the engine (e.g. an instrumented one); there is no
# fallback: a missing library raises FgiError.
LIB_PATH = os.environ.get("FGI_LIBRARY") or os.path.join(_HERE, "lib", "libfgi.so")

OK, EINVAL, ENOMEM, ECAPACITY, EDEVICE, ESTATE, ENOTSUP = range(7)
OPT_DEAD_FILTER, OPT_DIRECTION, OPT_PULL_ALPHA, OPT_LEVEL_TIMING, OPT_PULL_BETA, OPT_DEFRAG_PCT = 1, 2, 3, 4, 5, 6
OPT_PART_COLLECTIVES = 7
OPT_PULL_TPB = 8
OPT_FRONT_EXCHANGE = 9
OPT_HOT_HEADS = 10
OPT_FAULT_INJECT = 11
OPT_FUSED = 12
OPT_PART_PLAN = 13
OPT_PART_BUCKET = 14
OPT_FAULT_INJECT_TAIL = 16
OPT_PROBE_SUMMARY = 15
DIR_AUTO, DIR_PUSH, DIR_PULL = 0, 1, 2
NONE = 0xFFFFFFFF
COMPUTING, CONSISTENT, INVALIDATED = 0, 1, 2
F_IOSO, F_DELAY_STARTED, F_HAS_DELAY = 4, 8, 16
USED_ADDED, USED_DROPPED, USED_INVALIDATED, USED_ESTATE = range(4)

_STATUS = {0: "FGI_OK", 1: "FGI_EINVAL", 2: "FGI_ENOMEM", 3: "FGI_ECAPACITY", 4: "FGI_EDEVICE",
           5: "FGI_ESTATE", 6: "FGI_ENOTSUP"}


class FgiError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{_STATUS.get(status, status)}: {msg}")
        self.status = status


class Config(C.Structure):
    _fields_ = [("struct_size", C.c_uint32), ("device", C.c_int32), ("n_slots", C.c_uint32),
                ("n_detached", C.c_uint32), ("edge_capacity", C.c_uint64), ("rank", C.c_int32),
                ("world", C.c_int32), ("labels", C.c_int32), ("reserved", C.c_int32)]


class WaveStats(C.Structure):
    _fields_ = [("roots", C.c_uint64), ("levels", C.c_uint64), ("v_inv", C.c_uint64),
                ("e_trav", C.c_uint64), ("e_match", C.c_uint64), ("n_flagged", C.c_uint64),
                ("alg_bytes", C.c_uint64), ("kernel_ms", C.c_double), ("total_ms", C.c_double),
                ("remote_msgs", C.c_uint64), ("f_total", C.c_uint64), ("expand_launches", C.c_uint64),
                ("expand_ms", C.c_double), ("expand_bytes", C.c_uint64), ("pull_levels", C.c_uint64),
                ("pull_edges", C.c_uint64), ("pull_ms", C.c_double), ("pull_bytes", C.c_uint64),
                ("pull_launches", C.c_uint64), ("fused_launches", C.c_uint64), ("fused_ms", C.c_double),
                ("fused_push_bytes", C.c_uint64), ("host_syncs", C.c_uint64), ("pull_pushed", C.c_uint64)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class Step(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("n", C.c_uint32), ("handles", C.c_void_p), ("used", C.c_void_p),
                ("version", C.c_void_p), ("flags", C.c_void_p), ("out", C.c_void_p)]


class BatchStats(C.Structure):
    _fields_ = [("waves", C.c_uint64), ("levels", C.c_uint64), ("v_inv", C.c_uint64), ("e_trav", C.c_uint64),
                ("e_match", C.c_uint64), ("n_flagged", C.c_uint64), ("kernel_ms", C.c_double),
                ("wave_ms", C.c_double), ("total_ms", C.c_double), ("host_syncs", C.c_uint32), ("pad", C.c_uint32)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "pad"}


STEP_INVALIDATE, STEP_BEGIN_COMPUTE, STEP_ADD_USED, STEP_SET_OUTPUT = 1, 2, 3, 4


class PruneStats(C.Structure):
    _fields_ = [("old_edges", C.c_uint64), ("new_edges", C.c_uint64), ("pool_before", C.c_uint64),
                ("pool_after", C.c_uint64), ("kernel_ms", C.c_double), ("total_ms", C.c_double),
                ("live_edges", C.c_uint64), ("dropped_edges", C.c_uint64), ("first", C.c_uint32),
                ("count", C.c_uint32), ("stale_estimate", C.c_uint64)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)
_u8p = C.POINTER(C.c_uint8)
_G = C.c_void_p

# name -> argtypes (every function returns int fgi_status except fgi_last_error)
SIGNATURES = {
    "fgi_version": [_u32p, _u32p],
    "fgi_create": [C.POINTER(Config), C.POINTER(C.c_void_p)],
    "fgi_destroy": [_G],
    "fgi_register_nodes": [_G, C.c_uint32, _u32p, _u64p, _u32p],
    "fgi_load_edges": [_G, C.c_uint64, _u32p, _u32p, _u64p],
    "fgi_get_state": [_G, C.c_uint32, _u32p, _u64p, _u32p],
    "fgi_dump_states": [_G, _u64p, _u32p],
    "fgi_get_used_by": [_G, C.c_uint32, _u32p, _u64p, C.c_uint64, _u64p],
    "fgi_get_used_count": [_G, C.c_uint32, _u32p],
    "fgi_get_degrees": [_G, _u32p, _u64p],
    "fgi_begin_compute": [_G, C.c_uint32, _u32p, _u64p, _u8p, _u32p, C.POINTER(WaveStats)],
    "fgi_add_used": [_G, C.c_uint32, _u32p, _u32p, _u32p],
    "fgi_set_output": [_G, C.c_uint32, _u32p, _u8p, _u32p, C.c_uint64, _u64p, C.POINTER(WaveStats)],
    "fgi_invalidate": [_G, C.c_uint32, _u32p, _u8p, _u32p, C.c_uint64, _u64p, C.POINTER(WaveStats)],
    "fgi_invalidate_dev": [_G, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, _u64p, C.POINTER(WaveStats)],
    "fgi_invalidate_bits": [_G, C.c_uint32, _u32p, _u8p, C.c_void_p, C.c_uint64, _u64p, C.POINTER(WaveStats)],
    "fgi_alloc_pinned": [C.c_uint64, C.POINTER(C.c_void_p)],
    "fgi_free_pinned": [C.c_void_p],
    "fgi_wave_ids_dev": [_G, C.POINTER(C.c_void_p), _u64p],
    "fgi_last_wave_ids": [_G, _u32p, C.c_uint64, _u64p],
    "fgi_invalidate_all": [_G, _u32p, C.c_uint64, _u64p, C.POINTER(WaveStats)],
    "fgi_prune": [_G, C.POINTER(PruneStats)],
    "fgi_prune_range": [_G, C.c_uint32, C.c_uint32, C.POINTER(PruneStats)],
    "fgi_prune_step": [_G, C.c_uint32, C.c_uint32, C.POINTER(PruneStats)],
    "fgi_release": [_G, C.c_uint32, _u32p],
    "fgi_snapshot": [_G],
    "fgi_restore": [_G],
    "fgi_synth_layered": [_G, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64],
    "fgi_synth_rmat": [_G, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint64],
    "fgi_export_edges": [_G, _u32p, _u32p, _u64p, C.c_uint64, _u64p],
    "fgi_stream": [_G, C.POINTER(C.c_void_p)],
    "fgi_set_option": [_G, C.c_int, C.c_int64],
    "fgi_part_unique_id": [_u8p],
    "fgi_part_init": [_G, C.c_uint32, _u8p],
    "fgi_part_synth_rmat": [_G, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint64],
    "fgi_part_register_nodes": [_G, C.c_uint32, _u32p, _u64p, _u32p],
    "fgi_part_load_edges": [_G, C.c_uint64, _u32p, _u32p, _u64p],
    "fgi_part_invalidate": [_G, C.c_uint32, C.c_void_p, C.c_void_p, _u64p, C.POINTER(WaveStats)],
    "fgi_part_export_ids": [_G, _u32p, C.c_uint64, _u64p],
    "fgi_part_front_stats": [_G, _u64p, _u64p, _u64p],
    "fgi_part_init_local": [C.POINTER(C.c_void_p), C.c_uint32, C.c_uint32],
    "fgi_part_local_invalidate": [C.POINTER(C.c_void_p), C.c_uint32, C.c_uint32, _u32p, _u8p, C.POINTER(WaveStats)],
    "fgi_rccl_info": [C.POINTER(C.c_int), C.c_char_p, C.c_uint64],
    "fgi_run_batch": [_G, C.c_uint32, C.POINTER(Step), _u32p, C.c_uint64, _u64p, C.POINTER(BatchStats)],
    "fgi_part_begin_compute": [_G, C.c_uint32, _u32p, _u64p, _u8p, _u32p, _u32p, C.c_uint64, _u64p,
                               C.POINTER(WaveStats)],
    "fgi_part_add_used": [_G, C.c_uint32, _u32p, _u32p, _u32p],
    "fgi_part_set_output": [_G, C.c_uint32, _u32p, _u8p, _u32p, C.c_uint64, _u64p, C.POINTER(WaveStats)],
    "fgi_part_invalidate_all": [_G, _u32p, C.c_uint64, _u64p, C.POINTER(WaveStats)],
    "fgi_part_run_batch": [_G, C.c_uint32, C.POINTER(Step), _u32p, C.c_uint64, _u64p, C.POINTER(BatchStats)],
    "fgi_part_prune": [_G, C.POINTER(PruneStats)],
    "fgi_part_init_host": [_G, C.c_uint32, C.c_void_p, C.c_void_p],
    "fgi_invalidate_async": [_G, C.c_uint32, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64)],
    "fgi_wave_wait": [_G, C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_void_p), C.POINTER(WaveStats)],
    "fgi_invalidate_async_host": [_G, C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint8), C.POINTER(C.c_uint64)],
    "fgi_wave_wait_ids": [_G, C.c_uint64, C.POINTER(C.c_uint32), C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(WaveStats)],
    "fgi_part_local_run_batch": [C.POINTER(C.c_void_p), C.c_uint32, C.c_uint32, C.POINTER(Step), _u32p, C.c_uint64,
                                 _u64p, C.POINTER(BatchStats)],
    "fgi_part_local_prune": [C.POINTER(C.c_void_p), C.c_uint32, C.POINTER(PruneStats)],
}

_lib = None
# fgi_allgather_fn: int (*)(void* ctx, const void* send, uint64_t bytes, void* recv)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p)


def load_library(path: str = LIB_PATH) -> C.CDLL:
    """Load libfgi.so. Raises if it is missing: there is no CPU fallback for the engine."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise FgiError(EDEVICE, f"{path} not built (run __graft_entry__.build())")
    lib = C.CDLL(path)
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = C.c_int
    lib.fgi_last_error.argtypes = [_G]
    lib.fgi_last_error.restype = C.c_char_p
    _lib = lib
    return lib


def _ptr(a: Optional[np.ndarray], ct):
    if a is None:
        return None
    return a.ctypes.data_as(C.POINTER(ct))


def _u32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint32))


def _u64(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint64))


def _u8(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint8))


def build_steps(steps):
    """fgi_step array for fgi_run_batch / fgi_part_run_batch (see Graph.run_batch); returns (array,
    arrays to keep alive, per-step output arrays or None)."""
    arr = (Step * len(steps))()
    keep, outs = [], []
    for k, sp in enumerate(steps):
        kind = sp[0]
        h = _u32(sp[1])
        keep.append(h)
        st = arr[k]
        st.n = len(h)
        st.handles = h.ctypes.data
        out = None
        if kind == "invalidate":
            st.kind = STEP_INVALIDATE
            if len(sp) > 2 and sp[2] is not None:
                f = _u8(sp[2])
                keep.append(f)
                st.flags = f.ctypes.data
        elif kind == "begin_compute":
            st.kind = STEP_BEGIN_COMPUTE
            v = _u64(sp[2])
            keep.append(v)
            st.version = v.ctypes.data
            if len(sp) > 3 and sp[3] is not None:
                f = _u8(sp[3])
                keep.append(f)
                st.flags = f.ctypes.data
            out = np.empty(len(h), np.uint32)   # every element is written
        elif kind == "add_used":
            st.kind = STEP_ADD_USED
            u = _u32(sp[2])
            keep.append(u)
            st.used = u.ctypes.data
            out = np.empty(len(h), np.uint32)   # every element is written
        elif kind == "set_output":
            st.kind = STEP_SET_OUTPUT
            out = np.empty(len(h), np.uint8)
        else:
            raise ValueError(kind)
        if out is not None:
            st.out = out.ctypes.data
        outs.append(out)
    return arr, keep, outs


class Graph:
    """One engine instance (one ComputedRegistry worth of nodes) on one device."""

    def __init__(self, n_slots: int, n_detached: int = 0, edge_capacity: int = 0, device: int = 0,
                 rank: int = 0, world: int = 1, labels: int = 0):
        """labels: internal hub-first labels (fgi_config.labels): 0 auto, 1 always, -1 never."""
        self.lib = load_library()
        cfg = Config(C.sizeof(Config), device, n_slots, n_detached, edge_capacity, rank, world, labels, 0)
        h = C.c_void_p()
        st = self.lib.fgi_create(C.byref(cfg), C.byref(h))
        if st != OK:
            raise FgiError(st, f"fgi_create(n_slots={n_slots}) failed (is a GPU present?)")
        self.h = h
        self.n_slots = n_slots
        self.n_detached = n_detached
        self.n_handles = n_slots + n_detached

    def close(self):
        if getattr(self, "h", None):
            self.lib.fgi_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, st: int, what: str):
        if st != OK:
            msg = self.lib.fgi_last_error(self.h)
            raise FgiError(st, f"{what}: {msg.decode() if msg else ''}")

    # ---- registry / import ----
    def register_nodes(self, slots, versions, state_flags=None):
        s, v = _u32(slots), _u64(versions)
        f = None if state_flags is None else _u32(state_flags)
        self._check(self.lib.fgi_register_nodes(self.h, len(s), _ptr(s, C.c_uint32), _ptr(v, C.c_uint64),
                                                _ptr(f, C.c_uint32)), "register_nodes")

    def load_edges(self, used, dependant, tags):
        u, d, t = _u32(used), _u32(dependant), _u64(tags)
        self._check(self.lib.fgi_load_edges(self.h, len(u), _ptr(u, C.c_uint32), _ptr(d, C.c_uint32),
                                            _ptr(t, C.c_uint64)), "load_edges")

    def synth_layered(self, levels, width, fanout, seed):
        self._check(self.lib.fgi_synth_layered(self.h, levels, width, fanout, seed), "synth_layered")

    def synth_rmat(self, scale, edge_factor, seed, stale_pct=0, stale_seed=0):
        self._check(self.lib.fgi_synth_rmat(self.h, scale, edge_factor, seed, stale_pct, stale_seed), "synth_rmat")

    # ---- queries ----
    def get_state(self, handles) -> Tuple[np.ndarray, np.ndarray]:
        h = _u32(handles)
        v = np.zeros(len(h), np.uint64)
        f = np.zeros(len(h), np.uint32)
        self._check(self.lib.fgi_get_state(self.h, len(h), _ptr(h, C.c_uint32), _ptr(v, C.c_uint64),
                                           _ptr(f, C.c_uint32)), "get_state")
        return v, f

    def dump_states(self) -> Tuple[np.ndarray, np.ndarray]:
        v = np.zeros(self.n_handles, np.uint64)
        f = np.zeros(self.n_handles, np.uint32)
        self._check(self.lib.fgi_dump_states(self.h, _ptr(v, C.c_uint64), _ptr(f, C.c_uint32)), "dump_states")
        return v, f

    def used_by(self, handle) -> Tuple[np.ndarray, np.ndarray]:
        n = C.c_uint64()
        st = self.lib.fgi_get_used_by(self.h, handle, None, None, 0, C.byref(n))
        if st not in (OK, ECAPACITY):
            self._check(st, "used_by")
        d = np.zeros(n.value, np.uint32)
        t = np.zeros(n.value, np.uint64)
        self._check(self.lib.fgi_get_used_by(self.h, handle, _ptr(d, C.c_uint32), _ptr(t, C.c_uint64), n.value,
                                             C.byref(n)), "used_by")
        return d, t

    def used_count(self, handle) -> int:
        c = C.c_uint32()
        self._check(self.lib.fgi_get_used_count(self.h, handle, C.byref(c)), "used_count")
        return c.value

    def degrees(self) -> Tuple[np.ndarray, int]:
        d = np.zeros(self.n_handles, np.uint32)
        t = C.c_uint64()
        self._check(self.lib.fgi_get_degrees(self.h, _ptr(d, C.c_uint32), C.byref(t)), "degrees")
        return d, t.value

    def export_edges(self):
        n = C.c_uint64()
        st = self.lib.fgi_export_edges(self.h, None, None, None, 0, C.byref(n))
        if st not in (OK, ECAPACITY):
            self._check(st, "export_edges")
        u = np.zeros(n.value, np.uint32)
        d = np.zeros(n.value, np.uint32)
        t = np.zeros(n.value, np.uint64)
        self._check(self.lib.fgi_export_edges(self.h, _ptr(u, C.c_uint32), _ptr(d, C.c_uint32), _ptr(t, C.c_uint64),
                                              n.value, C.byref(n)), "export_edges")
        return u, d, t

    # ---- mutations ----
    def begin_compute(self, slots, versions, has_delay=None, stats: Optional[WaveStats] = None) -> np.ndarray:
        s, v = _u32(slots), _u64(versions)
        hd = None if has_delay is None else _u8(has_delay)
        out = np.zeros(len(s), np.uint32)
        self._check(self.lib.fgi_begin_compute(self.h, len(s), _ptr(s, C.c_uint32), _ptr(v, C.c_uint64),
                                               _ptr(hd, C.c_uint8), _ptr(out, C.c_uint32),
                                               C.byref(stats) if stats is not None else None), "begin_compute")
        return out

    def add_used(self, dependant, used) -> np.ndarray:
        d, u = _u32(dependant), _u32(used)
        out = np.zeros(len(d), np.uint32)
        self._check(self.lib.fgi_add_used(self.h, len(d), _ptr(d, C.c_uint32), _ptr(u, C.c_uint32),
                                          _ptr(out, C.c_uint32)), "add_used")
        return out

    def set_output(self, handles, stats: Optional[WaveStats] = None):
        h = _u32(handles)
        out_set = np.zeros(len(h), np.uint8)
        ids = np.zeros(self.n_handles, np.uint32)
        n = C.c_uint64()
        self._check(self.lib.fgi_set_output(self.h, len(h), _ptr(h, C.c_uint32), _ptr(out_set, C.c_uint8),
                                            _ptr(ids, C.c_uint32), len(ids), C.byref(n),
                                            C.byref(stats) if stats is not None else None), "set_output")
        return out_set, ids[:n.value].copy()

    def invalidate(self, roots, immediately=None, stats: Optional[WaveStats] = None) -> np.ndarray:
        r = _u32(roots)
        imm = None if immediately is None else _u8(immediately)
        ids = np.zeros(self.n_handles, np.uint32)
        n = C.c_uint64()
        self._check(self.lib.fgi_invalidate(self.h, len(r), _ptr(r, C.c_uint32), _ptr(imm, C.c_uint8),
                                            _ptr(ids, C.c_uint32), len(ids), C.byref(n),
                                            C.byref(stats) if stats is not None else None), "invalidate")
        return ids[:n.value].copy()

    def run_batch(self, steps, stats: Optional[BatchStats] = None, want_ids: bool = True):
        """fgi_run_batch. `steps`: a list of ("invalidate", handles[, immediately]),
        ("begin_compute", slots, versions[, has_delay]), ("add_used", dependants, used),
        ("set_output", handles). Returns (ids of every cascade of the batch, per-step outputs: detached
        handles / add_used results / set flags, None for invalidate)."""
        return self._batch(self.lib.fgi_run_batch, "run_batch", steps, stats, want_ids)

    def _batch(self, fn, what, steps, stats, want_ids):
        arr, keep, outs = build_steps(steps)
        n = C.c_uint64()
        if want_ids:
            cap = max(1, sum(1 for sp in steps if sp[0] != "add_used")) * self.n_handles
            buf = getattr(self, "_ids_buf", None)
            if buf is None or len(buf) < cap:
                buf = self._ids_buf = np.empty(cap, np.uint32)   # reused across batches
            self._check(fn(self.h, len(steps), arr, _ptr(buf, C.c_uint32), cap, C.byref(n),
                           C.byref(stats) if stats is not None else None), what)
            return buf[:n.value].copy(), outs
        self._check(fn(self.h, len(steps), arr, None, 0, C.byref(n), C.byref(stats) if stats is not None else None),
                    what)
        return n.value, outs

    def invalidate_into(self, roots, out_ptr: int, cap: int, stats: Optional[WaveStats] = None) -> int:
        """fgi_invalidate with a caller-owned host output buffer (e.g. pinned memory at out_ptr,
        `cap` entries): root H2D -> wave -> invalidated-slot D2H. Returns the count."""
        r = _u32(roots)
        n = C.c_uint64()
        self._check(self.lib.fgi_invalidate(self.h, len(r), _ptr(r, C.c_uint32), None,
                                            C.cast(C.c_void_p(out_ptr), _u32p), cap, C.byref(n),
                                            C.byref(stats) if stats is not None else None), "invalidate")
        return n.value

    def invalidate_bits(self, roots, immediately=None, stats: Optional[WaveStats] = None,
                        out_ptr: int = 0) -> Tuple[Optional[np.ndarray], int]:
        """fgi_invalidate_bits: the wave's invalidated set as a bitmap over handles (uint64 words,
        bit h of word h // 64). With out_ptr (a caller-owned, e.g. pinned, buffer of
        (n_handles + 63) // 64 words) the bitmap lands there and (None, V_inv) is returned."""
        r = _u32(roots)
        imm = None if immediately is None else _u8(immediately)
        words = (self.n_handles + 63) // 64
        bits = None if out_ptr else np.zeros(words, np.uint64)
        n = C.c_uint64()
        dst = C.c_void_p(out_ptr) if out_ptr else bits.ctypes.data_as(C.c_void_p)
        self._check(self.lib.fgi_invalidate_bits(self.h, len(r), _ptr(r, C.c_uint32), _ptr(imm, C.c_uint8), dst, words,
                                                 C.byref(n), C.byref(stats) if stats is not None else None),
                    "invalidate_bits")
        return bits, n.value

    def invalidate_dev(self, n_roots: int, roots_ptr: int, imm_ptr: int = 0,
                       stats: Optional[WaveStats] = None) -> int:
        n = C.c_uint64()
        self._check(self.lib.fgi_invalidate_dev(self.h, n_roots, C.c_void_p(roots_ptr),
                                                C.c_void_p(imm_ptr) if imm_ptr else None, None, C.byref(n),
                                                C.byref(stats) if stats is not None else None), "invalidate_dev")
        return n.value

    def invalidate_async(self, n_roots: int, roots_ptr: int, imm_ptr: int = 0) -> int:
        """fgi_invalidate_async: queue a wave from device-resident roots; returns its ticket."""
        t = C.c_uint64()
        self._check(self.lib.fgi_invalidate_async(self.h, n_roots, C.c_void_p(roots_ptr),
                                                  C.c_void_p(imm_ptr) if imm_ptr else None, C.byref(t)),
                    "invalidate_async")
        return t.value

    def wave_wait(self, ticket: int, stats: Optional[WaveStats] = None) -> Tuple[int, int]:
        """fgi_wave_wait: (V_inv, device pointer to the wave's ids) of the ticket's wave."""
        n = C.c_uint64()
        p = C.c_void_p()
        self._check(self.lib.fgi_wave_wait(self.h, ticket, C.byref(n), C.byref(p),
                                           C.byref(stats) if stats is not None else None), "wave_wait")
        return n.value, p.value or 0

    def invalidate_async_host(self, roots, immediately=None) -> int:
        """fgi_invalidate_async_host: queue a wave from roots in host memory; returns its ticket."""
        r = _u32(roots)
        imm = _u8(immediately) if immediately is not None else None
        t = C.c_uint64()
        self._check(self.lib.fgi_invalidate_async_host(self.h, len(r), _ptr(r, C.c_uint32), _ptr(imm, C.c_uint8),
                                                       C.byref(t)), "invalidate_async_host")
        return t.value

    def wave_wait_ids(self, ticket: int, stats: Optional[WaveStats] = None) -> np.ndarray:
        """fgi_wave_wait_ids: wait for the ticket's wave, its invalidated handles (ascending) on the host."""
        n = C.c_uint64()
        self._check(self.lib.fgi_wave_wait_ids(self.h, ticket, None, 0, C.byref(n),
                                               C.byref(stats) if stats is not None else None), "wave_wait_ids")
        ids = np.zeros(n.value, np.uint32)
        self._check(self.lib.fgi_wave_wait_ids(self.h, ticket, _ptr(ids, C.c_uint32), len(ids), C.byref(n), None),
                    "wave_wait_ids")
        return ids

    def last_wave_ids(self) -> np.ndarray:
        """Handles invalidated by the last wave (e.g. begin_compute's displacement cascade)."""
        n = C.c_uint64()
        self._check(self.lib.fgi_last_wave_ids(self.h, None, 0, C.byref(n)), "last_wave_ids")
        ids = np.zeros(n.value, np.uint32)
        self._check(self.lib.fgi_last_wave_ids(self.h, _ptr(ids, C.c_uint32), len(ids), C.byref(n)),
                    "last_wave_ids")
        return ids

    def invalidate_all(self, stats: Optional[WaveStats] = None) -> np.ndarray:
        ids = np.zeros(self.n_handles, np.uint32)
        n = C.c_uint64()
        self._check(self.lib.fgi_invalidate_all(self.h, _ptr(ids, C.c_uint32), len(ids), C.byref(n),
                                                C.byref(stats) if stats is not None else None), "invalidate_all")
        return ids[:n.value].copy()

    def prune(self) -> PruneStats:
        ps = PruneStats()
        self._check(self.lib.fgi_prune(self.h, C.byref(ps)), "prune")
        return ps

    def prune_range(self, first: int, count: int) -> PruneStats:
        ps = PruneStats()
        self._check(self.lib.fgi_prune_range(self.h, first, count, C.byref(ps)), "prune_range")
        return ps

    def prune_step(self, batch: int, stale_pct: int) -> PruneStats:
        ps = PruneStats()
        self._check(self.lib.fgi_prune_step(self.h, batch, stale_pct, C.byref(ps)), "prune_step")
        return ps

    def release(self, handles):
        h = _u32(handles)
        self._check(self.lib.fgi_release(self.h, len(h), _ptr(h, C.c_uint32)), "release")

    def snapshot(self):
        self._check(self.lib.fgi_snapshot(self.h), "snapshot")

    def restore(self):
        self._check(self.lib.fgi_restore(self.h), "restore")

    def set_option(self, option: int, value: int):
        self._check(self.lib.fgi_set_option(self.h, option, value), "set_option")

    def stream(self) -> int:
        s = C.c_void_p()
        self._check(self.lib.fgi_stream(self.h, C.byref(s)), "stream")
        return s.value or 0


    # ---- multi-GPU partition ----
    def part_init(self, n_global: int, unique_id: bytes):
        buf = (C.c_uint8 * 128).from_buffer_copy(unique_id)
        self._check(self.lib.fgi_part_init(self.h, n_global, buf), "part_init")

    def part_init_host(self, n_global: int, group=None):
        """Join the partition with host collectives (fgi_part_init_host): every collective is an
        all-gather of host bytes through torch.distributed (`group`: a process group, default the
        world; gloo works, so the ranks may share one GPU)."""
        import torch
        import torch.distributed as dist

        world = dist.get_world_size(group)

        def allgather(_ctx, send, nbytes, recv):
            try:
                src = torch.frombuffer((C.c_uint8 * nbytes).from_address(send), dtype=torch.uint8).clone() \
                    if nbytes else torch.zeros(0, dtype=torch.uint8)
                out = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(world)]
                dist.all_gather(out, src, group=group)
                if nbytes:
                    got = torch.cat(out).numpy()   # held: a temporary's buffer may be freed before the copy
                    C.memmove(recv, got.ctypes.data, nbytes * world)
                return 0
            except Exception as e:  # reported as FGI_EDEVICE by the engine
                import sys
                print(f"fgi host all-gather failed: {e!r}", file=sys.stderr)
                return 1

        self._allgather_cb = ALLGATHER_FN(allgather)   # kept alive with the graph
        self._check(self.lib.fgi_part_init_host(self.h, n_global, C.cast(self._allgather_cb, C.c_void_p), None),
                    "part_init_host")

    def part_synth_rmat(self, scale, edge_factor, seed, stale_pct=0, stale_seed=0):
        self._check(self.lib.fgi_part_synth_rmat(self.h, scale, edge_factor, seed, stale_pct, stale_seed),
                    "part_synth_rmat")

    def part_register_nodes(self, slots, versions, state_flags=None):
        """fgi_part_register_nodes: global slot ids; every rank gets the same list."""
        s, v = _u32(slots), _u64(versions)
        f = None if state_flags is None else _u32(state_flags)
        self._check(self.lib.fgi_part_register_nodes(self.h, len(s), _ptr(s, C.c_uint32), _ptr(v, C.c_uint64),
                                                     _ptr(f, C.c_uint32)), "part_register_nodes")

    def part_load_edges(self, used, dependant, tags):
        """fgi_part_load_edges: global ids; every rank gets the same batch."""
        u, d, t = _u32(used), _u32(dependant), _u64(tags)
        self._check(self.lib.fgi_part_load_edges(self.h, len(u), _ptr(u, C.c_uint32), _ptr(d, C.c_uint32),
                                                 _ptr(t, C.c_uint64)), "part_load_edges")

    def part_invalidate(self, n_roots: int, roots_ptr: int, imm_ptr: int = 0,
                        stats: Optional[WaveStats] = None) -> int:
        n = C.c_uint64()
        self._check(self.lib.fgi_part_invalidate(self.h, n_roots, C.c_void_p(roots_ptr),
                                                 C.c_void_p(imm_ptr) if imm_ptr else None, C.byref(n),
                                                 C.byref(stats) if stats is not None else None), "part_invalidate")
        return n.value

    def part_begin_compute(self, slots, versions, has_delay=None, stats: Optional[WaveStats] = None):
        """fgi_part_begin_compute: (detached local handles on the owner / FGI_NONE, this rank's ids
        of the displacement cascade)."""
        s, v = _u32(slots), _u64(versions)
        hd = None if has_delay is None else _u8(has_delay)
        out = np.zeros(len(s), np.uint32)
        ids = np.zeros(self.n_handles, np.uint32)
        n = C.c_uint64()
        self._check(self.lib.fgi_part_begin_compute(self.h, len(s), _ptr(s, C.c_uint32), _ptr(v, C.c_uint64),
                                                    _ptr(hd, C.c_uint8), _ptr(out, C.c_uint32), _ptr(ids, C.c_uint32),
                                                    len(ids), C.byref(n),
                                                    C.byref(stats) if stats is not None else None), "part_begin_compute")
        return out, ids[:n.value].copy()

    def part_add_used(self, dependant, used) -> np.ndarray:
        d, u = _u32(dependant), _u32(used)
        out = np.zeros(len(d), np.uint32)
        self._check(self.lib.fgi_part_add_used(self.h, len(d), _ptr(d, C.c_uint32), _ptr(u, C.c_uint32),
                                               _ptr(out, C.c_uint32)), "part_add_used")
        return out

    def part_set_output(self, slots, stats: Optional[WaveStats] = None):
        h = _u32(slots)
        out_set = np.zeros(len(h), np.uint8)
        ids = np.zeros(self.n_handles, np.uint32)
        n = C.c_uint64()
        self._check(self.lib.fgi_part_set_output(self.h, len(h), _ptr(h, C.c_uint32), _ptr(out_set, C.c_uint8),
                                                 _ptr(ids, C.c_uint32), len(ids), C.byref(n),
                                                 C.byref(stats) if stats is not None else None), "part_set_output")
        return out_set, ids[:n.value].copy()

    def part_invalidate_all(self, stats: Optional[WaveStats] = None) -> np.ndarray:
        ids = np.zeros(self.n_handles, np.uint32)
        n = C.c_uint64()
        self._check(self.lib.fgi_part_invalidate_all(self.h, _ptr(ids, C.c_uint32), len(ids), C.byref(n),
                                                     C.byref(stats) if stats is not None else None),
                    "part_invalidate_all")
        return ids[:n.value].copy()

    def part_run_batch(self, steps, stats: Optional[BatchStats] = None, want_ids: bool = True):
        """fgi_part_run_batch: run_batch's steps with global slot ids; every rank passes the same batch.
        Returns (this rank's ids of the batch's cascades, per-step outputs)."""
        return self._batch(self.lib.fgi_part_run_batch, "part_run_batch", steps, stats, want_ids)

    def part_prune(self) -> PruneStats:
        ps = PruneStats()
        self._check(self.lib.fgi_part_prune(self.h, C.byref(ps)), "part_prune")
        return ps

    def part_front_stats(self):
        """(full all-gathers, delta exchanges, bytes received) of this rank's frontier exchanges."""
        f, d, b = C.c_uint64(), C.c_uint64(), C.c_uint64()
        self._check(self.lib.fgi_part_front_stats(self.h, C.byref(f), C.byref(d), C.byref(b)), "part_front_stats")
        return f.value, d.value, b.value

    def part_export_ids(self) -> np.ndarray:
        n = C.c_uint64()
        st = self.lib.fgi_part_export_ids(self.h, None, 0, C.byref(n))
        self._check(st, "part_export_ids")
        out = np.zeros(n.value, np.uint32)
        self._check(self.lib.fgi_part_export_ids(self.h, _ptr(out, C.c_uint32), n.value, C.byref(n)), "part_export_ids")
        return out


def bits_to_ids(bits: np.ndarray) -> np.ndarray:
    """Handles whose bit is set in a fgi_invalidate_bits bitmap, ascending."""
    b = np.unpackbits(np.ascontiguousarray(bits, np.uint64).view(np.uint8), bitorder="little")
    return np.flatnonzero(b).astype(np.uint32)


class Pinned:
    """fgi_alloc_pinned / fgi_free_pinned: page-locked host memory (nbytes) as a numpy view."""

    def __init__(self, nbytes: int, dtype=np.uint8):
        self.lib = load_library()
        p = C.c_void_p()
        st = self.lib.fgi_alloc_pinned(nbytes, C.byref(p))
        if st != OK:
            raise FgiError(st, f"fgi_alloc_pinned({nbytes})")
        self.ptr = p.value or 0
        n = nbytes // np.dtype(dtype).itemsize
        self.array = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), (nbytes,)).view(dtype)[:n] if nbytes else \
            np.zeros(0, dtype)

    def close(self):
        if self.ptr:
            self.lib.fgi_free_pinned(C.c_void_p(self.ptr))
            self.ptr = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def part_unique_id() -> bytes:
    lib = load_library()
    buf = (C.c_uint8 * 128)()
    st = lib.fgi_part_unique_id(buf)
    if st != OK:
        raise FgiError(st, "fgi_part_unique_id")
    return bytes(buf)


def rccl_info():
    """(ncclGetVersion, library path) of the RCCL the engine's collectives are bound to."""
    lib = load_library()
    v = C.c_int()
    buf = C.create_string_buffer(4096)
    st = lib.fgi_rccl_info(C.byref(v), buf, len(buf))
    if st != OK:
        raise FgiError(st, "fgi_rccl_info")
    return v.value, buf.value.decode(errors="replace")


def part_init_local(graphs, n_global: int):
    """Bind graphs (rank i of world len(graphs)) into an in-process partition group."""
    lib = load_library()
    arr = (C.c_void_p * len(graphs))(*[g.h.value for g in graphs])
    st = lib.fgi_part_init_local(arr, len(graphs), n_global)
    if st != OK:
        raise FgiError(st, "fgi_part_init_local: " + (lib.fgi_last_error(graphs[0].h) or b"").decode())


def part_local_invalidate(graphs, roots, immediately=None):
    lib = load_library()
    arr = (C.c_void_p * len(graphs))(*[g.h.value for g in graphs])
    r = _u32(roots)
    imm = None if immediately is None else _u8(immediately)
    stats = (WaveStats * len(graphs))()
    st = lib.fgi_part_local_invalidate(arr, len(graphs), len(r), _ptr(r, C.c_uint32), _ptr(imm, C.c_uint8), stats)
    if st != OK:
        _local_error(lib, graphs, st, "fgi_part_local_invalidate")
    return list(stats)


def _local_error(lib, graphs, st, what):
    msgs = [(lib.fgi_last_error(g.h) or b"").decode() for g in graphs]
    raise FgiError(st, what + ": " + "; ".join(m for m in msgs if m))


def part_local_run_batch(graphs, steps):
    """fgi_part_local_run_batch: the batch on every rank of an in-process group. Returns (ids of the
    batch's cascades, rank 0's then rank 1's ..., merged per-step outputs, per-rank BatchStats)."""
    lib = load_library()
    arr_g = (C.c_void_p * len(graphs))(*[g.h.value for g in graphs])
    arr, keep, outs = build_steps(steps)
    cap = max(1, sum(1 for sp in steps if sp[0] != "add_used")) * sum(g.n_handles for g in graphs)
    ids = np.empty(cap, np.uint32)
    n = C.c_uint64()
    stats = (BatchStats * len(graphs))()
    st = lib.fgi_part_local_run_batch(arr_g, len(graphs), len(steps), arr, _ptr(ids, C.c_uint32), cap, C.byref(n),
                                      stats)
    if st != OK:
        _local_error(lib, graphs, st, "fgi_part_local_run_batch")
    return ids[:n.value].copy(), outs, list(stats)


def part_local_prune(graphs):
    lib = load_library()
    arr_g = (C.c_void_p * len(graphs))(*[g.h.value for g in graphs])
    stats = (PruneStats * len(graphs))()
    st = lib.fgi_part_local_prune(arr_g, len(graphs), stats)
    if st != OK:
        _local_error(lib, graphs, st, "fgi_part_local_prune")
    return list(stats)


def header_symbols(header_path: str) -> list:
    """Names of every function declared in include/fgi.h (for the ABI export test)."""
    import re
    txt = open(header_path).read()
    return sorted(set(re.findall(r"\b(fgi_[a-z0-9_]+)\s*\(", txt)) - {"fgi_status"})
