"""The reference's behaviour scenarios (tests/test_oracle_scenarios.py) replayed against the engine.

Each World-based scenario there is called here with a world whose backend is the engine through
the C-ABI (stl.fusion_amd.fgi.Graph) instead of the oracle. `EngineOracle` presents the oracle's
node-handle API on top of engine handles: a node id per Computed instance, mapped to its slot while
it is registered and to a detached handle once a newer computation displaced it.
"""
import functools
import inspect

import numpy as np
import pytest

import fgo as O
import test_oracle_scenarios as S

pytestmark = pytest.mark.gpu
NONE = O.NONE


class EngineOracle:
    def __init__(self, pkg, n):
        self.g = pkg.Graph(n, n_detached=64)
        self.n = n
        self.nodes = []          # node id -> [slot, version, has_delay, engine handle]
        self.slot_last = {}
        self.home = {}           # detached handle -> slot
        self.log = []

    def _log(self, ids):
        self.log += [int(h) if h < self.n else self.home[int(h)] for h in ids]

    def begin_compute(self, slot, version, has_delay=False, stats=None):
        old = self.slot_last.get(slot)
        det = int(self.g.begin_compute([slot], [version], [int(has_delay)])[0])
        self._log(self.g.last_wave_ids())
        if old is not None and det != NONE:
            self.nodes[old][3] = det
            self.home[det] = slot
        self.nodes.append([slot, version, bool(has_delay), slot])
        nid = len(self.nodes) - 1
        self.slot_last[slot] = nid
        return nid, (old if old is not None else NONE)

    def set_output(self, h, stats=None):
        out, ids = self.g.set_output([self.nodes[h][3]])
        self._log(ids)
        return int(out[0])

    def add_used(self, dependant_h, used_h):
        return int(self.g.add_used([self.nodes[dependant_h][3]], [self.nodes[used_h][3]])[0])

    def last(self, slot):
        return self.slot_last.get(slot, NONE)

    def node_info(self, h):
        slot, ver, hd, handle = self.nodes[h]
        v, f = self.g.get_state([handle])
        if int(v[0]) != ver:                      # the handle moved on: this node is gone
            return slot, ver, 2 | (16 if hd else 0)
        return slot, ver, int(f[0])

    def current(self, slot):
        h = self.last(slot)
        if h == NONE or (self.node_info(h)[2] & 3) == 2:
            return NONE
        return h

    def invalidate_slots(self, slots, immediately=None, threads=1, stats=None):
        self._log(self.g.invalidate(slots, immediately))

    def invalidate_nodes(self, handles, immediately=None, stats=None):
        self._log(self.g.invalidate([self.nodes[h][3] for h in handles], immediately))

    def inv_log(self):
        return np.array(self.log, np.uint32)

    def clear_log(self):
        self.log = []

    def used_by(self, h):
        d, t = self.g.used_by(self.nodes[h][3])
        d = np.array([x if x < self.n else self.home[int(x)] for x in d], np.uint32)
        return d, t

    def used_count(self, h):
        return self.g.used_count(self.nodes[h][3])

    def prune(self):
        ps = self.g.prune()
        return ps.old_edges, ps.new_edges


SCENARIOS = [f for name, f in sorted(vars(S).items())
             if name.startswith("test_") and "W" in inspect.signature(f).parameters]


@pytest.mark.parametrize("scenario", SCENARIOS, ids=[f.__name__[5:] for f in SCENARIOS])
def test_engine_scenario(pkg, gpu_available, scenario):
    scenario(W=functools.partial(S.World, make=lambda n: EngineOracle(pkg, n)))
