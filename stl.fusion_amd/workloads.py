"""Benchmark workloads of BASELINE.json — seeds and shapes in one place.

Graph generation runs on the device (fgi_synth_*); this module only holds the parameters and the
root-selection rule: k = 0, 1, 2, ...: candidate = splitmix64(seed + k) % range, accepted if its
out-degree is > 0 and it was not taken yet (same rule as the oracle's fgo_gen_roots).
"""
from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1

CONFIGS = {
    # BASELINE.json configs[0]: 1M-node [ComputeMethod] graph, fan-out 8, depth 6 (7 levels)
    "layered_1m": dict(kind="layered", levels=7, width=150_000, fanout=8, seed=0x5EED0001,
                       roots=1000, roots_seed=0x5EED1001, roots_range=150_000),
    # configs[1]: R-MAT scale 24 (16M nodes, 256M generated edges), 4k roots, one MI355X
    "rmat24": dict(kind="rmat", scale=24, edge_factor=16, seed=0x5EED0024, stale_pct=0, stale_seed=0,
                   roots=4096, roots_seed=0x5EED1024),
    # configs[2]: R-MAT scale 27, edge factor 8 (~1B edges), vertex-partitioned over 2/4/8 GPUs
    "rmat27": dict(kind="rmat", scale=27, edge_factor=8, seed=0x5EED0027, stale_pct=0, stale_seed=0,
                   roots=4096, roots_seed=0x5EED1027),
    # graph-size sweep on one device (not BASELINE configs): configs[1]'s generator at scales 25 / 26
    "rmat25": dict(kind="rmat", scale=25, edge_factor=16, seed=0x5EED0025, stale_pct=0, stale_seed=0,
                   roots=4096, roots_seed=0x5EED1025),
    "rmat26": dict(kind="rmat", scale=26, edge_factor=16, seed=0x5EED0026, stale_pct=0, stale_seed=0,
                   roots=4096, roots_seed=0x5EED1026),
    # configs[3]: config 2's graph with 50% stale (version-mismatched) edges
    "rmat24_churn": dict(kind="rmat", scale=24, edge_factor=16, seed=0x5EED0024, stale_pct=50,
                         stale_seed=0x5EED00C0, roots=4096, roots_seed=0x5EED1024),
}


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = (x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15))
    with np.errstate(over="ignore"):
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def pick_roots(n_roots: int, range_: int, seed: int, out_degree: np.ndarray) -> np.ndarray:
    taken = np.zeros(range_, bool)
    out = []
    k0 = 0
    limit = range_ * 64 + 1024
    while len(out) < n_roots and k0 < limit:
        ks = np.arange(k0, k0 + 65536, dtype=np.uint64)
        with np.errstate(over="ignore"):
            c = (splitmix64(ks + np.uint64(seed)) % np.uint64(range_)).astype(np.int64)
        for x in c:
            if not taken[x] and out_degree[x] > 0:
                taken[x] = True
                out.append(x)
                if len(out) == n_roots:
                    break
        k0 += 65536
    return np.array(out, np.uint32)


def n_slots(cfg: dict) -> int:
    if cfg["kind"] == "layered":
        return cfg["levels"] * cfg["width"]
    return 1 << cfg["scale"]


def build(graph, cfg: dict) -> None:
    if cfg["kind"] == "layered":
        graph.synth_layered(cfg["levels"], cfg["width"], cfg["fanout"], cfg["seed"])
    else:
        graph.synth_rmat(cfg["scale"], cfg["edge_factor"], cfg["seed"], cfg.get("stale_pct", 0),
                         cfg.get("stale_seed", 0))


def roots_for(graph, cfg: dict) -> np.ndarray:
    deg, _ = graph.degrees()
    rng = cfg.get("roots_range", n_slots(cfg))
    return pick_roots(cfg["roots"], rng, cfg["roots_seed"], deg[:rng])


# BASELINE.json configs[4]: streaming mix — hub slots (PseudoGet(tenant, prefix)-like,
# samples/TodoApp InMemoryKeyValueStore.cs:100-112) each used by `leaves_per_hub` leaf compute
# methods; per round the leaves invalidated in the previous round are recomputed
# (ComputeMethodFunctionBase.cs:19-53: new version -> Computing -> AddUsed(hub) -> TrySetOutput),
# then a wave invalidates `hubs_per_round` random hubs. 1% of leaves have an invalidation delay
# (TodoApp ITodos.GetSummary, InvalidationDelay = 1, samples/TodoApp/Abstractions/ITodos.cs:51):
# a wave only starts their delay; the host timer fires them next round with immediately = true.
STREAM = dict(hubs=10_000, leaves_per_hub=1_000, rounds=100, hubs_per_round=100, delay_pct=1,
              seed=0x5EED00E0)


class StreamMix:
    """Deterministic operation schedule of the streaming mix. Slots: hubs [0, H), leaves
    [H, H + H*L); leaf H + h*L + j uses hub h. Versions are minted on the host (a new version is the
    old one + 2: odd, positive, != old — LTagVersionGenerator.NextVersion's contract,
    src/Stl/Versioning/Providers/LTagVersionGenerator.cs:13-20)."""

    def __init__(self, hubs, leaves_per_hub, hubs_per_round, delay_pct, seed):
        self.H, self.L, self.k, self.seed = hubs, leaves_per_hub, hubs_per_round, seed
        self.n = hubs + hubs * leaves_per_hub
        slots = np.arange(self.n, dtype=np.uint64)
        self.version = (splitmix64(slots ^ np.uint64(seed)) & np.uint64((1 << 54) - 1)) | np.uint64(1)
        leaf = np.arange(hubs * leaves_per_hub, dtype=np.uint64)
        h = splitmix64(leaf ^ np.uint64(seed ^ 0xDE1A))
        self.has_delay = np.zeros(self.n, np.uint8)
        self.has_delay[hubs:] = ((h % np.uint64(100)) < np.uint64(delay_pct)).astype(np.uint8)
        self.round = 0

    def initial_edges(self):
        """(used, dependant, tag) of every leaf -> hub dependency, for fgi_load_edges."""
        leaf = np.arange(self.H, self.n, dtype=np.uint32)
        hub = ((leaf - self.H) // self.L).astype(np.uint32)
        return hub, leaf, self.version[leaf]

    def state_flags(self):
        """Initial flags: everything Consistent (state 1), hasDelay bit 4 on delayed leaves."""
        return (np.uint32(1) | (self.has_delay.astype(np.uint32) << np.uint32(4))).astype(np.uint32)

    def roots(self, r):
        """Distinct hubs for round r's wave."""
        ks = np.arange(self.k * 4, dtype=np.uint64) + np.uint64(r * self.k * 4)
        c = (splitmix64(ks + np.uint64(self.seed)) % np.uint64(self.H)).astype(np.int64)
        _, first = np.unique(c, return_index=True)
        return c[np.sort(first)][: self.k].astype(np.uint32)

    def children(self, hubs):
        hubs = np.asarray(hubs, np.int64)
        return (self.H + hubs[:, None] * self.L + np.arange(self.L)[None, :]).ravel().astype(np.uint32)

    def delayed_children(self, hubs):
        c = self.children(hubs)
        return c[self.has_delay[c] != 0]

    def new_versions(self, slots):
        self.version[slots] += np.uint64(2)
        return self.version[slots]

    def plan(self, prev_roots):
        """Round r's recompute work after round r-1's wave on `prev_roots`: the delayed leaves whose
        timers fire (Invalidate(immediately: true)), the hubs to recompute, and every leaf of those
        hubs (the wave invalidated the undelayed ones, the timers the rest)."""
        prev = np.asarray(prev_roots, np.uint32)
        return self.delayed_children(prev), prev, self.children(prev)

    def hub_of(self, leaves):
        return ((np.asarray(leaves, np.int64) - self.H) // self.L).astype(np.uint32)
