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
