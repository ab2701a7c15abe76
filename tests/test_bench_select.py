"""bench.py's workload selection: N = 1 measures BASELINE.json
configs[1] with configs[2]'s graph on the same GPU as a sub-record (the base of the scaling curve);
N > 1 measures configs[2] exactly as strong scaling, with the weak-scaling point as a secondary record."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import _pkg  # noqa: E402
import bench  # noqa: E402

_pkg.load()
from stl_fusion_amd import workloads as W  # noqa: E402


def test_single_gpu_headline_is_configs1_with_configs2_subrecord():
    sel = bench.select_workloads(1, "rmat24", False)
    assert sel["headline"] == "rmat24" and not sel["partitioned"]
    assert sel["secondary"] == [("configs2_single_gpu", "rmat27", None)]
    cfg = W.CONFIGS["rmat24"]
    assert (cfg["scale"], cfg["edge_factor"], cfg["seed"], cfg["roots"]) == (24, 16, 0x5EED0024, 4096)


def test_multi_gpu_runs_configs2_exactly_as_strong_scaling():
    for n in (2, 4, 8):
        sel = bench.select_workloads(n, "rmat24", False)
        assert sel["headline"] == "rmat27" and sel["partitioned"] and sel["scaling"] == "strong"
        cfg = W.CONFIGS[sel["headline"]]
        # BASELINE.json configs[2]: R-MAT scale 27, edge factor 8, seed 0x5EED0027, 4,096 roots
        assert (cfg["scale"], cfg["edge_factor"], cfg["seed"], cfg["roots"], cfg["roots_seed"]) == \
            (27, 8, 0x5EED0027, 4096, 0x5EED1027)
        # the weak-scaling point stays as a secondary record: 16.8M slots per GPU
        (key, name, scale), = sel["secondary"]
        assert key == "weak_scaling" and name == "rmat24" and (1 << scale) == n * (1 << 24)


def test_explicit_configs_are_kept():
    assert bench.select_workloads(1, "rmat27", False)["headline"] == "rmat27"
    assert bench.select_workloads(1, "rmat27", False)["secondary"] == []
    sel = bench.select_workloads(1, "rmat24", True)   # --partition at N = 1: the partitioned engine
    assert sel["partitioned"] and sel["headline"] == "rmat24" and sel["secondary"] == []
    assert bench.select_workloads(1, "layered_1m", False)["secondary"] == []


def test_communicator_selection():
    """One process per GPU -> RCCL; more ranks than GPUs (a rehearsal on a smaller box) -> host collectives
    (RCCL refuses two ranks on one device); a single device -> none; FGI_PART_COMM forces either."""
    assert bench.select_comm(1, 8, False) == ""
    assert bench.select_comm(1, 1, True) == ""          # --partition at N = 1: identity collectives
    for n in (2, 4, 8):
        assert bench.select_comm(n, 8, True) == "rccl"
        assert bench.select_comm(n, 1, True) == "host"
    assert bench.select_comm(8, 4, True) == "host"
    assert bench.select_comm(2, 8, True, "host") == "host"
    assert bench.select_comm(2, 1, True, "rccl") == "rccl"


def test_multi_gpu_line_head():
    """The N > 1 line's contract fields: value = invalidated nodes of all ranks / max-over-ranks time of the K
    steps, n_gpus = N, strong scaling on configs[2], the metric named as BASELINE.json names it."""
    import json
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    sel = bench.select_workloads(8, "rmat24", False)
    cfg = W.CONFIGS[sel["headline"]]
    v_inv, elapsed, K = 41_348_860 * 20, 0.01, 20
    h = bench.line_head(8, K, 5, "rmat24", elapsed, v_inv, "R-MAT 27 (configs[2])", 1 << 27, 1_066_000_000, 4096,
                        "vertex-partition x8 (RCCL all-gather counts + all-to-all frontier)", cfg)
    assert h["metric"] == base["metric"] and h["unit"] == "invalidated nodes/s"
    assert h["n_gpus"] == 8 and h["steps"] == K and h["warmup"] == 5 and h["higher_is_better"] is True
    assert h["value"] == v_inv / elapsed and abs(h["ms_per_step"] - elapsed / K * 1e3) < 1e-12
    assert h["scaling"] == "strong" and h["vs_baseline"] is None and h["data"] == "synthetic"
    assert h["config"]["scale"] == 27 and h["config"]["edge_factor"] == 8 and h["config"]["roots"] == 4096
    assert "x8" in h["config"]["parallelism"]
    json.dumps(h)   # one JSON line
