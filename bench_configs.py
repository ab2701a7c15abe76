#!/usr/bin/env python3
"""Measurements of BASELINE.json's other configurations (bench.py is the driver's headline line,
configs[1]). One JSON line per configuration on stdout:

  layered_1m  configs[0]: 1.05M-node compute-method graph (fan-out 8, depth 6), 1k roots. The GPU
              wave and the CPU oracle (reference-faithful cascade, parallel over roots) on the
              exact same graph and roots.
  churn       configs[3]: configs[1]'s graph with 50% stale edges — (i) a wave with
              filter-on-traverse, (ii) fgi_prune (PruneUsedBy over the registry + compaction),
              (iii) the same wave after the prune.
  stream      configs[4]: streaming mix (workloads.StreamMix): 10k hubs x 1,000 leaves; per round
              the previous round's 100k invalidated leaves are recomputed (begin_compute ->
              add_used -> set_output, through the C-ABI from host arrays), delay timers fire, then
              a wave on 100 random hubs. Sustained invalidated nodes/s including insert time.

  python bench_configs.py [--only stream,churn,layered_1m] [--steps K] [--rounds R]

The streaming mix runs first: its per-call host overheads grow ~2x when it follows the CPU oracle
leg in the same process (measured: 1.9 vs 3.3 ms/round).
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def timed_waves(g, pkg, d_roots, n_roots, steps, warmup):
    """Median-free mean over `steps` (restore + wave) steps after warm-up; returns (s/step, stats)."""
    import torch
    for _ in range(warmup + 1):
        g.restore()
        g.invalidate_dev(n_roots, d_roots.data_ptr(), 0, pkg.WaveStats())
    st = pkg.WaveStats()
    g.set_option(pkg.fgi.OPT_LEVEL_TIMING, 0)   # as bench.py's headline: no per-level events in the stream
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        g.restore()
        g.invalidate_dev(n_roots, d_roots.data_ptr(), 0, st)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    g.set_option(pkg.fgi.OPT_LEVEL_TIMING, 1)
    return dt, st


def cpu_oracle_layered(cfg, roots, threads, runs=3):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import fgo  # test infrastructure, timed here only as the CPU baseline
    n = cfg["levels"] * cfg["width"]
    s, d = fgo.gen_layered(cfg["levels"], cfg["width"], cfg["fanout"], cfg["seed"])
    o = fgo.Oracle(n)
    o.load_graph(fgo.version_of(cfg["seed"], np.arange(n)), None, s, d, fgo.gen_tags(s, d, cfg["seed"]))
    o.snapshot()
    out = {}
    for th in sorted({1, threads}):
        res = []
        for i in range(runs + 1):
            o.restore()
            st = fgo.Stats()
            t = time.perf_counter()
            o.invalidate_slots(roots, None, threads=th, stats=st)
            if i:
                res.append((time.perf_counter() - t, st.v_inv, st.e_trav))
        out[th] = (statistics.median(x[0] for x in res), res[0][1], res[0][2])
    o.close()
    return out


def run_layered(pkg, W, args):
    import torch
    cfg = W.CONFIGS["layered_1m"]
    n = W.n_slots(cfg)
    g = pkg.Graph(n)
    W.build(g, cfg)
    roots = W.roots_for(g, cfg)
    _, n_edges = g.degrees()
    d_roots = torch.from_numpy(roots.astype(np.int32)).cuda()
    g.snapshot()
    s, st = timed_waves(g, pkg, d_roots, len(roots), args.steps, 3)
    v_inv, e_trav = st.v_inv // args.steps, st.e_trav // args.steps
    out = {"config": "layered_1m", "workload": "BASELINE.json configs[0]: 7 levels x 150,000 slots, fan-out 8, "
           "1,000 roots", "nodes": n, "edges": int(n_edges), "gpu": {
               "value": v_inv / s, "unit": "invalidated nodes/s", "ms_per_step": s * 1e3,
               "gteps": e_trav / s / 1e9, "v_inv": v_inv, "e_trav": e_trav,
               "levels": st.levels / args.steps, "wave_kernel_ms": st.kernel_ms / args.steps}}
    g.close()
    if not args.no_cpu:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, len(os.sched_getaffinity(0)))
        c = cpu_oracle_layered(cfg, roots, threads)
        tm, cv, ce = c[threads]
        assert cv == v_inv and ce == e_trav, "CPU oracle and engine disagree on V_inv / E_trav"
        out["cpu_baseline"] = {"value": cv / tm, "unit": "invalidated nodes/s", "cores": threads, "kind": "port",
                               "sample": "the full configs[0] workload (same graph and roots), median of 3 after "
                                         "a warm-up, parallel over roots",
                               "s_per_wave": tm, "single_thread_value": c[1][1] / c[1][0]}
        out["speedup_vs_cpu"] = out["gpu"]["value"] / out["cpu_baseline"]["value"]
    return out


def run_churn(pkg, W, args):
    import torch
    cfg = W.CONFIGS["rmat24_churn"]
    n = W.n_slots(cfg)
    g = pkg.Graph(n)
    W.build(g, cfg)
    roots = W.roots_for(g, cfg)
    _, e0 = g.degrees()
    d_roots = torch.from_numpy(roots.astype(np.int32)).cuda()
    g.snapshot()
    s1, st1 = timed_waves(g, pkg, d_roots, len(roots), args.steps, 2)
    g.restore()
    torch.cuda.synchronize()
    t = time.perf_counter()
    ps = g.prune()
    prune_s = time.perf_counter() - t
    _, e1 = g.degrees()
    g.snapshot()
    s2, st2 = timed_waves(g, pkg, d_roots, len(roots), args.steps, 2)
    k = args.steps
    # (measurement variants selected by FGI_LIBRARY may compute wrong results on purpose)
    assert st1.v_inv == st2.v_inv or os.environ.get("FGI_LIBRARY"), "a prune changed the invalidated set"
    out = {"config": "rmat24_churn", "workload": "BASELINE.json configs[3]: R-MAT 24 with 50% stale edges, "
           "4,096 roots", "nodes": n, "edges_before_prune": int(e0), "edges_after_prune": int(e1),
           "wave_before_prune": {"value": st1.v_inv / k / s1, "unit": "invalidated nodes/s", "ms_per_step": s1 * 1e3,
                                 "v_inv": st1.v_inv // k, "e_trav": st1.e_trav // k,
                                 "gteps": st1.e_trav / k / s1 / 1e9},
           "prune": {"s": prune_s, "kernel_ms": ps.kernel_ms, "old_edges": ps.old_edges, "new_edges": ps.new_edges,
                     "pool_before": ps.pool_before, "pool_after": ps.pool_after,
                     "edges_per_s": ps.old_edges / prune_s if prune_s > 0 else None},
           "wave_after_prune": {"value": st2.v_inv / k / s2, "unit": "invalidated nodes/s", "ms_per_step": s2 * 1e3,
                                "v_inv": st2.v_inv // k, "e_trav": st2.e_trav // k,
                                "gteps": st2.e_trav / k / s2 / 1e9}}
    g.close()
    return out


def run_stream(pkg, W, args):
    p = dict(W.STREAM)
    if args.rounds:
        p["rounds"] = args.rounds
    mix = W.StreamMix(p["hubs"], p["leaves_per_hub"], p["hubs_per_round"], p["delay_pct"], p["seed"])
    n = mix.n
    t = time.perf_counter()
    g = pkg.Graph(n, edge_capacity=3 * (n - p["hubs"]))
    all_slots = np.arange(n, dtype=np.uint32)
    g.register_nodes(all_slots, mix.version, mix.state_flags())
    g.load_edges(*mix.initial_edges())
    load_s = time.perf_counter() - t
    ph = dict(timers=0.0, hubs=0.0, begin=0.0, add_used=0.0, set_output=0.0, wave=0.0)
    prev = mix.roots(0)
    ids = g.invalidate(prev)          # priming wave (untimed): round 1 recomputes its leaves
    v_inv = 0
    e_edges = 0
    ws = pkg.WaveStats()
    if args.stream_mode == "batch":
        # one fgi_run_batch per round: the same calls, in the same order, as one submission
        bst = pkg.fgi.BatchStats()
        # the application's batches (the synthetic schedule) are built before the timed loop
        tb = time.perf_counter()
        batches, expect = [], []
        R = p["rounds"]
        R_prof = max(10, R // 5)   # instrumented rounds after the timed ones: the cascades' share
        for r in range(1, R + R_prof + 1):
            timers, hs, ls = mix.plan(prev)
            roots = mix.roots(r)
            steps = []
            if len(timers):
                steps.append(("invalidate", timers, np.ones(len(timers), np.uint8)))
            steps += [("begin_compute", hs, mix.new_versions(hs).copy()), ("set_output", hs),
                      ("begin_compute", ls, mix.new_versions(ls).copy(), mix.has_delay[ls]),
                      ("add_used", ls, mix.hub_of(ls)), ("set_output", ls), ("invalidate", roots)]
            batches.append(steps)
            # the round's cascades, in step order: the timers' roots (each a delayed leaf whose delay
            # the previous wave started: Invalidate(true) invalidates it), then the wave, which is
            # the root hubs plus their undelayed leaves (Computed.cs:186-198: delayed ones only start)
            ch = mix.children(roots)
            expect.append(np.concatenate([np.sort(timers), np.sort(np.concatenate([roots, ch[mix.has_delay[ch] == 0]]))]))
            e_edges += len(ls)
            prev = roots
        build_s = time.perf_counter() - tb
        # timed rounds: no per-cascade timestamps between the launches (FGI_OPT_LEVEL_TIMING=0); the
        # process's one-time cooperative-launch setup is paid by an empty batch first (like the load)
        g.set_option(pkg.fgi.OPT_LEVEL_TIMING, 0)
        g.run_batch([])
        got = []
        t0 = time.perf_counter()
        for steps in batches[:R]:
            ids, _ = g.run_batch(steps, stats=bst)
            got.append(ids)
            v_inv += len(ids)
        total = time.perf_counter() - t0
        # every timed round's ids against the schedule's closed form (after the clock stops)
        bad = [r for r, (a, b) in enumerate(zip(got, expect)) if not np.array_equal(a, b.astype(a.dtype))]
        del got
        # instrumented rounds: every cascade between HIP events
        g.set_option(pkg.fgi.OPT_LEVEL_TIMING, 1)
        pst = pkg.fgi.BatchStats()
        tp = time.perf_counter()
        for steps in batches[R:]:
            g.run_batch(steps, stats=pst)
        prof_round_ms = (time.perf_counter() - tp) / R_prof * 1e3
        out = {"config": "stream", "mode": "batch (fgi_run_batch, one per round)",
               "workload": f"BASELINE.json configs[4]: {p['hubs']} hubs x {p['leaves_per_hub']} leaves ({n} slots), "
               f"{R} rounds of one batch: delay timers (Invalidate(true)) -> begin_compute/set_output on the "
               f"previous round's {p['hubs_per_round']} hubs -> begin_compute/add_used/set_output on their leaves "
               f"-> a wave on {p['hubs_per_round']} new hubs; {p['delay_pct']}% of leaves delayed", "nodes": n,
               "value": v_inv / total, "unit": "invalidated nodes/s (sustained, insert time included)",
               "rounds": R, "ms_per_round": total / R * 1e3, "v_inv_per_round": v_inv / R,
               "recompute_nodes_per_s": e_edges / total,
               "batch_kernel_ms_per_round": bst.kernel_ms / R,
               "wave_kernel_ms_per_round": pst.wave_ms / R_prof,
               "wave_share_of_round": (pst.wave_ms / R_prof) / prof_round_ms,
               "instrumented_rounds": R_prof, "instrumented_ms_per_round": prof_round_ms,
               "host_syncs_per_round": bst.host_syncs / R, "cascades_per_round": bst.waves / R,
               "run_batch_call_ms_per_round": bst.total_ms / R, "schedule_build_ms_per_round": build_s / R * 1e3,
               "initial_load_s": load_s,
               "checked_rounds": R, "rounds_with_wrong_ids": bad,
               "note": "host arrays cross the C-ABI once per round (one pinned upload, one download of the ids); "
                       "every timed round's ids checked against the schedule's closed form (timer roots, then "
                       "the wave's hubs and undelayed leaves); node words are checked against the oracle at "
                       "this size in tests/test_gpu_full_size.py"}
        g.close()
        assert not bad, f"configs[4]: rounds {bad[:8]} returned ids other than the schedule's"
        return out
    t0 = time.perf_counter()
    for r in range(1, p["rounds"] + 1):
        timers, hs, ls = mix.plan(prev)
        a = time.perf_counter()
        if len(timers):
            v_inv += len(g.invalidate(timers, np.ones(len(timers), np.uint8)))
        b = time.perf_counter()
        g.begin_compute(hs, mix.new_versions(hs))
        g.set_output(hs)
        c = time.perf_counter()
        g.begin_compute(ls, mix.new_versions(ls), mix.has_delay[ls])
        d = time.perf_counter()
        g.add_used(ls, mix.hub_of(ls))
        e = time.perf_counter()
        g.set_output(ls)
        f = time.perf_counter()
        roots = mix.roots(r)
        ids = g.invalidate(roots, stats=ws)
        h = time.perf_counter()
        v_inv += len(ids)
        e_edges += len(ls)
        for k_, dt in zip(ph, (b - a, c - b, d - c, e - d, f - e, h - f)):
            ph[k_] += dt
        prev = roots
    total = time.perf_counter() - t0
    R = p["rounds"]
    out = {"config": "stream", "mode": "calls (one ABI call per operation)", "workload": f"BASELINE.json configs[4]: {p['hubs']} hubs x {p['leaves_per_hub']} "
           f"leaves ({n} slots), {R} rounds of (recompute the previous round's invalidated leaves: begin_compute "
           f"-> add_used -> set_output; fire delay timers) + a wave on {p['hubs_per_round']} hubs; "
           f"{p['delay_pct']}% of leaves delayed", "nodes": n,
           "value": v_inv / total, "unit": "invalidated nodes/s (sustained, insert time included)",
           "rounds": R, "ms_per_round": total / R * 1e3, "v_inv_per_round": v_inv / R,
           "add_used_edges_per_s": e_edges / ph["add_used"] if ph["add_used"] > 0 else None,
           "recompute_nodes_per_s": e_edges / (ph["begin"] + ph["add_used"] + ph["set_output"]),
           "phase_ms_per_round": {k_: v / R * 1e3 for k_, v in ph.items()},
           "wave_kernel_ms_per_round": ws.kernel_ms / R, "initial_load_s": load_s,
           "note": "host arrays cross the C-ABI each call (PCIe-inclusive), as a host layer's batches would"}
    g.close()
    return out



def dump_maps():
    """FGI_MAPS_OUT=<file>: this process's /proc/self/maps (every library mapped by now), so the PCs of
    a crash at exit (e.g. under rocprofv3) can be mapped to libraries and symbols."""
    path = os.environ.get("FGI_MAPS_OUT")
    if path:
        with open("/proc/self/maps") as src, open(path, "w") as dst:
            dst.write(src.read())


def main():
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="stream,churn,layered_1m")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--stream-mode", choices=("batch", "calls"), default="batch")
    args = ap.parse_args()
    import torch
    import _pkg
    torch.cuda.set_device(0)
    pkg = _pkg.load()
    from stl_fusion_amd import workloads as W
    runs = {"layered_1m": run_layered, "churn": run_churn, "stream": run_stream}
    for name in args.only.split(","):
        t = time.time()
        res = runs[name](pkg, W, args)
        log(f"{name}: {time.time() - t:.1f}s")
        json_out.write(json.dumps(res) + "\n")
        json_out.flush()


if __name__ == "__main__":
    main()
    dump_maps()
