#!/usr/bin/env python3
"""Benchmark: batched cascading invalidation (Computed.Invalidate() cascade) on MI355X.

One step = reset the node table from a pristine on-device copy (fgi_restore, ~0.2 GB of copies)
+ one invalidation wave from the workload's root batch, with the roots already resident in HBM.
Both are inside the timed region. Rank 0 prints one JSON line (the driver's contract).

  python bench.py [--gpus N --steps K --warmup W] [--config rmat24] [--no-cpu]

N=1 runs BASELINE.json configs[1] (R-MAT scale 24, 4,096 roots, one MI355X). The CPU baseline leg
times the C++ restatement of the reference cascade (oracle/, parallelised over roots) on a bounded
sample of the same workload family on this host's cores.
"""
import argparse
import glob
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "invalidated nodes/sec + GTEPS at 1/2/4/8 MI355X; achieved HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cpu_info():
    """What the CPU baseline runs on: nproc (honours the box's OMP_NUM_THREADS share), the cgroup
    CPU quota, the affinity mask size and the lscpu model name."""
    import subprocess
    info = {"affinity": len(os.sched_getaffinity(0))}
    try:
        info["nproc"] = int(subprocess.run(["nproc"], capture_output=True, text=True).stdout.strip())
    except (OSError, ValueError):
        info["nproc"] = info["affinity"]
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        info["cgroup_cpus"] = None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        info["cgroup_cpus"] = None
    try:
        for line in subprocess.run(["lscpu"], capture_output=True, text=True).stdout.splitlines():
            if line.startswith("Model name:"):
                info["model"] = line.split(":", 1)[1].strip()
    except OSError:
        pass
    return info


def peak_rss_gb():
    try:
        for line in open("/proc/self/status"):
            if line.startswith("VmHWM:"):
                return int(line.split()[1]) / 2**20
    except OSError:
        pass
    return None


def cpu_baseline(threads: int, cfg: dict, scale: int, gpu_roots=None, gpu_ids=None, runs=5, single=False):
    """Time the oracle (reference-faithful CPU cascade: per-node mutex, HashSetSlim3 `_usedBy`,
    hash registry; oracle/fgo.cpp restating Computed.cs:162-230) parallel over roots. At the
    workload's own scale it builds the IDENTICAL graph and root batch (same generator and seeds;
    the roots are checked equal to the GPU's); a smaller --cpu-scale gives a labelled sample.
    SURVEY.md §8(d): one warm-up wave, then `runs` timed waves, each from a restored pristine copy; the
    median is reported. The oracle's invalidated set is compared with the GPU's (gpu_ids) as a set.
    single: one more timed wave at T = 1 (a minute at configs[1]; off by default)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import fgo  # test infrastructure: the CPU restatement, used here only as the baseline
    fgo.set_threads(threads)
    seed = cfg["seed"]
    n = 1 << scale
    t0 = time.time()
    s, d = fgo.gen_rmat(scale, cfg["edge_factor"], seed)
    tags = fgo.gen_tags(s, d, seed, cfg.get("stale_pct", 0), cfg.get("stale_seed", 0))
    o = fgo.Oracle(n)
    o.load_graph(fgo.version_of(seed, np.arange(n)), None, s, d, tags)
    n_roots = cfg["roots"] if scale == cfg["scale"] else max(64, cfg["roots"] >> (cfg["scale"] - scale))
    r = fgo.gen_roots(n_roots, n, cfg["roots_seed"], np.bincount(s, minlength=n))
    m = len(s)
    del s, d, tags
    identical_roots = gpu_roots is not None and scale == cfg["scale"] and np.array_equal(r, gpu_roots)
    o.snapshot()
    build_s = time.time() - t0

    def timed(th):
        o.restore()
        st = fgo.Stats()
        o.clear_log()
        t = time.perf_counter()
        o.invalidate_slots(r, None, threads=th, stats=st)
        return time.perf_counter() - t, st

    out = {}
    times = []
    st = None
    for k in range(runs + 1):   # run 0 is the warm-up
        dt, st = timed(threads)
        if k:
            times.append(dt)
        log(f"cpu baseline T={threads} run {k}{' (warm-up)' if k == 0 else ''}: {dt:.2f} s, {st.v_inv} nodes")
    same_set = None
    if gpu_ids is not None and scale == cfg["scale"]:
        same_set = bool(np.array_equal(np.sort(o.inv_log()), np.sort(gpu_ids)))
    out[threads] = dict(s=statistics.median(times), runs=times, v_inv=st.v_inv, e_trav=st.e_trav)
    if single and threads != 1:
        dt, st1 = timed(1)
        out[1] = dict(s=dt, runs=[dt], v_inv=st1.v_inv, e_trav=st1.e_trav)
        log(f"cpu baseline T=1: {dt:.2f} s")
    o.close()
    return out, build_s, m, len(r), identical_roots, same_set


def profiled_traffic(kname, config_scale, live_avg_ms):
    """HBM bytes per launch of `kname` from the newest committed rocprofv3 PMC summary of this bench
    configuration (profiles/<tag>_summary.json, made by profiles/summarize.py: 2 x FETCH_SIZE +
    WRITE_SIZE per MI355X_MICROARCH.md). Used only if that run's average launch time is within 25%
    of the live one (same kernel build); otherwise (None, reason)."""
    here = os.path.dirname(os.path.abspath(__file__))
    import re

    def order(path):   # r9a < r10b < r11c1: by round number, then the rest of the tag
        m = re.match(r"r(\d+)(.*)_summary\.json$", os.path.basename(path))
        return (int(m.group(1)), m.group(2)) if m else (-1, path)
    cands = sorted(glob.glob(os.path.join(here, "profiles", "r*_summary.json")), key=order)
    for path in reversed(cands):
        try:
            doc = json.load(open(path))
            bj = path.replace("_summary.json", "_bench_under_rocprof.json")
            bcfg = json.load(open(bj)).get("config", {}) if os.path.exists(bj) else {}
        except (OSError, ValueError):
            continue
        k = doc.get("kernels", {}).get(kname)
        if not k or "hbm_bytes_per_launch" not in k or bcfg.get("scale") != config_scale:
            continue
        prof_ms = k["avg_launch_us"] / 1e3
        rel = os.path.relpath(path, here)
        if live_avg_ms <= 0 or abs(prof_ms - live_avg_ms) > 0.25 * live_avg_ms:
            return None, f"{rel}: stale (profiled avg {prof_ms:.4f} ms vs live {live_avg_ms:.4f} ms)"
        return k["hbm_bytes_per_launch"], rel
    return None, "no matching profiles/*_summary.json"



def dump_maps():
    """FGI_MAPS_OUT=<file>: this process's /proc/self/maps (every library mapped by now), so the PCs of
    a crash at exit (e.g. under rocprofv3) can be mapped to libraries and symbols."""
    path = os.environ.get("FGI_MAPS_OUT")
    if path:
        with open("/proc/self/maps") as src, open(path, "w") as dst:
            dst.write(src.read())


def select_workloads(world: int, config: str, partition: bool) -> dict:
    """Which workloads a run measures (pinned by tests/test_bench_select.py).

    N = 1: the headline is `config` (default rmat24 = BASELINE.json configs[1], the configuration the
    metric is quoted on and which fits one GPU); with the default config the line also carries a
    `configs2_single_gpu` sub-record — configs[2]'s graph on the same GPU, the base of the 2/4/8-GPU
    curve. N > 1: BASELINE.json configs[2] exactly (R-MAT 27, edge factor 8, seed 0x5EED0027, 4,096
    roots) over the N ranks — strong scaling, the total work fixed — and, secondary, the weak-scaling
    point (configs[1]'s generator at scale 24 + log2 N, 16.8 M slots per GPU)."""
    out = {"headline": config, "scaling": "weak", "secondary": []}
    partitioned = world > 1 or partition
    if world > 1 and config in ("rmat24", "rmat27"):
        out["headline"] = "rmat27"
        out["scaling"] = "strong"
        out["secondary"] = [("weak_scaling", "rmat24", 24 + (world - 1).bit_length())]
    elif world == 1 and config == "rmat24" and not partitioned:
        out["secondary"] = [("configs2_single_gpu", "rmat27", None)]
    out["partitioned"] = partitioned
    return out


def select_comm(world: int, n_gpus: int, partitioned: bool, forced: str = "") -> str:
    """The partition's communicator (pinned by tests/test_bench_select.py): none for a single device; RCCL
    with one process per GPU; host collectives (torch.distributed over gloo, fgi_part_init_host) when the
    ranks outnumber the node's GPUs (RCCL refuses two ranks on one device); FGI_PART_COMM forces either."""
    if not partitioned:
        return ""
    if forced:
        return forced
    if world <= 1:
        return ""
    return "host" if world > max(1, n_gpus) else "rccl"


def line_head(world, steps, warmup, config, elapsed, v_inv, workload, n, n_edges, n_roots, parallelism, cfg) -> dict:
    """The bench line's contract fields (pinned by tests/test_bench_select.py): value = the invalidated
    nodes of all ranks over the max-over-ranks time of the K timed steps."""
    return {
        "metric": METRIC,
        "value": v_inv / elapsed,
        "unit": "invalidated nodes/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": elapsed / steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if config in ("rmat24", "rmat27") else "weak",
        "scaling_note": ("N > 1 runs BASELINE.json configs[2] (R-MAT 27, edge factor 8) over the N GPUs: total work "
                         "fixed. At N = 1 the headline is configs[1] (the metric's one-GPU configuration) and the "
                         "curve's base is the `configs2_single_gpu` sub-record (configs[2]'s graph on this GPU)"),
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic",
        "config": {
            "workload": workload,
            "nodes": n, "edges": int(n_edges), "roots": int(n_roots),
            "parallelism": parallelism,
            "scale": cfg.get("scale"), "edge_factor": cfg.get("edge_factor"),
        },
    }


def main():
    # Libraries (RCCL prints a banner on communicator init) must not write to stdout: the driver
    # reads exactly one JSON line from it. Route fd 1 to stderr and keep a handle on the real one.
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="rmat24")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-scale", type=int, default=0,
                    help="R-MAT scale of the CPU baseline (default: the workload's own, i.e. the identical graph)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (host roots -> host ids) leg")
    ap.add_argument("--no-pipelined", action="store_true",
                    help="skip the pipelined (asynchronous) leg (profiling runs: the last waves are then the timed ones)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary workloads (configs2_single_gpu / weak_scaling; profiling runs)")
    ap.add_argument("--partition", action="store_true",
                    help="use the partitioned RCCL engine even at N=1 (it is always used for N>1)")
    ap.add_argument("--cpu-runs", type=int, default=5, help="timed CPU waves after one warm-up (median reported)")
    ap.add_argument("--no-cpu-single", action="store_true",
                    help="skip the single-threaded CPU wave (one wave at T = 1 on the identical graph, ~1 min)")
    ap.add_argument("--cpu-c2-scale", type=int, default=25,
                    help="R-MAT scale of the labelled configs[2] CPU sample (configs[2]'s generator; 0 skips it)")
    ap.add_argument("--scale", type=int, default=0,
                    help="rehearsals and tests only: the headline workload's generator at this R-MAT scale")
    args = ap.parse_args()

    import torch
    import _pkg

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = local_rank % max(1, n_gpus_visible())
    torch.cuda.set_device(gpu)
    dist = None
    if world > 1:
        import datetime
        import torch.distributed as dist
        # fail fast: every wait of a rank on its peers is bounded (the engine's RCCL init and collectives,
        # its host waits, torch's bookkeeping group) and a failure exits non-zero naming the rank and the
        # collective (main's caller), instead of the run hanging until the driver's limit
        os.environ.setdefault("FGI_WAIT_TIMEOUT_S", "240")
        os.environ.setdefault("FGI_RCCL_INIT_TIMEOUT_S", "180")
        pg_timeout = datetime.timedelta(seconds=int(os.environ.get("FGI_BENCH_TIMEOUT_S", "600")))
        # The engine's collectives run over RCCL through libfgi's own communicator (fgi_part_init,
        # /opt/rocm's librccl). torch's group carries only the bench's bookkeeping — the communicator's
        # unique id, the barriers around the timed region, the max of the per-rank times, the root
        # degrees — so it is a gloo group: the process then holds one RCCL instance, the engine's
        # (FGI_BENCH_TORCH_BACKEND=nccl selects torch's RCCL for it instead).
        backend = os.environ.get("FGI_BENCH_TORCH_BACKEND", "gloo")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu), timeout=pg_timeout)
        else:
            dist.init_process_group(backend, timeout=pg_timeout)
    tdev = "cpu" if (dist is not None and dist.get_backend() != "nccl") else f"cuda:{gpu}"

    pkg = _pkg.load()
    from stl_fusion_amd import workloads as W
    sel = select_workloads(world, args.config, args.partition)
    partitioned = sel["partitioned"]
    # one process per GPU; ranks beyond the node's GPUs (a rehearsal of N ranks on a smaller box) share
    # device local_rank % count, and then the engine's collectives go through the host (torch's gloo
    # group, fgi_part_init_host): RCCL refuses two ranks on one GPU
    comm = select_comm(world, n_gpus_visible(), partitioned, os.environ.get("FGI_PART_COMM", ""))
    knobs = (("FGI_PULL_ALPHA", "OPT_PULL_ALPHA"), ("FGI_PULL_BETA", "OPT_PULL_BETA"), ("FGI_PULL_TPB", "OPT_PULL_TPB"),
             ("FGI_PART_PLAN", "OPT_PART_PLAN"), ("FGI_PROBE_SUMMARY", "OPT_PROBE_SUMMARY"),
             ("FGI_HOT_HEADS", "OPT_HOT_HEADS"))

    def build(name, scale=None):
        """The workload's graph (single device, or this rank's partition) and its root batch."""
        cfg = dict(W.CONFIGS[name])
        if scale:
            cfg["scale"] = scale
        elif args.scale and name == sel["headline"]:
            cfg["scale"] = args.scale
        n = W.n_slots(cfg)
        t0 = time.time()
        if partitioned:
            if cfg["kind"] != "rmat":
                raise SystemExit("the partitioned engine runs R-MAT workloads")
            block = -(-n // world)
            g = pkg.Graph(block, device=gpu, rank=rank, world=world)
            if comm == "host":
                g.part_init_host(n)
            else:
                uid = [pkg.fgi.part_unique_id() if rank == 0 else None]
                if dist:
                    dist.broadcast_object_list(uid, src=0)
                g.part_init(n, uid[0])
            g.part_synth_rmat(cfg["scale"], cfg["edge_factor"], cfg["seed"], cfg.get("stale_pct", 0),
                              cfg.get("stale_seed", 0))
            n_local = min(block, n - rank * block)
            deg_local, _ = g.degrees()
            mine = torch.zeros(block, dtype=torch.int32, device=tdev)
            mine[:n_local] = torch.from_numpy(deg_local[:n_local].astype(np.int32)).to(mine.device)
            if dist and tdev == "cpu":
                parts = [torch.zeros(block, dtype=torch.int32) for _ in range(world)]
                dist.all_gather(parts, mine)
                deg = torch.cat(parts)
            elif dist:
                deg = torch.zeros(block * world, dtype=torch.int32, device=tdev)
                dist.all_gather_into_tensor(deg, mine)
            else:
                deg = mine
            deg_all = deg.cpu().numpy()[:n]
            roots = W.pick_roots(cfg["roots"], n, cfg["roots_seed"], deg_all)
            n_edges = int(deg_all.astype(np.int64).sum())
        else:
            g = pkg.Graph(n, device=gpu)
            W.build(g, cfg)
            roots = W.roots_for(g, cfg)
            _, n_edges = g.degrees()
        for k, v in knobs:
            if os.environ.get(k):   # measurement knobs (results never depend on them)
                g.set_option(getattr(pkg.fgi, v), int(os.environ[k]))
        g.snapshot()
        build_s = time.time() - t0
        log(f"[rank {rank}] built {name} (scale {cfg.get('scale')}): {n} slots, {n_edges} edges, "
            f"{len(roots)} roots in {build_s:.1f}s, partitioned={partitioned}, comm={comm or 'none'}")
        return g, cfg, n, roots, n_edges, build_s

    def measure(g, roots):
        """W untimed warm-up steps, then K timed steps between barriers (max over ranks), then the
        same K steps again with per-level HIP events (the roofline figures)."""
        if os.environ.get("FGI_BENCH_DROP_RANK") == str(rank):
            # tests only: this rank leaves before its first wave, as a rank that died would; its peers'
            # first collective must then fail within the bounded waits, naming itself
            log(f"[rank {rank}] FGI_BENCH_DROP_RANK: leaving before the first wave")
            os._exit(0)
        d_roots = torch.from_numpy(roots.astype(np.int32)).to(f"cuda:{gpu}")

        def step(stats):
            g.restore()
            if partitioned:
                return g.part_invalidate(len(roots), d_roots.data_ptr(), 0, stats)
            return g.invalidate_dev(len(roots), d_roots.data_ptr(), 0, stats)

        # the first wave may build the pull dependency-list cache (a per-topology index, like the
        # rows themselves); it is timed separately and reported, never inside the timed steps
        t_first = time.perf_counter()
        step(pkg.WaveStats())
        torch.cuda.synchronize()
        first_wave_s = time.perf_counter() - t_first
        for _ in range(args.warmup):
            step(pkg.WaveStats())
        # headline: K steps with no per-level HIP events in the stream; the roofline figures come from
        # a second, instrumented pass of the same steps, which times every k_level launch on the
        # engine's stream
        st = pkg.WaveStats()
        g.set_option(pkg.fgi.OPT_LEVEL_TIMING, 0)
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t_start = time.perf_counter()
        for _ in range(args.steps):
            step(st)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        elapsed = time.perf_counter() - t_start
        g.set_option(pkg.fgi.OPT_LEVEL_TIMING, 1)
        st_k = pkg.WaveStats()
        t_k = time.perf_counter()
        for _ in range(args.steps):
            step(st_k)
        torch.cuda.synchronize()
        instrumented_ms = (time.perf_counter() - t_k) / args.steps * 1e3
        v_inv, e_trav, e_match = st.v_inv, st.e_trav, st.e_match
        pipe = None
        if not partitioned and not args.no_pipelined:
            # pipelined leg (fgi_invalidate_async / fgi_wave_wait, ComputedExt.WhenInvalidated): the next
            # wave is queued before the previous one is waited for, so the host's wait, the published
            # counters' read and the next wave's launches overlap the device's work
            g.set_option(pkg.fgi.OPT_LEVEL_TIMING, 0)
            st_p = pkg.WaveStats()

            def pipeline(k_steps, stats):
                prev, counts = None, []
                for _ in range(k_steps):
                    g.restore()
                    t = g.invalidate_async(len(roots), d_roots.data_ptr())
                    if prev is not None:
                        counts.append(g.wave_wait(prev, stats)[0])
                    prev = t
                counts.append(g.wave_wait(prev, stats)[0])
                return counts

            pipeline(max(2, args.warmup), pkg.WaveStats())
            if dist:
                dist.barrier()
            torch.cuda.synchronize()
            t_p = time.perf_counter()
            counts = pipeline(args.steps, st_p)
            torch.cuda.synchronize()
            p_s = time.perf_counter() - t_p
            g.set_option(pkg.fgi.OPT_LEVEL_TIMING, 1)
            pipe = {"ms_per_step": p_s / args.steps * 1e3, "value": st_p.v_inv / p_s,
                    "v_inv_per_step": st_p.v_inv // args.steps,
                    "same_counts_as_sync": bool(all(c == v_inv // args.steps for c in counts)
                                               and st_p.v_inv == v_inv),
                    "note": "restore + fgi_invalidate_async(wave k) + fgi_wave_wait(wave k-1): two waves in "
                            "flight; the same roots and graph as the headline's synchronous steps"}
        if dist:
            t = torch.tensor([elapsed], dtype=torch.float64, device=tdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
            c = torch.tensor([v_inv, e_trav, e_match], dtype=torch.float64, device=tdev)
            dist.all_reduce(c, op=dist.ReduceOp.SUM)
            v_inv, e_trav, e_match = int(c[0].item()), int(c[1].item()), int(c[2].item())
        return dict(st=st, st_k=st_k, elapsed=elapsed, first_wave_s=first_wave_s, instrumented_ms=instrumented_ms,
                    v_inv=v_inv, e_trav=e_trav, e_match=e_match, pipelined=pipe)

    def brief(m, cfg, n, roots, n_edges, build_s):
        """A secondary workload's figures (the same measurement as the headline's)."""
        st, st_k, K = m["st"], m["st_k"], args.steps
        return {"workload": workload_name(cfg), "nodes": n, "edges": int(n_edges), "roots": int(len(roots)),
                "scale": cfg.get("scale"), "edge_factor": cfg.get("edge_factor"),
                "value": m["v_inv"] / m["elapsed"], "unit": "invalidated nodes/s",
                "ms_per_step": m["elapsed"] / K * 1e3, "gteps": m["e_trav"] / m["elapsed"] / 1e9,
                "v_inv_per_step": m["v_inv"] // K, "e_trav_per_step": m["e_trav"] // K,
                "levels_per_step": st.levels / K, "pull_levels_per_step": st.pull_levels / K,
                "host_syncs_per_step": st.host_syncs / K, "wave_kernel_ms": st.kernel_ms / K,
                "pull_ms_per_step": st_k.pull_ms / K, "push_ms_per_step": st_k.expand_ms / K,
                "first_wave_s": m["first_wave_s"], "build_s": build_s,
                "pipelined": m["pipelined"],
                "roofline": kernel_roofline(st_k, K, cfg),
                "parallelism": parallelism(), "n_gpus": world}

    def kernel_roofline(st_k, K, cfg):
        """k_level's achieved GB/s (algorithmic bytes / measured launch time, the instrumented pass) against
        the HBM peak, and the PMC traffic of the matching committed profile (profiled_traffic)."""
        k_ms = st_k.pull_ms + st_k.expand_ms
        k_bytes = st_k.pull_bytes + st_k.expand_bytes
        k_launches = st_k.pull_launches + st_k.expand_launches
        gbs = (k_bytes / (k_ms * 1e-3) / 1e9) if k_ms > 0 else 0.0
        traffic, src = profiled_traffic("k_level", cfg.get("scale"), k_ms / max(1, k_launches))
        return {"bound": "hbm", "kernel": "k_level", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": gbs / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": src,
                "launches_per_step": k_launches / K, "avg_launch_ms": k_ms / max(1, k_launches),
                "alg_bytes_per_launch": k_bytes / max(1, k_launches)}

    def parallelism():
        if not partitioned:
            return "single"
        how = "host (gloo) collectives" if comm == "host" else "RCCL all-gather counts + all-to-all frontier"
        return f"vertex-partition x{world} ({how})"

    def workload_name(cfg):
        names = {("rmat", 24, 16): "R-MAT scale 24 (16,777,216 nodes, 268,435,456 generated edges, dedup), "
                                   "4,096-root batched invalidation (BASELINE.json configs[1])",
                 ("rmat", 27, 8): "R-MAT scale 27, edge factor 8 (134,217,728 nodes, 1,073,741,824 generated edges, "
                                  "dedup), 4,096 roots (BASELINE.json configs[2])",
                 ("layered", None, None): "1.05M-node compute-method graph, fan-out 8, depth 6, 1k roots (configs[0])"}
        key = (cfg["kind"], cfg.get("scale"), cfg.get("edge_factor"))
        if cfg.get("stale_pct"):
            return "configs[1] graph with 50% stale edges (configs[3])"
        return names.get(key, names.get((cfg["kind"], None, None)) if cfg["kind"] == "layered" else
                         f"R-MAT scale {cfg.get('scale')}, edge factor {cfg.get('edge_factor')} "
                         f"({'weak-scaling point: configs[1] generator, 16.8M slots per GPU' if partitioned else 'size sweep'})")

    g, cfg, n, roots, n_edges, build_s = build(sel["headline"])
    m = measure(g, roots)
    st, st_k = m["st"], m["st_k"]
    elapsed = m["elapsed"]

    # end-to-end leg (SURVEY.md §8(d)'s t: root H2D -> wave -> V_inv D2H complete): fgi_invalidate
    # with the roots in host memory and the invalidated ids copied into a pinned host buffer
    e2e = None
    ids_host = None
    if not partitioned and not args.no_e2e:
        out_host = torch.empty(g.n_handles, dtype=torch.int32).pin_memory()
        g.set_option(pkg.fgi.OPT_LEVEL_TIMING, 0)
        for _ in range(max(1, args.warmup)):
            g.restore()
            g.invalidate_into(roots, out_host.data_ptr(), g.n_handles)
        st_e = pkg.WaveStats()
        torch.cuda.synchronize()
        t_e = time.perf_counter()
        n_out = 0
        for _ in range(args.steps):
            g.restore()
            n_out = g.invalidate_into(roots, out_host.data_ptr(), g.n_handles, st_e)
        torch.cuda.synchronize()
        e2e_s = time.perf_counter() - t_e
        g.set_option(pkg.fgi.OPT_LEVEL_TIMING, 1)
        ids_leg = {"ms_per_step": e2e_s / args.steps * 1e3, "value": st_e.v_inv / e2e_s,
                   "ids_copied_per_step": n_out, "d2h_bytes_per_step": 4 * n_out,
                   "note": "restore + fgi_invalidate(host roots -> pinned host id list)"}
        ids_host = out_host[:n_out].numpy().astype(np.uint32).copy()
        del out_host
        # the same with the invalidated set returned as a bitmap over handles (fgi_invalidate_bits):
        # n_handles / 8 bytes cross PCIe instead of 4 B per invalidated node
        words = (g.n_handles + 63) // 64
        pin = pkg.fgi.Pinned(words * 8, np.uint64)
        g.set_option(pkg.fgi.OPT_LEVEL_TIMING, 0)
        for _ in range(max(1, args.warmup)):
            g.restore()
            g.invalidate_bits(roots, out_ptr=pin.ptr)
        st_b = pkg.WaveStats()
        torch.cuda.synchronize()
        t_b = time.perf_counter()
        for _ in range(args.steps):
            g.restore()
            g.invalidate_bits(roots, stats=st_b, out_ptr=pin.ptr)
        torch.cuda.synchronize()
        b_s = time.perf_counter() - t_b
        g.set_option(pkg.fgi.OPT_LEVEL_TIMING, 1)
        bit_ids = np.nonzero(np.unpackbits(pin.array.view(np.uint8), bitorder="little"))[0]
        pin.close()
        e2e = {"ms_per_step": b_s / args.steps * 1e3, "value": st_b.v_inv / b_s,
               "gteps": st_b.e_trav / b_s / 1e9,
               "output": "bitmap", "d2h_bytes_per_step": 8 * words, "bits_set": int(len(bit_ids)),
               "same_set_as_ids": bool(np.array_equal(bit_ids, np.sort(ids_host))),
               "note": "SURVEY.md §8(d)'s t: restore + fgi_invalidate_bits (roots H2D from host memory, wave, "
                       "invalidated set D2H into a pinned host bitmap over handles); PCIe-inclusive, so never "
                       "`value` (the bench contract: inputs resident in HBM)",
               "ids_output": ids_leg}

    if e2e is None and not partitioned:
        g.restore()
        ids_host = np.asarray(g.invalidate(roots), np.uint32)
    v_inv, e_trav, e_match_all = m["v_inv"], m["e_trav"], m["e_match"]
    try:
        rv, rpath = pkg.fgi.rccl_info()
        # libfgi resolves RCCL from /opt/rocm's librccl.so.1 at run time (RTLD_LOCAL, part.hip rccl()),
        # so torch's bundled librccl, loaded first in this process, does not take its place
        linked = "/opt/rocm"
        differs = not os.path.realpath(rpath).startswith(os.path.realpath(linked))
        rccl = {"version": rv, "path": rpath, "linked": linked + "/lib/librccl.so.1",
                "differs_from_linked": differs, "torch_loaded_first": True}
        log(f"[rank {rank}] libfgi RCCL: ncclGetVersion {rv} from {rpath}")
        if differs:
            log(f"[rank {rank}] WARNING: libfgi is bound to {rpath}, not {linked}/lib/librccl.so.1")
    except Exception as e:  # informational only
        rccl = {"error": repr(e)}
    g.close()

    value = v_inv / elapsed
    gteps = e_trav / elapsed / 1e9
    # roofline of the dominant kernel: k_level (push and pull levels are one kernel; the split is
    # reported beside it)
    kname = "k_level"
    k_ms = st_k.pull_ms + st_k.expand_ms
    k_bytes = st_k.pull_bytes + st_k.expand_bytes
    k_launches = st_k.pull_launches + st_k.expand_launches
    k_gbs = (k_bytes / (k_ms * 1e-3) / 1e9) if k_ms > 0 else 0.0
    traffic, traffic_src = profiled_traffic(kname, cfg.get("scale"), k_ms / max(1, k_launches))
    wave_gbs = (st.alg_bytes / (st.kernel_ms * 1e-3) / 1e9) if st.kernel_ms > 0 else 0.0
    result = line_head(world, args.steps, args.warmup, args.config, elapsed, v_inv, workload_name(cfg), n, n_edges,
                       len(roots), parallelism(), cfg)
    result.update({
        "gteps": gteps,
        "v_inv_per_step": v_inv // args.steps,
        "e_trav_per_step": e_trav // args.steps,
        "e_trav_semantics": ("sum of |_usedBy| over the invalidated nodes at wave start; rows keep RemoveUsedBy'd "
                             "entries until the next prune, so later waves of a mutated graph count them. Here every "
                             "timed wave runs on the freshly built graph (restore only), which has none"),
        "levels_per_step": st.levels / args.steps,
        "host_syncs_per_step": st.host_syncs / args.steps,
        "wave_kernel_ms": st.kernel_ms / args.steps,
        "wave_alg_gbs": wave_gbs,
        "pull_levels_per_step": st.pull_levels / args.steps,
        "remote_msgs_per_step": st.remote_msgs / args.steps,
        "first_wave_s": m["first_wave_s"],
        "build_s": build_s,
        "roofline": {
            "bound": "hbm",
            "kernel": kname,
            "achieved": k_gbs,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": k_gbs / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "launches_per_step": k_launches / args.steps,
            "avg_launch_ms": k_ms / max(1, k_launches),
            "alg_bytes_per_launch": k_bytes / max(1, k_launches),
            "timing_pass_ms_per_step": m["instrumented_ms"],
            "push_levels": {"ms_per_step": st_k.expand_ms / args.steps,
                            "launches_per_step": st_k.expand_launches / args.steps,
                            "gbs": (st_k.expand_bytes / (st_k.expand_ms * 1e-3) / 1e9) if st_k.expand_ms > 0 else 0.0},
            "pull_levels": {"ms_per_step": st_k.pull_ms / args.steps,
                            "launches_per_step": st_k.pull_launches / args.steps,
                            "gbs": (st_k.pull_bytes / (st_k.pull_ms * 1e-3) / 1e9) if st_k.pull_ms > 0 else 0.0},
        },
        "rccl": rccl,
    })
    # SURVEY.md §8(d)'s layout-A formula B = 28 V_exp + 24 E_trav + 4 E_match + 4 R counts every
    # edge of every expanded node, as a push-only traversal would read them. Pull levels read
    # dependency-list heads instead of those edges, so B / t is a push-equivalent rate that can exceed
    # the HBM peak; it is reported for recomputation, while `roofline` uses the bytes the kernels
    # actually have to move. Without stale edges every traversed edge matches (E_match = E_trav).
    per_wave = lambda x: x / args.steps
    e_match = e_trav if not cfg.get("stale_pct") else e_match_all
    b_formula = 28 * v_inv + 24 * e_trav + 4 * e_match + 4 * len(roots) * args.steps
    result["survey_formula"] = {
        "layout": "A", "V_exp": per_wave(v_inv), "E_trav": per_wave(e_trav), "E_match": per_wave(e_match),
        "R": len(roots), "bytes_per_wave": per_wave(b_formula),
        "push_equivalent_gbs": b_formula / elapsed / 1e9,
        "note": "push-equivalent: pull levels do not read these edges; see roofline for the bytes moved"}
    if m["pipelined"]:
        result["pipelined_ms_per_step"] = m["pipelined"]["ms_per_step"]
        result["pipelined"] = m["pipelined"]
    if e2e:
        result["e2e_ms_per_step"] = e2e["ms_per_step"]
        result["e2e"] = e2e

    # secondary workloads: configs[2] on this one GPU (N = 1), the weak-scaling point (N > 1)
    for key, name, scale in ([] if args.no_secondary else sel["secondary"]):
        g2, cfg2, n2, roots2, e2, b2 = build(name, scale)
        m2 = measure(g2, roots2)
        g2.close()
        result[key] = brief(m2, cfg2, n2, roots2, e2, b2)
        log(f"[rank {rank}] {key}: {result[key]['ms_per_step']:.4f} ms/step, {result[key]['value'] / 1e9:.2f} G nodes/s")

    if rank == 0 and world == 1 and not args.no_cpu and cfg["kind"] == "rmat":
        result["cpu_baseline"] = cpu_legs(args, cfg, roots, ids_host, st, value, result.get("configs2_single_gpu"))
    if rank == 0:
        json_out.write(json.dumps(result) + "\n")
        json_out.flush()
    if dist:
        dist.destroy_process_group()


def cpu_legs(args, cfg, roots, ids_host, st, value, c2):
    """The cpu_baseline object: the oracle on the identical configs[1] graph and roots at T = nproc
    (median of --cpu-runs after a warm-up) and at T = 1 (one wave: the closure of 4,096 roots is the
    giant component's, so fewer roots would not shorten it), and a labelled sample of configs[2]'s
    generator at --cpu-c2-scale beside the GPU's configs[2] figure."""
    info = host_cpu_info()
    threads = info["nproc"]
    cscale = args.cpu_scale or cfg["scale"]
    try:
        cpu, cbuild, cm, cr, same_roots, same_set = cpu_baseline(threads, cfg, cscale, roots, ids_host,
                                                                  args.cpu_runs, not args.no_cpu_single)
    except Exception as e:  # the CPU leg must not hide the GPU number
        return {"value": None, "error": repr(e)}
    best = cpu[threads]
    same = cscale == cfg["scale"]
    rec = {
        "value": best["v_inv"] / best["s"],
        "unit": "invalidated nodes/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"oracle (C++ restatement of the Computed.Invalidate cascade: per-node mutex, HashSetSlim3 "
                   f"usedBy, hash registry, RemoveUsedBy) on "
                   + (f"the identical {cfg['scale']}-scale graph and {cr}-root batch (BASELINE.json configs[1]: R-MAT "
                      f"scale {cscale}, {cm} edges; roots equal to the GPU's: {same_roots})" if same else
                      f"a labelled sample: R-MAT scale {cscale} ({cm} edges), {cr} roots")
                   + f", parallel over roots at T = nproc = {threads}; median of {len(best['runs'])} timed "
                     f"waves after a warm-up, each from a restored pristine copy; "
                     f"{best['v_inv']} nodes / {best['e_trav']} edges per wave"),
        "gteps": best["e_trav"] / best["s"] / 1e9,
        "wave_s": best["s"],
        "wave_s_runs": best["runs"],
        "single_thread_value": (cpu[1]["v_inv"] / cpu[1]["s"]) if 1 in cpu else None,
        "single_thread_wave_s": cpu[1]["s"] if 1 in cpu else None,
        "single_thread_sample": ("one wave at T = 1 on the same graph and roots, after the T = nproc waves"
                                 if 1 in cpu else None),
        "same_result_as_gpu": bool(same and same_set and best["v_inv"] == st.v_inv // args.steps
                                   and best["e_trav"] == st.e_trav // args.steps),
        "same_set_as_gpu": same_set,
        "host": info,
        "build_s": cbuild,
        "peak_rss_gb": peak_rss_gb(),
    }
    if same:
        rec["gpu_speedup"] = value / rec["value"]
        if 1 in cpu:
            rec["gpu_speedup_vs_single_thread"] = value / rec["single_thread_value"]
    log(f"cpu baseline: {cpu} (build {cbuild:.1f}s, host {info})")
    if c2 is not None and args.cpu_c2_scale:
        from stl_fusion_amd import workloads as W
        cfg2 = W.CONFIGS["rmat27"]
        try:
            cpu2, b2, m2, r2, _, _ = cpu_baseline(threads, cfg2, args.cpu_c2_scale, None, None, runs=2)
            v2 = cpu2[threads]["v_inv"] / cpu2[threads]["s"]
            rec["configs2_sample"] = {
                "value": v2, "unit": "invalidated nodes/s", "cores": threads,
                "sample": (f"labelled sample of configs[2]: its generator (edge factor 8, seed 0x5EED0027) at R-MAT "
                           f"scale {args.cpu_c2_scale} ({m2} edges, {r2} roots) instead of 27, T = {threads}, median of "
                           f"2 timed waves after a warm-up"),
                "v_inv_per_wave": cpu2[threads]["v_inv"], "wave_s": cpu2[threads]["s"], "build_s": b2,
                "gpu_configs2_value": c2["value"],
                "gpu_speedup": c2["value"] / v2,
                "note": "GPU: configs[2] itself (R-MAT 27) on one MI355X (configs2_single_gpu); CPU: the scale stated"}
            log(f"cpu configs[2] sample: {cpu2} (build {b2:.1f}s)")
        except Exception as e:
            rec["configs2_sample"] = {"value": None, "error": repr(e)}
    return rec


def n_gpus_visible() -> int:
    """GPUs this process can use (torch.cuda.device_count does not initialise the device)."""
    import torch
    return torch.cuda.device_count()


if __name__ == "__main__":
    try:
        main()
    except Exception as e:  # a failed rank exits non-zero with its rank and the failing call named
        log(f"[rank {os.environ.get('RANK', '0')} of {os.environ.get('WORLD_SIZE', '1')}] bench failed: "
            f"{type(e).__name__}: {e}")
        raise SystemExit(3)
    dump_maps()
