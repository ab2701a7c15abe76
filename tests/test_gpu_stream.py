"""GPU parity of the streaming mix (BASELINE.json configs[4], workloads.StreamMix): recompute
(begin_compute -> add_used -> set_output), delay timers firing with immediately = true, and hub
waves, on the engine and the oracle round by round — the same schedule bench_configs.py times at
10k hubs x 1,000 leaves."""
import numpy as np
import pytest

import _pkg
import fgo as O
from harness import assert_states_equal, build_pair, canon_edges, oracle_edges

pytestmark = pytest.mark.gpu


def _mix(pkg, hubs, leaves, k, delay_pct, seed):
    from stl_fusion_amd import workloads as W
    return W.StreamMix(hubs, leaves, k, delay_pct, seed)


def _oracle_round(o, mix, timers, hubs, leaves, versions_h, versions_l):
    o.clear_log()
    if len(timers):
        o.invalidate_slots(timers, np.ones(len(timers), np.uint8))
    t_ids = o.inv_log()
    for s, v in zip(hubs, versions_h):
        o.begin_compute(int(s), int(v), False)
    for s in hubs:
        o.set_output(o.last(int(s)))
    for s, v in zip(leaves, versions_l):
        o.begin_compute(int(s), int(v), bool(mix.has_delay[s]))
    for s, h in zip(leaves, mix.hub_of(leaves)):
        o.add_used(o.last(int(s)), o.last(int(h)))
    for s in leaves:
        o.set_output(o.last(int(s)))
    return t_ids


@pytest.mark.parametrize("hubs,leaves,k,delay_pct", [(40, 30, 4, 10), (64, 200, 8, 5), (7, 1, 7, 50)])
def test_stream_mix_rounds_match_oracle(pkg, gpu_available, hubs, leaves, k, delay_pct):
    mix = _mix(pkg, hubs, leaves, k, delay_pct, 0x5EED00E0)
    n = mix.n
    used, dep, tag = mix.initial_edges()
    g, o = build_pair(pkg, n, mix.version.copy(), mix.state_flags(), used, dep, tag)
    prev = np.zeros(0, np.uint32)
    for r in range(8):
        timers, hs, ls = mix.plan(prev)
        vh = mix.new_versions(hs).copy()
        vl = mix.new_versions(ls).copy()
        t_oracle = _oracle_round(o, mix, timers, hs, ls, vh, vl)
        if len(timers):
            t_ids = g.invalidate(timers, np.ones(len(timers), np.uint8))
            assert np.array_equal(np.sort(t_ids), np.sort(t_oracle))
        g.begin_compute(hs, vh)
        g.set_output(hs)
        g.begin_compute(ls, vl, mix.has_delay[ls])
        res = g.add_used(ls, mix.hub_of(ls))
        assert np.all(res == _pkg.load().fgi.USED_ADDED)
        oset, _ = g.set_output(ls)
        assert np.all(oset == 1)
        assert_states_equal(g, o, n)
        roots = mix.roots(r)
        o.clear_log()
        o.invalidate_slots(roots)
        ids = g.invalidate(roots)
        assert np.array_equal(np.sort(ids), np.sort(o.inv_log())), f"round {r}"
        # the wave is the root hubs plus their undelayed leaves
        ch = mix.children(roots)
        expect = np.concatenate([roots, ch[mix.has_delay[ch] == 0]])
        assert np.array_equal(np.sort(ids), np.sort(expect))
        assert_states_equal(g, o, n)
        prev = roots
    g.prune()
    o.prune()
    u, d, t = g.export_edges()
    ge = canon_edges(u, d, t)
    ge = ge[ge[:, 0] < n] if len(ge) else ge
    assert np.array_equal(ge, oracle_edges(o, n))
