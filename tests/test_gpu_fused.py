"""Fused waves (FGI_OPT_FUSED): the roots and the small push levels run inside two
persistent launches (head / tail, software grid barriers) and only the pull levels — and push
levels larger than one round of the fused grid — as k_level launches, whose level the device picks.
Every variant must give the oracle's wave bit-exactly (set, V_inv, E_trav, every node word), on
push-only, pull-only and automatic directions:

  0            the level groups (no fusion)
  1            fused, mid launches predicted from the previous wave
  1 | 2        no prediction: every k_level level is found by an extra round (host loop)
  1 | 4        every push level as a k_level launch (the mid push path, collects after pulls)
  1 | 8        every push level inside the fused grid, however large
  1 | 2 | 4    both

Graphs: R-MAT with 0% / 50% stale edges (pull levels, a push after pulls), the layered compute-method
graph of configs[0] (push after pull at every level), and a mixed-state graph (Computing, delays,
Invalidated and empty slots, immediately roots).
"""
import numpy as np
import pytest

import fgo as O
from harness import assert_states_equal, build_pair, random_states
from test_gpu_parity import _edges_from_live

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("variants")]

MODES = [0, 1, 1 | 2, 1 | 4, 1 | 8, 1 | 2 | 4]


def _oracle_for_rmat(scale, ef, seed, stale, roots_seed, n_roots):
    n = 1 << scale
    s, d = O.gen_rmat(scale, ef, seed)
    tags = O.gen_tags(s, d, seed, stale, 0x5EED00C0)
    o = O.Oracle(n)
    o.load_graph(O.version_of(seed, np.arange(n)), None, s, d, tags)
    roots = O.gen_roots(n_roots, n, roots_seed, np.bincount(s, minlength=n))
    st = o.invalidate_slots(roots)
    want = np.sort(o.inv_log())
    ov, of = o.dump_states()
    o.close()
    return roots, want, st, ov, of


@pytest.mark.parametrize("stale", [0, 50])
def test_fused_modes_rmat(pkg, gpu_available, stale):
    scale, ef, seed = 18, 16, 0x5EED0024
    n = 1 << scale
    roots, want, st, ov, of = _oracle_for_rmat(scale, ef, seed, stale, 0x5EED1024, 1024)
    g = pkg.Graph(n)
    g.synth_rmat(scale, ef, seed, stale, 0x5EED00C0)
    g.snapshot()
    g.invalidate(roots)   # the first wave builds the pull lists
    for direction in (0, 1, 2):
        g.set_option(pkg.fgi.OPT_DIRECTION, direction)
        for mode in MODES:
            g.set_option(pkg.fgi.OPT_FUSED, mode)
            for rep in range(2):   # the second wave runs on the first one's prediction
                g.restore()
                ws = pkg.WaveStats()
                ids = g.invalidate(roots, stats=ws)
                key = (direction, mode, rep)
                assert len(np.unique(ids)) == len(ids), key
                assert np.array_equal(np.sort(ids), want), (key, len(ids), len(want))
                assert (ws.v_inv, ws.e_trav) == (st.v_inv, st.e_trav), (key, ws.v_inv, st.v_inv, ws.e_trav, st.e_trav)
                if direction == 2:
                    assert ws.pull_levels == ws.levels, key
                if mode & 1:
                    assert ws.fused_launches >= 2, key
                    if mode == 1 and rep == 1:
                        assert ws.host_syncs == 1, (key, ws.host_syncs)
                else:
                    # level groups: fused_launches counts the wave tail's persistent launches (k_wave_tail,
                    # at most one per group), never more than the host synchronisations
                    assert ws.fused_launches <= ws.host_syncs, key
                v, f = g.dump_states()
                assert np.array_equal(v[:n], ov) and np.array_equal(f[:n], of), key
    g.close()


def test_fused_modes_layered(pkg, gpu_available):
    levels, width, fanout, seed = 7, 20_000, 8, 0x5EED0001
    n = levels * width
    s, d = O.gen_layered(levels, width, fanout, seed)
    o = O.Oracle(n)
    o.load_graph(O.version_of(seed, np.arange(n)), None, s, d, O.gen_tags(s, d, seed))
    roots = O.gen_roots(300, width, 0x5EED1001, np.bincount(s, minlength=n)[:width])
    st = o.invalidate_slots(roots)
    want = np.sort(o.inv_log())
    ov, of = o.dump_states()
    o.close()
    g = pkg.Graph(n)
    g.synth_layered(levels, width, fanout, seed)
    g.snapshot()
    g.invalidate(roots)
    for direction in (0, 1, 2):
        g.set_option(pkg.fgi.OPT_DIRECTION, direction)
        for mode in MODES:
            g.set_option(pkg.fgi.OPT_FUSED, mode)
            g.restore()
            ws = pkg.WaveStats()
            ids = g.invalidate(roots, stats=ws)
            key = (direction, mode)
            assert np.array_equal(np.sort(ids), want), key
            assert (ws.v_inv, ws.e_trav) == (st.v_inv, st.e_trav), key
            v, f = g.dump_states()
            assert np.array_equal(v[:n], ov) and np.array_equal(f[:n], of), key
    g.close()


@pytest.mark.parametrize("mode", MODES)
def test_fused_modes_mixed_states(pkg, gpu_available, mode):
    """Computing nodes (InvalidateOnSetOutput), delays (DelayStarted), Invalidated and empty slots,
    stale edges and immediately roots: three waves on the same graph, each against the oracle."""
    rng = np.random.default_rng(7 + mode)
    n = 60_000
    versions, flags = random_states(n, rng)
    src, dst, tags = _edges_from_live(versions, flags, rng, 600_000, n, stale_p=0.3)
    g, o = build_pair(pkg, n, versions, flags, src, dst, tags)
    g.set_option(pkg.fgi.OPT_FUSED, mode)
    for w in range(3):
        g.set_option(pkg.fgi.OPT_DIRECTION, (1, 2, 0)[w])   # push only, pull only (builds the lists), auto
        roots = rng.choice(n, 400, replace=False).astype(np.uint32)
        imm = (rng.random(400) < 0.2).astype(np.uint8) if w == 1 else None
        o.clear_log()
        ost = o.invalidate_slots(roots, imm)
        ws = pkg.WaveStats()
        ids = g.invalidate(roots, imm, stats=ws)
        assert np.array_equal(np.sort(ids), np.sort(o.inv_log())), (mode, w)
        assert ws.v_inv == ost.v_inv, (mode, w)
        if w == 0:   # E_trav is exact on a graph's first wave (fgi.h: later ones count lazily removed entries)
            assert ws.e_trav == ost.e_trav, (mode, w)
        assert_states_equal(g, o, n)
    g.close()
    o.close()


def test_fused_bits_output_matches_ids(pkg, gpu_available):
    """fgi_invalidate_bits on a fused wave: the bitmap holds exactly the id list's handles."""
    scale, ef, seed = 17, 16, 0x5EED0024
    n = 1 << scale
    g = pkg.Graph(n)
    g.synth_rmat(scale, ef, seed, 0, 0)
    deg, _ = g.degrees()
    roots = O.gen_roots(512, n, 0x5EED1024, deg[:n])
    g.snapshot()
    g.invalidate(roots)
    g.restore()
    ids = np.sort(g.invalidate(roots))
    g.restore()
    bits, n_inv = g.invalidate_bits(roots)
    got = np.nonzero(np.unpackbits(bits.view(np.uint8), bitorder="little"))[0]
    assert n_inv == len(ids) and np.array_equal(got, ids)
    g.close()
