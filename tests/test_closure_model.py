"""CPU check of the independent closure checker (tests/closure_check.py) that test_gpu_scale.py and
test_gpu_configs.py use on the full-size configs[1] / [2] / [3] waves: on smaller R-MAT graphs (with
stale edges) its least closure must be the oracle's set, the oracle's own wave must pass every check,
and a wave with a node missing or added must fail them."""
import numpy as np
import pytest

import fgo as O
from closure_check import DeviceEdges


@pytest.mark.parametrize("scale,stale", [(12, 0), (14, 30)])
def test_closure_bfs_matches_oracle(fgo, scale, stale):
    seed = 0x5EED0024
    n = 1 << scale
    s, d = O.gen_rmat(scale, 16, seed)
    t = O.gen_tags(s, d, seed, stale, 0x5EED00C0)
    o = O.Oracle(n)
    ver = O.version_of(seed, np.arange(n))
    o.load_graph(ver, None, s, d, t)
    roots = O.gen_roots(64, n, 0x5EED1024, np.bincount(s, minlength=n))
    st = o.invalidate_slots(roots)
    ids = np.sort(o.inv_log())
    want = np.zeros(n, bool)
    want[ids] = True
    e = DeviceEdges(n, s, d, t, ver, device="cpu")
    got = e.least_closure(roots).numpy()
    assert np.array_equal(got, want)
    assert e.check_wave(ids, roots, st.e_trav) == len(ids)
    # a node short (a non-root) or a node too many must be caught
    extra = np.setdiff1d(np.arange(n), ids)[:1]
    non_root = np.setdiff1d(ids, roots)
    for bad in (np.setdiff1d(ids, non_root[-1:]), np.sort(np.concatenate([ids, extra]))):
        with pytest.raises(AssertionError):
            e.check_wave(bad, roots, st.e_trav)


def test_parallel_oracle_import_is_thread_count_independent(fgo):
    """fgo_set_threads only splits the bulk work: the generator output and the imported graph are
    the same for any thread count."""
    seed = 0x5EED0024
    outs = []
    for th in (1, 4):
        O.set_threads(th)
        s, d = O.gen_rmat(13, 16, seed)
        t = O.gen_tags(s, d, seed, 50, 7)
        o = O.Oracle(1 << 13)
        o.load_graph(O.version_of(seed, np.arange(1 << 13)), None, s, d, t)
        o.snapshot()
        st = o.invalidate_slots(O.gen_roots(32, 1 << 13, 3, np.bincount(s, minlength=1 << 13)), threads=th)
        outs.append((s.tobytes(), d.tobytes(), t.tobytes(), o.total_used_by(), st.v_inv, st.e_trav,
                     np.sort(o.inv_log()).tobytes()))
        o.restore()
        assert o.total_used_by() == len(s)
    O.set_threads(1)
    assert outs[0] == outs[1]
