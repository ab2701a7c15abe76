"""Independent checks of a whole wave at the benchmarked sizes (test infrastructure).

A wave's result is fully determined by the graph: the invalidated set is the least set that holds
the roots and is closed under version-matching `_usedBy` entries (Computed.cs:212-216 recurses
into exactly those), when every node is Consistent without delay (R-MAT workloads). These helpers
compute that set with torch's own gather / scatter kernels over the engine's exported edge set —
no engine kernel is involved — and check a wave's output against it:

  least closure — the fixpoint of seen |= {d : (u, d, t) with seen[u] and t == version(d)}
  closure       — every matching entry of an invalidated node reaches an invalidated node
  witness       — every invalidated non-root has an invalidated parent with a matching entry
  E_trav        — the sum of |_usedBy| over the invalidated nodes (the TEPS numerator)

Edges are moved to the device in chunks; at R-MAT 27 (1.07 G edges) the arrays take ~17 GB of HBM.
"""
import numpy as np

CHUNK = 1 << 27


class DeviceEdges:
    """The exported edge set (u, d, t) plus version(d) == t, resident on a torch device."""

    def __init__(self, n, u, d, t, ver, device="cuda"):
        import torch
        self.torch = torch
        self.n, self.m, self.dev = n, len(u), device
        assert n < (1 << 31)
        ver_g = torch.from_numpy(np.ascontiguousarray(ver).view(np.int64)).to(device)
        self.u, self.d, self.live = [], [], []
        self.deg = torch.zeros(n, dtype=torch.int64, device=device)
        for a in range(0, self.m, CHUNK):
            b = min(self.m, a + CHUNK)
            uc = torch.from_numpy(np.ascontiguousarray(u[a:b]).view(np.int32)).to(device)
            dc = torch.from_numpy(np.ascontiguousarray(d[a:b]).view(np.int32)).to(device)
            tc = torch.from_numpy(np.ascontiguousarray(t[a:b]).view(np.int64)).to(device)
            self.live.append(tc == ver_g[dc.long()])
            self.deg += torch.bincount(uc.long(), minlength=n)
            self.u.append(uc)
            self.d.append(dc)
            del tc
        del ver_g

    def least_closure(self, roots):
        torch = self.torch
        seen = torch.zeros(self.n, dtype=torch.bool, device=self.dev)
        seen[torch.from_numpy(np.asarray(roots, np.int64)).to(self.dev)] = True
        while True:
            nxt = seen.clone()
            for uc, dc, lc in zip(self.u, self.d, self.live):
                m = lc & seen[uc.long()]
                nxt[dc[m].long()] = True
            if torch.equal(nxt, seen):
                return seen
            seen = nxt

    def check_wave(self, ids, roots, e_trav):
        """Asserts the wave's invalidated ids are exactly the least closure of the roots; returns
        the set size."""
        torch = self.torch
        inv = torch.zeros(self.n, dtype=torch.bool, device=self.dev)
        ids_g = torch.from_numpy(np.asarray(ids, np.int64)).to(self.dev)
        inv[ids_g] = True
        assert int(inv.sum()) == len(ids), "a node was listed twice"
        is_root = torch.zeros(self.n, dtype=torch.bool, device=self.dev)
        is_root[torch.from_numpy(np.asarray(roots, np.int64)).to(self.dev)] = True
        assert bool(inv[is_root].all()), "a root (Consistent, no delay) was not invalidated"
        has_parent = torch.zeros(self.n, dtype=torch.bool, device=self.dev)
        for uc, dc, lc in zip(self.u, self.d, self.live):
            m = lc & inv[uc.long()]
            reached = dc[m].long()
            assert bool(inv[reached].all()), "an invalidated node has a matching dependant the wave did not invalidate"
            has_parent[reached] = True
        assert not bool((inv & ~is_root & ~has_parent).any()), "an invalidated node has no invalidated parent"
        assert int(self.deg[inv].sum()) == e_trav, "E_trav differs from the sum of the invalidated rows"
        want = self.least_closure(roots)
        assert torch.equal(want, inv), (int(want.sum()), int(inv.sum()))
        return len(ids)
