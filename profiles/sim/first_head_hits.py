import sys, numpy as np, time
sys.path.insert(0, '/root/repo/oracle'); sys.path.insert(0, '/root/repo/stl.fusion_amd')
import fgo, workloads as W
scale, ef, seed = 24, 16, 0x5EED0024
s, d = fgo.gen_rmat(scale, ef, seed)
N = 1 << scale
outdeg = np.bincount(s, minlength=N); indeg = np.bincount(d, minlength=N).astype(np.int64)
roots = W.pick_roots(4096, N, 0x5EED1024, outdeg)
o = np.argsort(s, kind='stable'); ds = d[o]; soff = np.concatenate([[0], np.cumsum(outdeg)])
w = indeg[s]; key = (d.astype(np.int64) << 32) | (0xFFFFFFFF - w)
o2 = np.lexsort((s, key)); ls = s[o2]; loff = np.concatenate([[0], np.cumsum(indeg)])
has = indeg > 0; has2 = indeg > 1
h0 = np.full(N, -1); h1 = np.full(N, -1); h0[has] = ls[loff[:-1][has]]; h1[has2] = ls[loff[:-1][has2] + 1]
cnt = np.bincount(np.concatenate([h0[h0 >= 0], h1[h1 >= 0]]), minlength=N)
order = np.argsort(-cnt, kind='stable'); rank = np.empty(N, np.int64); rank[order] = np.arange(N)
vis = np.zeros(N, bool); inv = np.zeros(N, bool); vis[roots] = True; inv[roots] = True
ch = np.concatenate([ds[soff[r]:soff[r+1]] for r in roots]); win = np.unique(ch[~vis[ch]]); vis[win] = True; inv[win] = True
cand = np.nonzero(has & ~vis)[0]
a0 = h0[cand]; a1 = h1[cand]
hit0 = inv[a0]; hit1 = (a1 >= 0) & inv[np.maximum(a1, 0)]
print(f"L1 live {len(cand)}: head0 hits {hit0.mean():.3f}, head1-only hits {(hit1 & ~hit0).mean():.3f}, has head1 {(a1>=0).mean():.3f}")
for K in [65536, 262144]:
    print(f"  K={K}: head0 hot {(rank[a0] < K).mean():.3f}; head1 hot (of present) {(rank[a1[a1>=0]] < K).mean():.3f}; "
          f"head1 needed (head0 missed, present) {((~hit0) & (a1>=0)).mean():.3f} of which hot {(rank[a1[(~hit0)&(a1>=0)]] < K).mean():.3f}")
