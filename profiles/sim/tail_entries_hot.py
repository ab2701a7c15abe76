import sys, numpy as np
sys.path.insert(0, '/root/repo/oracle'); sys.path.insert(0, '/root/repo/stl.fusion_amd')
import fgo, workloads as W
scale, ef, seed, rseed = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3], 16), int(sys.argv[4], 16)
s, d = fgo.gen_rmat(scale, ef, seed)
N = 1 << scale
outdeg = np.bincount(s, minlength=N); indeg = np.bincount(d, minlength=N).astype(np.int64)
roots = W.pick_roots(4096, N, rseed, outdeg)
o = np.argsort(s, kind='stable'); ds = d[o]; del o
soff = np.concatenate([[0], np.cumsum(outdeg)])
w = indeg[s]; key = (d.astype(np.int64) << 32) | (0xFFFFFFFF - w); del w
o2 = np.lexsort((s, key)); del key
ls = s[o2]; del o2
loff = np.concatenate([[0], np.cumsum(indeg)])
has = indeg > 0; has2 = indeg > 1
h0 = np.full(N, -1); h1 = np.full(N, -1); h0[has] = ls[loff[:-1][has]]; h1[has2] = ls[loff[:-1][has2] + 1]
cnt = np.bincount(np.concatenate([h0[h0 >= 0], h1[h1 >= 0]]), minlength=N)
order = np.argsort(-cnt, kind='stable'); rank = np.empty(N, np.int64); rank[order] = np.arange(N)
vis = np.zeros(N, bool); inv = np.zeros(N, bool); vis[roots] = True; inv[roots] = True
ch = np.concatenate([ds[soff[r]:soff[r+1]] for r in roots]); win = np.unique(ch[~vis[ch]]); vis[win] = True; inv[win] = True
cand = np.nonzero(has & ~vis)[0]
hit = inv[h0[cand]] | ((h1[cand] >= 0) & inv[np.maximum(h1[cand], 0)])
q = cand[~hit & (indeg[cand] > 2)]
# entries 2 .. of queued lists (up to first hit): which are hot (rank < K)?
starts = loff[q] + 2; lens = indeg[q] - 2
idx = np.repeat(starts, lens) + (np.arange(lens.sum()) - np.repeat(np.cumsum(lens) - lens, lens))
ent = ls[idx]
for K in [65536, 262144, 1 << 20]:
    print(f"scale {scale}: queued {len(q)}, tail entries {len(ent)}; hot (rank < {K}): {(rank[ent] < K).mean():.3f}")
