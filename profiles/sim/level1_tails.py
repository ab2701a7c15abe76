import sys, numpy as np, time
sys.path.insert(0, '/root/repo/oracle'); sys.path.insert(0, '/root/repo/stl.fusion_amd')
import fgo, workloads as W
scale, ef, seed = 24, 16, 0x5EED0024
s, d = fgo.gen_rmat(scale, ef, seed)
N = 1 << scale
outdeg = np.bincount(s, minlength=N)
indeg = np.bincount(d, minlength=N).astype(np.int64)
roots = W.pick_roots(4096, N, 0x5EED1024, outdeg)
# CSR by src (push)
o = np.argsort(s, kind='stable'); ds = d[o]; soff = np.concatenate([[0], np.cumsum(outdeg)])
# dependency lists by dst, weight-ordered (weight = indeg of parent, desc; ties by src asc)
w = indeg[s]
key = (d.astype(np.int64) << 32) | (0xFFFFFFFF - w)
o2 = np.lexsort((s, key)); ls = s[o2]
loff = np.concatenate([[0], np.cumsum(indeg)])
inv = np.zeros(N, bool); inv[roots] = True
# L0 push: children of roots
ch = np.concatenate([ds[soff[r]:soff[r+1]] for r in roots])
vis = np.zeros(N, bool); vis[roots] = True
win0 = np.unique(ch[~vis[ch]])
inv[win0] = True; vis[win0] = True
print("L0 winners", len(win0), "edges", len(ch), flush=True)
# L1 pull: candidates = indeg>0 and not visited
cand = np.nonzero((indeg > 0) & ~vis)[0]
print("L1 live candidates", len(cand))
# position of first invalidated parent in each list
invl = inv[ls]                       # per list entry
# first hit index per candidate: use cumulative trick
pos = np.full(N, -1, np.int64)
idx = np.nonzero(invl)[0]
dd = np.searchsorted(loff, idx, side='right') - 1
# first occurrence per dst
first = np.full(N, np.iinfo(np.int64).max); np.minimum.at(first, dd, idx - loff[dd])
fh = first[cand]; L = indeg[cand]
hit = fh < L
head = hit & (fh < 2)
tail = ~head & (L > 2)
exam = np.where(hit, fh + 1, L)        # entries examined
print("head hits", head.sum(), "tail queued", tail.sum(), "tail hits", (tail & hit).sum())
te = exam[tail]
print("tail examined: mean %.1f  p99 %d  max %d  sum %d" % (te.mean(), np.percentile(te, 99), te.max(), te.sum()))
# per block (13 tiles x 1024 slots)
blk = cand[tail] // (13 * 1024)
per = np.bincount(blk, weights=np.minimum(te, 10**9), minlength=N // (13*1024) + 1)
steps = np.bincount(blk, weights=np.ceil(np.maximum(te - 4, 0) / 8), minlength=len(per))
print("per-block tail entries: median %.0f  max %.0f; pass-2 steps: median %.0f max %.0f" % (np.median(per), per.max(), np.median(steps), steps.max()))
big = np.argsort(te)[-10:]
print("longest tail scans (examined, list len, hit):", list(zip(te[big], L[tail][big], hit[tail][big])))
