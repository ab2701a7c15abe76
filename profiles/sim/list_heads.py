import sys, numpy as np, time
sys.path.insert(0, '/root/repo/oracle')
import fgo
scale, ef, seed = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3], 16)
t=time.time()
s, d = fgo.gen_rmat(scale, ef, seed)
N = 1 << scale
print("edges", len(s), time.time()-t, flush=True)
indeg = np.bincount(d, minlength=N).astype(np.int64)   # uin_len (weight)
# order edges by (d, weight desc, pool order ~ s asc)
w = indeg[s]
key = (d.astype(np.int64) << 32) | (0xFFFFFFFF - w)
o = np.lexsort((s, key))   # stable by s within ties
s_sorted = s[o]; d_sorted = d[o]
start = np.searchsorted(d_sorted, np.arange(N))
has = indeg > 0
h0 = np.full(N, -1, np.int64); h1 = np.full(N, -1, np.int64)
h0[has] = s_sorted[start[has]]
has2 = indeg > 1
h1[has2] = s_sorted[start[has2] + 1]
heads = np.concatenate([h0[h0 >= 0], h1[h1 >= 0]])
cnt = np.bincount(heads, minlength=N)
nd = (cnt > 0).sum()
print(f"candidates {has.sum()}  distinct heads {nd} ({nd/N:.3f} of N)  -> head bitmap {nd/8/1024:.0f} KB vs {N/8/1024:.0f} KB")
cs = np.sort(cnt)[::-1]
tot = cs.sum()
for k in [65536, 262144, 1<<20, 2<<20, 4<<20]:
    print(f"  top {k}: {cs[:k].sum()/tot:.3f} of head probes")
