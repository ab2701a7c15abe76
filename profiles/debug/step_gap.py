"""Where the ~20 us between a wave's kernels and the next step go (configs[1]): per-step Python wall,
the C call's own wall (WaveStats.total_ms), the wave's kernels (kernel_ms), restore alone, and an
empty wave (no roots). FGI_DIAG_SPIN=<flags> calls hipSetDeviceFlags before the device is touched."""
import ctypes, os, sys, time
sys.path.insert(0, os.getcwd())
if os.environ.get("FGI_DIAG_SPIN"):
    hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
    print("hipSetDeviceFlags ->", hip.hipSetDeviceFlags(ctypes.c_uint(int(os.environ["FGI_DIAG_SPIN"]))), flush=True)
import numpy as np
import torch
import _pkg
pkg = _pkg.load()
from stl_fusion_amd import workloads as W
cfg = dict(W.CONFIGS["rmat24"])
g = pkg.Graph(W.n_slots(cfg), device=0)
W.build(g, cfg)
roots = W.roots_for(g, cfg)
d_roots = torch.from_numpy(roots.astype(np.int32)).to("cuda:0")
g.snapshot()
g.set_option(pkg.fgi.OPT_LEVEL_TIMING, 0)
K = 200
def run(nr, stats, rest=True):
    for _ in range(10):
        g.restore(); g.invalidate_dev(nr, d_roots.data_ptr(), 0, pkg.WaveStats())
    torch.cuda.synchronize()
    st = pkg.WaveStats() if stats else None
    t = time.perf_counter()
    for _ in range(K):
        if rest: g.restore()
        g.invalidate_dev(nr, d_roots.data_ptr(), 0, st)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / K * 1e3
    if st is None:
        return f"step {ms:.4f} ms"
    return f"step {ms:.4f} ms  call {st.total_ms / K:.4f}  kernels {st.kernel_ms / K:.4f}"
for rep in range(2):
    print("full, stats   :", run(len(roots), True), flush=True)
    print("full, nostats :", run(len(roots), False), flush=True)
    print("full, norestore:", run(len(roots), True, False), flush=True)
    print("empty, stats  :", run(0, True), flush=True)
    print("1 root, stats :", run(1, True), flush=True)
t = time.perf_counter()
for _ in range(K): g.restore()
torch.cuda.synchronize()
print(f"restore alone {(time.perf_counter() - t) / K * 1e3:.4f} ms")
g.close()
