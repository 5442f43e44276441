"""GPU probe: one batched solve of the C5 workload; prints status/iteration stats, the
solver counters and the per-kernel HIP-event times.  usage: python tools/solve_probe.py [B] [N]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mpc_fatigue_amd import _lib, problems as PR  # noqa: E402
from mpc_fatigue_amd.ocp import OCP  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
N = int(sys.argv[2]) if len(sys.argv) > 2 else 100
dev = torch.device("cuda", 0)
spec = PR.pilz6_bench(N=N)
ocp = OCP(spec)
q0 = torch.tensor(PR.pilz6_batch_q0(B, seed=0), dtype=torch.float64, device=dev).contiguous()
pos = torch.empty((B, 3), dtype=torch.float64, device=dev)
_lib.check(_lib.lib().mf_fk_dev(ocp.model.handle, ocp.model.frame_id(spec["frame"]), q0.data_ptr(), pos.data_ptr(),
                                None, B, 0))
lref = pos[:, :2].contiguous()
out = {"w": torch.empty((B, ocp.wsize), dtype=torch.float64, device=dev),
       "status": torch.empty(B, dtype=torch.int32, device=dev), "iters": torch.empty(B, dtype=torch.int32, device=dev),
       "kkt": torch.empty(B, dtype=torch.float64, device=dev), "obj": torch.empty(B, dtype=torch.float64, device=dev)}
ptrs = {k: v.data_ptr() for k, v in out.items()}
opts = dict(tol=1e-8, constr_viol_tol=1e-8, max_iter=300, mu_init=0.1, F_init=PR.BENCH_F_INIT)
for rep in range(2):
    ocp.timing(rep == 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ocp.solve_dev(q0.data_ptr(), lref.data_ptr(), B, ptrs, **opts)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    st = out["status"].cpu().numpy()
    it = out["iters"].cpu().numpy()
    print(f"rep {rep}: {1e3 * (t1 - t0):.1f} ms  -> {B / (t1 - t0):.0f} horizons/s  status counts "
          f"{np.bincount(st + 1).tolist()} iters mean {it.mean():.1f} max {it.max()}", flush=True)
stats = ocp.kernel_stats()
tot = sum(v[0] for v in stats.values())
for k, (ms, n) in stats.items():
    print(f"  {k:12s} {ms:9.2f} ms {n:5d} launches  {ms / max(n, 1) * 1e3:9.1f} us/launch  {100 * ms / tot:5.1f}%")
if hasattr(ocp, "counters"):
  c = ocp.counters(B)
  print("counters per problem (mean): inertia corrections", c["n_ic"].mean(), "Riccati sweeps", c["n_try"].mean(),
      "| ls fails", c["n_ls_fail"].sum(), "ls trials past round 0",
      c["n_lsfb"].mean())
if os.environ.get("MF_LIB", "").endswith("_stamps.so"):
    import ctypes as C
    nb = (B + 63) // 64
    buf = (C.c_ulonglong * (8 * nb))()
    _lib.lib().mf_debug_stamps(buf, nb, 1)
    a = np.array(buf[:], dtype=np.float64).reshape(nb, 8)
    names = ["regularise+fence", "stage waits", "stage compute", "forward sweep", "", "", "", "try bookkeeping"]
    tot = a.sum(1).mean()
    print("k_riccati stamps (mean per wave over both reps, s_memtime ticks):")
    for i, nm in enumerate(names):
        if nm:
            print(f"  {nm:18s} {a[:, i].mean():14.0f}  {100 * a[:, i].mean() / tot:5.1f}%")
