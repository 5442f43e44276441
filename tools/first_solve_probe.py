"""Probe: does the first solve on a fresh workspace differ from later ones?  (bench batch, dev path)"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpc_fatigue_amd import _lib, problems as PR  # noqa: E402
from mpc_fatigue_amd.ocp import OCP  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
dev = torch.device("cuda", 0)
spec = PR.pilz6_bench(N=100)
opts = dict(tol=1e-8, constr_viol_tol=1e-8, max_iter=300, mu_init=0.1, F_init=PR.BENCH_F_INIT)
Q0 = PR.pilz6_batch_q0(B, seed=0)
for stream_kind in ("own", "default"):
    ocp = OCP(spec)
    q0 = torch.tensor(Q0, dtype=torch.float64, device=dev)
    pos = torch.empty((B, 3), dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev) if stream_kind == "default" else torch.cuda.Stream(dev)
    _lib.check(_lib.lib().mf_fk_dev(ocp.model.handle, ocp.model.frame_id(spec["frame"]), q0.data_ptr(), pos.data_ptr(),
                                    None, B, torch.cuda.current_stream(dev).cuda_stream))
    lref = pos[:, :2].contiguous()
    out = {"w": torch.empty((B, ocp.wsize), dtype=torch.float64, device=dev),
           "status": torch.empty(B, dtype=torch.int32, device=dev), "iters": torch.empty(B, dtype=torch.int32, device=dev),
           "kkt": torch.empty(B, dtype=torch.float64, device=dev), "obj": torch.empty(B, dtype=torch.float64, device=dev)}
    torch.cuda.synchronize(dev)
    for rep in range(2):
        t = time.perf_counter()
        ocp.solve_dev(q0.data_ptr(), lref.data_ptr(), B, {k: v.data_ptr() for k, v in out.items()},
                      stream=st.cuda_stream, **opts)
        torch.cuda.synchronize(dev)
        s = out["status"].cpu().numpy()
        it = out["iters"].cpu().numpy()
        print(f"stream {stream_kind} solve {rep}: {time.perf_counter() - t:.2f}s conv {(s == 0).sum()} "
              f"status {np.bincount(s, minlength=4).tolist()} mean it {it.mean():.2f} max {it.max()}", flush=True)
    del ocp
