"""Program profiled by tools/pmc_traffic.sh: one calibration copy of a known byte count
(elementwise torch copy, 512 MiB read + 512 MiB written) and one batched solve of the bench
workload (C5, 8192 horizons by default).  usage: python tools/traffic_run.py [B [NODES_JSON]]
NODES_JSON receives the solve's node-evaluation count (the per-node normaliser of the PMC totals)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mpc_fatigue_amd import _lib, problems as PR  # noqa: E402
from mpc_fatigue_amd.ocp import OCP  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
dev = torch.device("cuda", 0)
x = torch.rand(64 * 1024 * 1024, dtype=torch.float64, device=dev)  # 512 MiB
y = torch.empty_like(x)
y.copy_(x)
torch.cuda.synchronize()
del x, y
spec = PR.pilz6_bench(N=100)
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
ocp.solve_dev(q0.data_ptr(), lref.data_ptr(), B, ptrs, tol=1e-8, constr_viol_tol=1e-8, max_iter=300, mu_init=0.1,
              F_init=PR.BENCH_F_INIT)
torch.cuda.synchronize()
it = out["iters"].cpu()
print("solve done: iterations mean", float(it.double().mean()), "node evaluations", int(((it + 1) * 100).sum()))
if len(sys.argv) > 2:
    json.dump({"node_evals": int(((it + 1) * 100).sum()), "batch": B}, open(sys.argv[2], "w"))
