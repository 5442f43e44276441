"""Program profiled by tools/pmc_traffic_ipopt.sh: one calibration copy of a known byte count (elementwise torch copy,
512 MiB read + 512 MiB written) and the headline solve -- C2 as the reference solves it (IPOPT mode from x0 = 0,
csrc/gipm.hip chain family) on the C5 batch -- capped at ITERS iterations, so that every launch profiled is a
full-batch launch.  usage: python tools/traffic_run_ipopt.py [B [ITERS [NODES_JSON]]]
NODES_JSON receives the device-counted node evaluations of the solve (the per-node normaliser of the PMC totals)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mpc_fatigue_amd import _lib, problems as PR  # noqa: E402
from mpc_fatigue_amd.gocp import GOCP  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
ITERS = int(sys.argv[2]) if len(sys.argv) > 2 else 30
dev = torch.device("cuda", 0)
x = torch.rand(64 * 1024 * 1024, dtype=torch.float64, device=dev)  # 512 MiB
y = torch.empty_like(x)
y.copy_(x)
torch.cuda.synchronize()
del x, y
spec = PR.pilz6_bench(N=100)
g = GOCP(spec)
q0 = torch.tensor(PR.pilz6_batch_q0(B, seed=0), dtype=torch.float64, device=dev).contiguous()
pos = torch.empty((B, 3), dtype=torch.float64, device=dev)
m = g.models[0]
_lib.check(_lib.lib().mf_fk_dev(m.handle, m.frame_id(spec["frame"]), q0.data_ptr(), pos.data_ptr(), None, B, 0))
lref = pos[:, :2].contiguous()
out = {"w": torch.empty((B, g.wsize), dtype=torch.float64, device=dev),
       "status": torch.empty(B, dtype=torch.int32, device=dev), "iters": torch.empty(B, dtype=torch.int32, device=dev),
       "kkt": torch.empty(B, dtype=torch.float64, device=dev), "obj": torch.empty(B, dtype=torch.float64, device=dev)}
ptrs = {k: v.data_ptr() for k, v in out.items()}
g.timing(True)
g.solve_dev(q0.data_ptr(), None, None, lref.data_ptr(), B, ptrs, stream=0, init_zero=True, filter=True,
            bound_relax=1e-8, max_iter=ITERS, max_soc=4)
torch.cuda.synchronize()
nev = g.node_evals()
st = g.kernel_stats()
g.timing(False)
print("solve done: node evaluations", nev, "launches", {k: v[1] for k, v in st.items()})
if len(sys.argv) > 3:
    json.dump({"node_evals": int(nev), "batch": B, "iters": ITERS, "eval_launches": st["k_geval"][1]},
              open(sys.argv[3], "w"))
