import sys, os, time
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from mpc_fatigue_amd import problems as PR, pin
from mpc_fatigue_amd.ocp import OCP
torch.cuda.init()
dev = torch.device("cuda", 0)
sp = PR.pilz6_bench(N=100)
ocp = OCP(sp)
Q = PR.pilz6_batch_q0(64, seed=0)
LR = pin.generate_forward_kin(PR.read_urdf(sp["urdf"]), sp["frame"]).batch(Q)[0][:, :2]
q0 = torch.tensor(Q, dtype=torch.float64, device=dev); lr = torch.tensor(np.ascontiguousarray(LR), dtype=torch.float64, device=dev)
st = torch.cuda.Stream(dev)
for nb in (1, 8, 64):
    out = {"w": torch.empty((nb, ocp.wsize), dtype=torch.float64, device=dev), "status": torch.empty(nb, dtype=torch.int32, device=dev),
           "iters": torch.empty(nb, dtype=torch.int32, device=dev), "kkt": torch.empty(nb, dtype=torch.float64, device=dev),
           "obj": torch.empty(nb, dtype=torch.float64, device=dev)}
    pt = {k: v.data_ptr() for k, v in out.items()}
    ts = []
    for r in range(6):
        torch.cuda.synchronize(dev); t = time.perf_counter()
        ocp.solve_dev(q0.data_ptr(), lr.data_ptr(), nb, pt, stream=st.cuda_stream, F_init=PR.BENCH_F_INIT, tol=1e-8, constr_viol_tol=1e-8, max_iter=300)
        st.synchronize(); ts.append(time.perf_counter() - t)
    print(nb, "median ms", round(float(np.median(ts[1:])) * 1e3, 2), "iters", out["iters"].cpu().numpy()[:4], flush=True)
