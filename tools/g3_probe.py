import sys, numpy as np, os
sys.path.insert(0, '/root/repo')
import torch; torch.cuda.init()
from mpc_fatigue_amd import problems as PR
from mpc_fatigue_amd.gocp import GOCP
G = {n: np.loadtxt(f'/root/repo/tests/golden/{n}_solution.csv', delimiter=',') for n in ['G1_box_N50','G2_box_N80','G3_box_N80','G4_box_N80']}
IP = dict(init_zero=True, bound_relax=1e-8, filter=True, max_iter=1500, max_soc=4)
for case, name, kw in [("G1","G1_box_N50",dict(N=50)),("G2","G2_box_N80",dict(N=80)),("G3","G3_box_N80",dict(N=80,left_const=True)),("G4","G4_box_N80",dict(N=80,right_const=False))]:
    g = G[name]
    spec = PR.box_dual(q0=g[:12], **kw)
    o = GOCP(spec)
    r = o.solve(**IP)
    q = o.q_traj(r.w[0])
    w_or = np.loadtxt(f'/root/repo/tests/golden/ipopt_mode_{case}.csv', delimiter=',')
    print(case, 'status', int(r.status[0]), 'iters', int(r.iters[0]), 'obj', float(r.obj[0]), 'dq vs reference CSV', np.abs(q - o.q_traj(g)).max(), 'dq vs oracle fixture', np.abs(q - o.q_traj(w_or)).max(), flush=True)
