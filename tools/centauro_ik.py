"""Initial configuration of the substitute Centauro (C4): the inverse-kinematics problem of
Centauro_functions.py:207-260 -- min 1000|p_L - (B + L/2 e_y)|^2 + 1000|p_R - (B - L/2 e_y)|^2
+ 10|R_L - rot_ref|_F^2 + 10|R_R - rot_ref|_F^2 within the joint limits, B = (0.9, 0, 1.3), L = 0.4
(RepeatedMPCwithThermal.py:78-83) -- solved with scipy on the numpy kinematics of oracle/pin_np.py,
written to mpc_fatigue_amd/data/centauro_q0.json.  usage: python tools/centauro_ik.py
"""
import json
import os
import sys

import numpy as np
from scipy.optimize import minimize

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import pin_np as P  # noqa: E402
from oracle.urdf_np import load_urdf_file  # noqa: E402
from tools.make_centauro_urdf import LB, UB  # noqa: E402

B, L = np.array([0.9, 0.0, 1.3]), 0.4
ROT_REF = np.array([[0, 0, -1], [0, 1, 0], [1, 0, 0]], float)
U = os.path.join(ROOT, "mpc_fatigue_amd", "urdf")
M1 = load_urdf_file(os.path.join(U, "centauro_substitute_arm1.urdf"))
M2 = load_urdf_file(os.path.join(U, "centauro_substitute_arm2.urdf"))


def cost(q):
    pL, RL = P.forward_kinematics(M1, q[:7], "mass1_ee")
    pR, RR = P.forward_kinematics(M2, q[7:], "mass2_ee")
    c = 1000 * np.sum((pL - (B + [0, L / 2, 0])) ** 2) + 1000 * np.sum((pR - (B - [0, L / 2, 0])) ** 2)
    return c + 10 * np.sum((RL - ROT_REF) ** 2) + 10 * np.sum((RR - ROT_REF) ** 2)


def solve():
    bounds = list(zip(LB, UB))
    rng = np.random.default_rng(0)
    best = None
    home = np.array([-1.2, 0.3, 0.0, -1.0, 0.0, -0.3, 0.0])
    mir = np.array([1, -1, -1, 1, -1, 1, -1])
    starts = [np.r_[home, home * mir]] + [rng.uniform(LB, UB) for _ in range(20)]
    for x0 in starts:
        r = minimize(cost, np.clip(x0, LB, UB), method="L-BFGS-B", bounds=bounds, options={"maxiter": 5000})
        if best is None or r.fun < best.fun:
            best = r
    return best


if __name__ == "__main__":
    r = solve()
    q = r.x
    pL, RL = P.forward_kinematics(M1, q[:7], "mass1_ee")
    pR, RR = P.forward_kinematics(M2, q[7:], "mass2_ee")
    print("cost", r.fun, "pL", pL, "pR", pR)
    out = os.path.join(ROOT, "mpc_fatigue_amd", "data", "centauro_q0.json")
    json.dump({"q0": [round(float(v), 10) for v in q], "cost": float(r.fun),
               "note": "tools/centauro_ik.py: IK of Centauro_functions.py:207-260 on the substitute arms"},
              open(out, "w"), indent=1)
    print("wrote", out)
