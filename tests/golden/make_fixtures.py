"""Generates the committed fixtures that are not copied from the reference.

* ``mpc_fatigue_amd/data/pilz6_q0.json`` -- IK initial state of the Pilz-6DOF
  force problem (``force_optimization_pilz_6DOF.py:43-63``: prbt_link_5 at
  (0.1, 0.4, 0.2), solved from q = 0).  The reference uses IPOPT on
  ||fk(q) - p||^2; we use damped least squares from q = 0 on the numpy oracle's
  FK (``oracle/pin_np.py``).  Any exact IK is a valid start; the value is frozen
  because IK branches are solver dependent (hard parts).

Run:  python tests/golden/make_fixtures.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import pin_np as P  # noqa: E402
from oracle.urdf_np import load_urdf_file  # noqa: E402


def ik(model, frame, target, q=None, iters=500):
    q = np.zeros(model.nq) if q is None else np.array(q, float)
    lam = 1e-2
    for _ in range(iters):
        p, _ = P.forward_kinematics(model, q, frame)
        e = target - p
        if np.linalg.norm(e) < 1e-15:
            break
        J = P.jacobian(model, q, frame)[:3]
        dq = J.T @ np.linalg.solve(J @ J.T + lam * np.eye(3), e)
        step = np.abs(dq).max()
        if step > 0.1:            # step-limited so the iterate stays on the branch nearest q = 0
            dq *= 0.1 / step
        q = q + dq
    return q


def main():
    m = load_urdf_file(os.path.join(ROOT, "mpc_fatigue_amd", "urdf", "pilz_robot_6DOF.urdf"))
    target = np.array([0.1, 0.4, 0.2])
    q0 = ik(m, "prbt_link_5", target)
    p, _ = P.forward_kinematics(m, q0, "prbt_link_5")
    out = dict(q0=[float(x) for x in q0], frame="prbt_link_5", target=target.tolist(),
               residual=float(np.linalg.norm(p - target)),
               source="damped least squares from q=0 on oracle/pin_np.py FK (tests/golden/make_fixtures.py)")
    with open(os.path.join(ROOT, "mpc_fatigue_amd", "data", "pilz6_q0.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(out)


if __name__ == "__main__":
    main()
