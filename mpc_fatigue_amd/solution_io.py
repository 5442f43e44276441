"""Solution I/O in the reference's formats.

* ``write_solution_csv`` / ``read_solution_csv``: one CSV row holding the whole decision vector
  ``sol = r['x']`` in the OCP's layout, as ``Box_Pilz_6DOF.py:464-466`` writes it
  (``csv.writer(...).writerow(sol)``) and its plotting section reads it back (L472-477:
  split on commas, float each field).  The reference's committed solutions
  (``plotter/solution.csv``, ``plotter/Result_*/solution.csv``) are files of this format.
* ``unroll``: the per-node records a ROS-free replacement of the unroller / talker nodes needs
  (``Centauro_script/unroller_node.py:13-24`` reads [trajectory | force | torque] blocks per
  node): joint angles, velocities, forces and the joint torques tau = ID(q, qd, 0) - J^T [F; 0]
  of every node, evaluated on the GPU through the bridge functions.
"""
from __future__ import annotations

import csv

import numpy as np

from . import _lib
from .mpc import split_w


def write_solution_csv(path: str, w) -> None:
    """One row, the decision vector in its layout, full double precision (repr)."""
    w = np.asarray(w, dtype=np.float64).ravel()
    with open(path, "w", newline="") as f:
        csv.writer(f).writerow([repr(float(x)) for x in w])


def read_solution_csv(path: str) -> np.ndarray:
    """The reader of Box_Pilz_6DOF.py:472-477: every comma-separated field of every line."""
    out = []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if line:
                out.extend(float(v) for v in line.split(","))
    return np.array(out)


def unroll(w, spec: dict, model: _lib.Model | None = None) -> dict:
    """Per-node records of a C1/C2-layout solution: q (N+1, n), qd (N, n), F (N, nf),
    tau (N, n) with tau_k = ID(q_k, qd_k, 0) - J_f(q_k)^T [sum_a F_a fdir_a; 0]."""
    from .pin import ForwardKinematics, FrameJacobian, InverseDynamics  # noqa: F401 (GPU bridge)
    from . import problems as PR

    n = len(spec["q0"])
    N, nf = spec["N"], spec["nf"]
    q, qd, F = (a[0] for a in split_w(np.asarray(w, float)[None], n, nf, N))
    if model is None:
        model = _lib.Model(PR.read_urdf(spec["urdf"]))
    idyn = InverseDynamics(model)
    tau = idyn.batch(q[:N], qd, np.zeros((N, n)))
    if nf > 0:
        J = FrameJacobian(model, spec["frame"]).batch(q[:N])  # (N, 6, n)
        Fw = F @ np.asarray(spec["fdir"], float).reshape(nf, 3)  # (N, 3) world force
        tau = tau - np.einsum("kri,kr->ki", J[:, :3, :], Fw)
    return {"q": q, "qd": qd, "F": F, "tau": tau}


def centauro_split(w, N: int, thermal: bool = True, nq: int = 14) -> dict:
    """Blocks of a Centauro solution vector.  Thermal layout (RepeatedMPCwithThermal.py:183-391):
    [q_0, T_0 | (qd_k, F_L, F_R, q_{k+1}, T_{k+1}) x N]; non-thermal layout of the committed
    Centauro_solutions/**/solution.csv (Centauro_dynamics.py / CentaurOCP.py):
    [(q_k, qd_k, F_L, F_R) x N | q_N].  Returns q (N+1, nq), qd (N, nq), F (N, 6) and T (N+1, nq)."""
    w = np.asarray(w, dtype=np.float64).ravel()
    if thermal:
        nx, nu = 2 * nq, nq + 6
        blk = w[nx:].reshape(N, nu + nx)
        x = np.vstack([w[:nx][None], blk[:, nu:]])
        return {"q": x[:, :nq], "T": x[:, nq:], "qd": blk[:, :nq], "F": blk[:, nq:nu]}
    st = 2 * nq + 6
    blk = w[:N * st].reshape(N, st)
    q = np.vstack([blk[:, :nq], w[N * st:][None]])
    return {"q": q, "T": None, "qd": blk[:, nq:2 * nq], "F": blk[:, 2 * nq:st]}


def centauro_invariants(w, N: int, h: float, mg: float, thermal: bool = True) -> dict:
    """The checks a Centauro solution file must pass whatever the robot model:
    explicit-Euler continuity max |q_{k+1} - q_k - h qd_k| and the force balance of the box,
    max |F_Lz + F_Rz - m g| and max |F_L,xy + F_R,xy| (RepeatedMPCwithThermal.py:238-246)."""
    b = centauro_split(w, N, thermal)
    q, qd, F = b["q"], b["qd"], b["F"]
    return {"continuity": float(np.abs(q[1:] - q[:-1] - h * qd).max()),
            "force_z": float(np.abs(F[:, 2] + F[:, 5] - mg).max()),
            "force_xy": float(np.abs(F[:, 0:2] + F[:, 3:5]).max())}
