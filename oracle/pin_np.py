"""ORACLE (test infrastructure only) — numpy restatement of the three Functions the
reference generates in ``src/casadi_pinocchio_bridge.hpp``.

* ``inverse_dynamics(model, q, qdot, qddot)`` — ``pinocchio::rnea`` as traced at
  ``casadi_pinocchio_bridge.hpp:76`` (Function ``inverse_dynamics``,
  ``{q,qdot,qddot}→{tau}``, L78).  Classic body-frame recursive Newton-Euler with
  the base acceleration set to ``-gravity`` (pinocchio's convention, gravity
  ``(0,0,-9.81)``).
* ``forward_kinematics(model, q, frame)`` — ``framesForwardKinematics`` +
  ``data.oMf[frame]`` (L103-111): returns ``(ee_pos (3,), ee_rot (3,3))``.
* ``jacobian(model, q, frame)`` — ``computeJointJacobians`` +
  ``getFrameJacobian(..., LOCAL_WORLD_ALIGNED)`` (L141-146): 6×nv, rows
  ``[linear; angular]`` of the frame origin, world-aligned axes.

Deliberately written in the *body-frame* Featherstone form so that it is an
independent restatement of the world-frame formulation used by the C oracle and
the HIP kernels.  Only tests / smoke / bench's CPU leg may import it.
"""
from __future__ import annotations

import numpy as np

from .urdf_np import Model


def _skew(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])


def _axis_rot(axis, q):
    K = _skew(axis)
    return np.eye(3) + np.sin(q) * K + (1 - np.cos(q)) * (K @ K)


def joint_transforms(model: Model, q):
    """Per joint: (R, t) of the joint frame in its parent joint frame at q."""
    out = []
    for j, jt in enumerate(model.joints):
        if jt.jtype == "revolute":
            R = jt.R @ _axis_rot(jt.axis, q[j])
            t = jt.t.copy()
        else:
            R = jt.R.copy()
            t = jt.t + jt.R @ (jt.axis * q[j])
        out.append((R, t))
    return out


def joint_placements(model: Model, q):
    """oMi for every movable joint."""
    loc = joint_transforms(model, q)
    oMi = []
    for j, jt in enumerate(model.joints):
        R, t = loc[j]
        if jt.parent < 0:
            oMi.append((R, t))
        else:
            Rp, tp = oMi[jt.parent]
            oMi.append((Rp @ R, Rp @ t + tp))
    return oMi


def frame_placement(model: Model, q, frame: str):
    if frame not in model.frames:
        raise KeyError(frame)
    f = model.frames[frame]
    if f.parent < 0:
        return f.R.copy(), f.t.copy()
    Rp, tp = joint_placements(model, q)[f.parent]
    return Rp @ f.R, Rp @ f.t + tp


def forward_kinematics(model: Model, q, frame: str):
    R, t = frame_placement(model, np.asarray(q, float), frame)
    return t, R


def _ancestors(model: Model, j: int):
    out = []
    while j >= 0:
        out.append(j)
        j = model.joints[j].parent
    return out


def jacobian(model: Model, q, frame: str):
    q = np.asarray(q, float)
    f = model.frames[frame]
    oMi = joint_placements(model, q)
    Rf, pf = frame_placement(model, q, frame)
    J = np.zeros((6, model.nv))
    if f.parent < 0:
        return J
    for j in _ancestors(model, f.parent):
        R, o = oMi[j]
        z = R @ model.joints[j].axis
        if model.joints[j].jtype == "revolute":
            J[0:3, j] = np.cross(z, pf - o)
            J[3:6, j] = z
        else:
            J[0:3, j] = z
    return J


# --- spatial algebra, pinocchio ordering [linear; angular] -------------------

def _motion_act_inv(R, t, v):
    lin, ang = v[:3], v[3:]
    return np.concatenate([R.T @ (lin - np.cross(t, ang)), R.T @ ang])


def _force_act(R, t, f):
    lin, ang = f[:3], f[3:]
    fl = R @ lin
    return np.concatenate([fl, R @ ang + np.cross(t, fl)])


def _motion_cross(v, m):
    vl, va = v[:3], v[3:]
    ml, ma = m[:3], m[3:]
    return np.concatenate([np.cross(va, ml) + np.cross(vl, ma), np.cross(va, ma)])


def _force_cross(v, f):
    vl, va = v[:3], v[3:]
    fl, fa = f[:3], f[3:]
    return np.concatenate([np.cross(va, fl), np.cross(va, fa) + np.cross(vl, fl)])


def _inertia_apply(I, v):
    lin, ang = v[:3], v[3:]
    h = I.m * (lin + np.cross(ang, I.c))      # linear momentum of the com
    return np.concatenate([h, I.Ic @ ang + np.cross(I.c, h)])


def inverse_dynamics(model: Model, q, qd, qdd):
    q = np.asarray(q, float).reshape(-1)
    qd = np.asarray(qd, float).reshape(-1)
    qdd = np.asarray(qdd, float).reshape(-1)
    n = model.nv
    loc = joint_transforms(model, q)
    S = []
    for jt in model.joints:
        if jt.jtype == "revolute":
            S.append(np.concatenate([np.zeros(3), jt.axis]))
        else:
            S.append(np.concatenate([jt.axis, np.zeros(3)]))
    a0 = np.concatenate([-model.gravity, np.zeros(3)])
    v = [None] * n
    a = [None] * n
    f = [None] * n
    for i, jt in enumerate(model.joints):
        R, t = loc[i]
        vp = np.zeros(6) if jt.parent < 0 else v[jt.parent]
        ap = a0 if jt.parent < 0 else a[jt.parent]
        vJ = S[i] * qd[i]
        v[i] = _motion_act_inv(R, t, vp) + vJ
        a[i] = _motion_act_inv(R, t, ap) + S[i] * qdd[i] + _motion_cross(v[i], vJ)
        f[i] = _inertia_apply(jt.inertia, a[i]) + _force_cross(v[i], _inertia_apply(jt.inertia, v[i]))
    tau = np.zeros(n)
    for i in range(n - 1, -1, -1):
        jt = model.joints[i]
        tau[i] = S[i] @ f[i]
        if jt.parent >= 0:
            R, t = loc[i]
            f[jt.parent] = f[jt.parent] + _force_act(R, t, f[i])
    return tau
