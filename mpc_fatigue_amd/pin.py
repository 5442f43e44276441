"""Drop-in for the reference's ``mpc_fatigue.pynocchio_casadi`` module.

Reference (bindings/python/pynocchio_casadi.cpp:11-19) exports three functions
that take a URDF string and return a *serialized CasADi Function*; every script
then calls ``casadi.Function.deserialize`` and evaluates it numerically, e.g.

    Idyn(q=qc, qdot=qcdot, qddot=qcddot)['tau']      # force_optimization_pilz_6DOF.py:263
    jac_dict(q=qc)["J"][0:6,0:6]                       # force_optimization_pilz_6DOF.py:259
    fk(q=qc)['ee_pos'][0:2]                            # force_optimization_pilz_6DOF.py:152

Here the three generators return callables with exactly that call surface
(keyword call -> dict, positional call -> output / list of outputs), evaluated
on the GPU through libmpcfatigue.so.  Outputs are numpy arrays with CasADi DM
shapes: tau (nv,1), ee_pos (3,1), ee_rot (3,3), J (6,nv).  Symbolic (SX)
arguments cannot be supported on a GPU; the symbolic transcription is replaced
by ``mpc_fatigue_amd.ocp`` (problem spec -> batched solve).
"""
from __future__ import annotations

import numpy as np

from . import _lib


def _vec(x, n: int, name: str) -> np.ndarray:
    a = np.asarray(x, dtype=np.float64).reshape(-1)
    if a.size != n:
        raise ValueError(f"argument '{name}' has {a.size} entries, expected {n}")
    return np.ascontiguousarray(a)


def _rows(x, n: int, name: str) -> np.ndarray:
    a = np.asarray(x, dtype=np.float64)
    a = a.reshape(-1, n) if a.ndim != 2 or a.shape[1] != n else a
    return np.ascontiguousarray(a)


class _Function:
    name = "function"
    _in: tuple = ()
    _out: tuple = ()

    def name_in(self):
        return list(self._in)

    def name_out(self):
        return list(self._out)

    def n_in(self):
        return len(self._in)

    def n_out(self):
        return len(self._out)

    def __call__(self, *args, **kw):
        if args and kw:
            raise TypeError("use either positional or keyword arguments")
        if kw:
            unknown = set(kw) - set(self._in)
            if unknown:
                raise KeyError(f"{self.name}: unknown input(s) {sorted(unknown)}; inputs are {list(self._in)}")
            vals = [kw.get(k) for k in self._in]
            res = self._eval(*vals)
            return dict(zip(self._out, res))
        if len(args) != len(self._in):
            raise TypeError(f"{self.name} takes {len(self._in)} positional inputs")
        res = self._eval(*args)
        return res[0] if len(res) == 1 else list(res)


class InverseDynamics(_Function):
    """Function 'inverse_dynamics' {q, qdot, qddot} -> {tau} (casadi_pinocchio_bridge.hpp:78)."""

    name = "inverse_dynamics"
    _in = ("q", "qdot", "qddot")
    _out = ("tau",)

    def __init__(self, model: _lib.Model):
        self.model = model

    def _eval(self, q, qdot, qddot):
        n = self.model.nq
        qdot = np.zeros(n) if qdot is None else qdot
        qddot = np.zeros(n) if qddot is None else qddot
        tau = self.batch(_vec(q, n, "q")[None], _vec(qdot, n, "qdot")[None], _vec(qddot, n, "qddot")[None])
        return (tau.reshape(n, 1),)

    def batch(self, q, qd, qdd) -> np.ndarray:
        n = self.model.nq
        q, qd, qdd = _rows(q, n, "q"), _rows(qd, n, "qdot"), _rows(qdd, n, "qddot")
        tau = np.zeros_like(q)
        _lib.check(_lib.lib().mf_id(self.model.handle, _lib.dptr(q), _lib.dptr(qd), _lib.dptr(qdd), _lib.dptr(tau),
                                    q.shape[0]))
        return tau


class ForwardKinematics(_Function):
    """Function 'forward_kinematics' {q} -> {ee_pos, ee_rot} (casadi_pinocchio_bridge.hpp:111)."""

    name = "forward_kinematics"
    _in = ("q",)
    _out = ("ee_pos", "ee_rot")

    def __init__(self, model: _lib.Model, frame: str):
        self.model = model
        self.frame = model.frame_id(frame)

    def _eval(self, q):
        p, R = self.batch(_vec(q, self.model.nq, "q")[None])
        return p[0].reshape(3, 1), R[0]

    def batch(self, q):
        q = _rows(q, self.model.nq, "q")
        B = q.shape[0]
        pos, rot = np.zeros((B, 3)), np.zeros((B, 9))
        _lib.check(_lib.lib().mf_fk(self.model.handle, self.frame, _lib.dptr(q), _lib.dptr(pos), _lib.dptr(rot), B))
        return pos, rot.reshape(B, 3, 3).transpose(0, 2, 1)  # column-major -> (row, col)


class FrameJacobian(_Function):
    """Function 'jacobian' {q} -> {J}, LOCAL_WORLD_ALIGNED 6 x nv (casadi_pinocchio_bridge.hpp:141-146)."""

    name = "jacobian"
    _in = ("q",)
    _out = ("J",)

    def __init__(self, model: _lib.Model, frame: str):
        self.model = model
        self.frame = model.frame_id(frame)

    def _eval(self, q):
        return (self.batch(_vec(q, self.model.nq, "q")[None])[0],)

    def batch(self, q):
        n = self.model.nq
        q = _rows(q, n, "q")
        B = q.shape[0]
        J = np.zeros((B, 6 * n))
        _lib.check(_lib.lib().mf_jac(self.model.handle, self.frame, _lib.dptr(q), _lib.dptr(J), B))
        return J.reshape(B, n, 6).transpose(0, 2, 1)


_models: dict[int, _lib.Model] = {}


def _model(urdf: str) -> _lib.Model:
    key = hash(urdf)
    if key not in _models:
        _models[key] = _lib.Model(urdf)
    return _models[key]


def generate_inv_dyn(urdf_string: str) -> InverseDynamics:
    """Replaces ``pin.generate_inv_dyn`` (pynocchio_casadi.cpp:14, bridge L57-85)."""
    return InverseDynamics(_model(urdf_string))


def generate_forward_kin(urdf_string: str, body_name: str) -> ForwardKinematics:
    """Replaces ``pin.generate_forward_kin`` (pynocchio_casadi.cpp:15, bridge L87-117)."""
    return ForwardKinematics(_model(urdf_string), body_name)


def generate_jacobian(urdf_string: str, body_name: str) -> FrameJacobian:
    """Replaces ``pin.generate_jacobian`` (pynocchio_casadi.cpp:16, bridge L119-153)."""
    return FrameJacobian(_model(urdf_string), body_name)
