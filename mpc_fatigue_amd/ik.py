"""Batched inverse kinematics on the GPU.

Every reference script computes its initial state by solving min ||fk(q) - p||^2 with
IPOPT from q = 0 (``python/Pilz_6_DOF/force_optimization_pilz_6DOF.py:55-63``,
``python/2_pilz_6_DOF/Box_Pilz_6DOF.py:123-156``).  ``ik_batch`` solves a batch of such
targets at once through ``mf_ik_batch`` (one lane per target, damped least squares with a
capped step, ``csrc/capi.hip`` k_ik), e.g. to produce feasible initial states for a batch
of MPC horizons.  IK branches are solver dependent: from q = 0 with the default step cap
the iterate stays on the branch nearest zero, which is the branch the frozen C2 initial
state (``data/pilz6_q0.json``) was produced on.
"""
from __future__ import annotations

import numpy as np

from . import _lib


def ik_batch(model: _lib.Model, frame: str | int, targets, q_init=None, iters: int = 500, lam: float = 1e-2,
             max_step: float = 0.1, tol: float = 1e-15):
    """q (B, n), residual |p - fk(q)| (B,) for the frame-position targets (B, 3)."""
    fid = model.frame_id(frame) if isinstance(frame, str) else int(frame)
    t = np.ascontiguousarray(np.atleast_2d(np.asarray(targets, dtype=np.float64)))
    if t.shape[1] != 3:
        raise ValueError("targets must be (B, 3)")
    B, n = t.shape[0], model.nq
    qi = None
    if q_init is not None:
        qi = np.ascontiguousarray(np.broadcast_to(np.asarray(q_init, dtype=np.float64), (B, n)))
    q = np.zeros((B, n))
    res = np.zeros(B)
    _lib.check(_lib.lib().mf_ik_batch(model.handle, fid, _lib.dptr(t), _lib.dptr(qi) if qi is not None else None,
                                      _lib.dptr(q), _lib.dptr(res), B, iters, lam, max_step, tol))
    return q, res


def ik_batch_dev(model: _lib.Model, frame: int, targets_ptr: int, q_out_ptr: int, batch: int, q_init_ptr=None,
                 residual_ptr=None, iters: int = 500, lam: float = 1e-2, max_step: float = 0.1, tol: float = 1e-15,
                 stream=None):
    """Device-pointer form (e.g. torch tensors' data_ptr()), asynchronous on ``stream``."""
    _lib.check(_lib.lib().mf_ik_batch_dev(model.handle, frame, targets_ptr, q_init_ptr, q_out_ptr, residual_ptr, batch,
                                          iters, lam, max_step, tol, stream))
