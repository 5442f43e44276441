"""GPU parity of the batched IK (mf_ik_batch) against the numpy
damped-least-squares restatement that produced the frozen C2 initial state
(tests/golden/make_fixtures.py:ik on oracle/pin_np.py FK).

Tolerances: same iteration on FK values that agree to 1e-13, so iterates agree to 1e-9 rad;
residuals are held to 1e-12 m.  The reference's own IK (IPOPT from q = 0) has no committed
output for C2, so its branch choice is parity unpinned; the G1 box targets
(Box_Pilz_6DOF.py:96-105) pin reachability through the residual only.
"""
import json
import os

import numpy as np
import pytest

from mpc_fatigue_amd import _lib
from mpc_fatigue_amd.ik import ik_batch
from oracle import pin_np as P
from oracle.urdf_np import load_urdf_file
from tests.conftest import ROOT
from tests.golden.make_fixtures import ik as ik_np

pytestmark = pytest.mark.gpu
URDF = os.path.join(ROOT, "mpc_fatigue_amd", "urdf")


def model(name):
    with open(os.path.join(URDF, name)) as f:
        return _lib.Model(f.read()), load_urdf_file(os.path.join(URDF, name))


def test_ik_reproduces_frozen_c2_initial_state():
    m, _ = model("pilz_robot_6DOF.urdf")
    fx = json.load(open(os.path.join(ROOT, "mpc_fatigue_amd", "data", "pilz6_q0.json")))
    q, res = ik_batch(m, "prbt_link_5", [fx["target"]])
    np.testing.assert_allclose(q[0], fx["q0"], atol=1e-9)
    assert res[0] < 1e-12


def test_ik_batch_matches_numpy_restatement():
    m, ref = model("pilz_robot_6DOF.urdf")
    rng = np.random.default_rng(3)
    q0 = np.array(json.load(open(os.path.join(ROOT, "mpc_fatigue_amd", "data", "pilz6_q0.json")))["q0"])
    B = 96
    qs = q0 + rng.uniform(-0.3, 0.3, size=(B, 6))
    targets = np.array([P.forward_kinematics(ref, qq, "prbt_link_5")[0] for qq in qs])
    q, res = ik_batch(m, "prbt_link_5", targets)
    assert np.all(res < 1e-12)
    for b in range(0, B, 8):
        np.testing.assert_allclose(q[b], ik_np(ref, "prbt_link_5", targets[b]), atol=1e-9)
        np.testing.assert_allclose(P.forward_kinematics(ref, q[b], "prbt_link_5")[0], targets[b], atol=1e-12)


def test_ik_box_targets_reachable(golden):
    """Box_Pilz_6DOF.py:96-105: E1 = (0.2, 0.6, 0.4) on the first arm, E2 = (0.4, 0.6, 0.4) on the second."""
    for urdf, target in [("pilz_robot_6DOF_first.urdf", (0.2, 0.6, 0.4)), ("pilz_robot_6DOF_second.urdf", (0.4, 0.6, 0.4))]:
        m, ref = model(urdf)
        q, res = ik_batch(m, "end_effector", [target], iters=2000)
        assert res[0] < 1e-10, (urdf, res[0])
        np.testing.assert_allclose(P.forward_kinematics(ref, q[0], "end_effector")[0], target, atol=1e-10)


def test_ik_errors():
    m, _ = model("pilz_robot_6DOF.urdf")
    with pytest.raises(_lib.MFError):
        ik_batch(m, "no_such_frame", [[0.1, 0.4, 0.2]])
    with pytest.raises(_lib.MFError):
        ik_batch(m, "prbt_link_5", [[0.1, 0.4, 0.2]], lam=0.0)
