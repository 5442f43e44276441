"""Problem specs: the reference's OCP transcriptions as plain data.

Each spec is a dict consumed both by the product (``mpc_fatigue_amd.ocp`` →
``mf_problem_create``) and by the test oracle.  Constants are taken verbatim
from the reference scripts (file:line cited per field).

Stage structure shared by every spec (``force_optimization_pilz_6DOF.py:103-172``):
    w = [q_0 | (qd_k, F_k, q_{k+1}) for k in 0..N-1]
    q_0 fixed, qd_0 fixed (= qd0), q_{k+1} = q_k + h qd_k
    tau_k = ID(q_k, qd_k, 0) - J_frame(q_k)^T [fdir F_k; 0]  in [tau_lo[k], tau_hi[k]]
    optional line constraint fk_frame(q_k)[0:2] = line_ref  (k >= 1; k = 0 is fixed data)
    cost = sum_k wF |F_k|^2 + wqd |qd_k|^2 + wtau |tau_k|^2
"""
from __future__ import annotations

import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
URDF_DIR = os.path.join(HERE, "urdf")
INF = float("inf")


def urdf_path(name: str) -> str:
    return os.path.join(URDF_DIR, name)


def read_urdf(name: str) -> str:
    with open(urdf_path(name)) as f:
        return f.read()


def torque_envelope(N: int, h: float, tau0: float, alpha: float, bound: float) -> np.ndarray:
    """Fatigue envelope B_k = tau0 e^{-alpha k h} if that exceeds ``bound`` else ``bound``.

    ``force_optimization_pilz_6DOF.py:136-148`` (same rule in
    ``inverse_dynamics_pilz_3DOF.py:127-139``).
    """
    k = np.arange(N)
    t = tau0 * np.exp(-alpha * k * h)
    return np.where(t > bound, t, bound)


# IK initial state for the Pilz-6DOF force problem: prbt_link_5 at (0.1, 0.4, 0.2)
# (force_optimization_pilz_6DOF.py:43-63).  The reference solves this with IPOPT
# from q = 0; we freeze our own damped-least-squares IK from q = 0 as a fixture
# (tests/golden/make_fixtures.py) because IK branches are solver-dependent.
_Q0_FILE = os.path.join(HERE, "data", "pilz6_q0.json")


def pilz6_q0() -> np.ndarray:
    with open(_Q0_FILE) as f:
        return np.array(json.load(f)["q0"], float)


# The reference's fatigue floor (bound_torque = 15 Nm, force_optimization_pilz_6DOF.py:89)
# makes the Pilz-6DOF force problem infeasible: over every configuration with
# prbt_link_5 on the line x=0.1, y=0.4 the smallest achievable max joint torque
# (gravity, best x-force) is 16.64 Nm (tests/test_problems.py reproduces it).
# The benchmark instance keeps every other constant and uses the smallest round
# floor that is feasible from the IK start, 30 Nm.
REFERENCE_FLOOR = 15.0
BENCH_FLOOR = 30.0
BENCH_F_INIT = 1.0   # IPOPT's x0 = 0 starts on the F = 0 saddle of -F^2


def pilz6_force(N: int = 100, T: float = 2.0, q0=None, line_ref=(0.1, 0.4), tau_floor: float = REFERENCE_FLOOR) -> dict:
    """C2: ``python/Pilz_6_DOF/force_optimization_pilz_6DOF.py`` at N shooting nodes.

    T=2 (L78), tau0=50, alpha=2, qd in +-0.4, bound 15 (L84-89), line on
    prbt_link_5 x/y (L150-156), cost -F^T F with F = [Fx,0,0,0,0,0] (L131-134, L177).
    """
    h = T / N
    B = torque_envelope(N, h, 50.0, 2.0, tau_floor)
    n = 6
    return dict(
        name="pilz6_force", urdf="pilz_robot_6DOF.urdf", frame="prbt_link_5", tau_floor=tau_floor,
        N=N, h=h, nf=1, fdir=[[1.0, 0.0, 0.0]],
        use_line=True, line_ref=list(line_ref),
        wF=-1.0, wqd=0.0, wtau=0.0,
        q0=list(pilz6_q0() if q0 is None else q0), qd0=[0.0] * n,
        qd_lo=[-0.4] * n, qd_hi=[0.4] * n,
        q_lo=[-INF] * n, q_hi=[INF] * n,
        tau_lo=np.repeat(-B[:, None], n, 1), tau_hi=np.repeat(B[:, None], n, 1),
    )


def pilz3_working(N: int = 50, T: float = 4.0) -> dict:
    """C1: ``python/Pilz_3_DOF/inverse_dynamics_pilz_3DOF_working.py`` (all 3 joints).

    q0 = [0, 1.2124, -0.5] (inverse_dynamics_pilz_3DOF.py:71), qd in +-100,
    tau0=50, alpha=2, bound 10, q in +-[2.96, 2.53, 2.35], cost tau^T tau + 100 qd^T qd.
    """
    h = T / N
    B = torque_envelope(N, h, 50.0, 2.0, 10.0)
    n = 3
    return dict(
        name="pilz3_working", urdf="pilz_robot_3DOF.urdf", frame="prbt_link_5",
        N=N, h=h, nf=0, fdir=[],
        use_line=False, line_ref=[0.0, 0.0],
        wF=0.0, wqd=100.0, wtau=1.0,
        q0=[0.0, 1.2124, -0.5], qd0=[0.0] * n,
        qd_lo=[-100.0] * n, qd_hi=[100.0] * n,
        q_lo=[-2.96, -2.53, -2.35], q_hi=[2.96, 2.53, 2.35],
        tau_lo=np.repeat(-B[:, None], n, 1), tau_hi=np.repeat(B[:, None], n, 1),
    )


# ---------------------------------------------------------------- phase-scheduled limits (s.8 a7)
# The solver takes any per-node torque bounds (tau_lo / tau_hi are N x n); these builders
# reproduce the reference's phase tables exactly.

# both_robots_torque_limited_2_pilz.py:120-147: limits switched at t = 0.75 s and 1.5 s
TIME_PHASE_LISTS = ([60, 30, 1000, 300, 300, 50], [10, 100, 50, 500, 1500, 50], [50, 110, 400, 300, 500, 50])


def time_phase_limits(N: int, T: float, t1: float = 0.75, t2: float = 1.5, lists=TIME_PHASE_LISTS):
    """(lo, hi), each N x 6: node i < n1 -> +-list_1, n1 <= i < n2 -> +-list_2, else +-list_3,
    n1 = int(t1 / h), n2 = int(t2 / h), h = T / N (both_robots_torque_limited_2_pilz.py:120-147)."""
    h = T / N
    n1, n2 = int(t1 / h), int(t2 / h)
    i = np.arange(N)[:, None]
    lim = np.where(i < n1, np.asarray(lists[0], float), np.where(i < n2, np.asarray(lists[1], float),
                                                                np.asarray(lists[2], float)))
    return -lim, lim


# Box_Pilz_6DOF.py:287-383: joints 0-2 of the right arm and 0-1 of the left arm follow a
# three-phase table switched at k = int(N/3), int(2N/3); every other torque row is +-500
BOX_RIGHT = ([(-200.0, 100.0), (-60.0, 60.0), (-30.0, 40.0)],
             [(-50.0, 50.0), (-30.0, 10.0), (-20.0, 20.0)],
             [(-5.0, 5.0), (-5.0, 5.0), (-10.0, 5.0)])
BOX_LEFT = ([(-600.0, 400.0), (-60.0, 60.0)],
            [(-50.0, 50.0), (-30.0, 40.0)],
            [(-5.0, 5.0), (-5.0, 5.0)])


def box_phase_limits(N: int, arm: str = "right", constrained: bool = True):
    """(lo, hi), each N x 6, of one arm of Box_Pilz_6DOF.py (RightConst / LeftConst)."""
    lo, hi = np.full((N, 6), -500.0), np.full((N, 6), 500.0)
    if not constrained:
        return lo, hi
    table = BOX_RIGHT if arm == "right" else BOX_LEFT
    for k in range(N):
        ph = 0 if k < int(N / 3) else (1 if k < int(2 * N / 3) else 2)
        for j, (a, b) in enumerate(table[ph]):
            lo[k, j], hi[k, j] = a, b
    return lo, hi


def pilz6_phase(N: int = 100, T: float = 2.0, q0=None, line_ref=(0.1, 0.4), scale: float = 1.0) -> dict:
    """The C2 force task under the time-phase schedule of both_robots_torque_limited_2_pilz.py
    (scaled by ``scale``) instead of the exponential envelope: the single-arm instance that runs
    the a7 bound tables through the solver (the dual-arm OCP itself is s.8f rank 1)."""
    sp = pilz6_force(N=N, T=T, q0=q0, line_ref=line_ref)
    lo, hi = time_phase_limits(N, T)
    sp.update(name="pilz6_phase", tau_lo=lo * scale, tau_hi=hi * scale)
    return sp


def pilz6_batch_q0(batch: int, seed: int = 0, spread: float = 0.05, q0=None) -> np.ndarray:
    """C5 initial states: q0_i = q0 + U(-spread, spread) per joint, numpy default_rng(seed)."""
    base = pilz6_q0() if q0 is None else np.asarray(q0, float)
    rng = np.random.default_rng(seed)
    return base[None, :] + rng.uniform(-spread, spread, size=(batch, base.size))


def pilz6_bench(N: int = 100, q0=None, line_ref=(0.1, 0.4)) -> dict:
    """The benchmark instance of C2 (feasible fatigue floor, see BENCH_FLOOR)."""
    return pilz6_force(N=N, q0=q0, line_ref=line_ref, tau_floor=BENCH_FLOOR)
