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


# ---------------------------------------------------------------- C3: dual-arm box (s.8 a5, a10, a11)
# Box_Pilz_6DOF.py: joint limits L176-177, qd in [-1, 0.5] L179-180, m = 30 kg L182,
# equilibrium tolerance pos_toll = 1e-4 L184, Lbox = 0.2 and the IK targets L94-114.
BOX_JOINT_LIM = [2.96, 2.53, 2.35, 2.96, 2.96, 3.12]
_BOX_Q0_FILE = os.path.join(HERE, "data", "box_q0.json")


def box_q0() -> np.ndarray:
    """The dual-arm IK start (Box_Pilz_6DOF.py:123-156), as the reference's committed solution holds it."""
    with open(_BOX_Q0_FILE) as f:
        return np.array(json.load(f)["q0"], float)


def box_dual(N: int = 50, T: float = 2.0, q0=None, right_const: bool = True, left_const: bool = False,
             torque_const: bool = True, mass: float = 30.0, Lbox: float = 0.2, qd_lo: float = -1.0,
             qd_hi: float = 0.5) -> dict:
    """C3: ``python/2_pilz_6_DOF/Box_Pilz_6DOF.py`` (two Pilz arms holding a box).

    x = [q_L(6), q_R(6)], u = [qd_L(6), qd_R(6), F_L(3), F_R(3)] (L213-262).  Rows per node:
    force equilibrium F_L + F_R = (0, 0, m g) and moment equilibrium (E1 - E2) x (F_L - F_R) = 0
    within +-pos_toll (L268-277), torques tau = ID - J^T [F; 0] of both arms in the phase tables
    (L285-399), end-effector distance |E1 - E2|^2 = L (L279-282), cost
    100 |(E1 + E2)/2 - p_des|^2 + qd^T qd (L415-416), explicit Euler (L423-436).
    """
    h = T / N
    p1 = np.array([0.2, 0.6, 0.4])
    p2 = p1 + np.array([Lbox, 0.0, 0.0])
    lim = np.array(BOX_JOINT_LIM * 2)
    if torque_const:
        lo_l, hi_l = box_phase_limits(N, "left", left_const)
        lo_r, hi_r = box_phase_limits(N, "right", right_const)
    else:
        lo_l = lo_r = np.full((N, 6), -INF)
        hi_l = hi_r = np.full((N, 6), INF)
    return dict(
        name="box_dual", family="box", urdf=["pilz_robot_6DOF_first.urdf", "pilz_robot_6DOF_second.urdf"],
        frame="end_effector", N=N, h=h, n=12, nf=6,
        q0=list(box_q0() if q0 is None else q0), qd0=[0.0] * 12,
        qd_lo=[qd_lo] * 12, qd_hi=[qd_hi] * 12, q_lo=list(-lim), q_hi=list(lim),
        pos_toll=1e-4, box_mg=9.81 * mass, box_L=float((p1 - p2) @ (p1 - p2)), p_des=list((p1 + p2) / 2),
        w_box=100.0, w_qd=1.0,
        tau_lo=np.hstack([lo_l, lo_r]), tau_hi=np.hstack([hi_l, hi_r]),
    )


def box_homotopy_tolerances():
    """Equilibrium-tolerance homotopy of the C3 solve: pos_toll 1 -> 1e-2 -> the
    reference's 1e-4, each stage warm-started from the previous primal point.  Only the path to the
    solution changes; the last stage is Box_Pilz_6DOF.py's problem verbatim."""
    return [1.0, 1e-2, 1e-4]


def box_u_init(spec: dict) -> np.ndarray:
    """Initial control: qd = 0, each arm carries half the box weight (the warm-start force of
    RepeatedMPCwithThermal.py:148, F0 = [0, 0, m g / 2] per arm)."""
    mg = spec["box_mg"]
    return np.r_[np.zeros(12), 0.0, 0.0, mg / 2, 0.0, 0.0, mg / 2]


# ---------------------------------------------------------------- thermal fatigue state (s.8 a8)
# Tmodel_library.py:9-32: Ra = 10, Rh = 2, R_theta = R1 R2 / (R1 + R2) (R1 = 300, R2 = 9), C_theta = 15,
# T_theta = R_theta C_theta; ktau per joint (L32).  Recursion RepeatedMPCwithThermal.py:371-376:
#   T_{k+1} = a T_k + R_theta (1 - a) (Ra (tau / ktau)^2 + qd^2 / Rh),  a = exp(-h / T_theta)
# with T in [0, 80] (L122-123) and T_0 = 20 (L140).
TH_RA, TH_RH = 10.0, 2.0
TH_RTHETA = 300.0 * 9.0 / (300.0 + 9.0)
TH_TTHETA = TH_RTHETA * 15.0
KTAU14 = (30.0, 40.0, 40.0, 40.0, 40.0, 30.0, 50.0, 30.0, 30.0, 40.0, 40.0, 40.0, 40.0, 50.0)


def thermal_coeffs(h: float):
    """(a, b): T' = a T + b P with a = e^{-h / T_theta}, b = R_theta (1 - a)."""
    a = float(np.exp(-h / TH_TTHETA))
    return a, TH_RTHETA * (1.0 - a)


def with_thermal(spec: dict, T0=20.0, T_lo: float = 0.0, T_hi: float = 80.0, ktau=None) -> dict:
    """Adds the motor-winding temperature of every joint as state: x = [q, T], the thermal recursion as
    dynamics, T in [T_lo, T_hi] for k >= 1.  T0 may be a vector (a receding horizon carries T_N - 0.05,
    mpc_principal.py:365-374).  ktau defaults to the first n entries of the reference table."""
    n = len(spec["q0"])
    a, b = thermal_coeffs(spec["h"])
    sp = dict(spec)
    sp.update(name=spec["name"] + "_thermal", thermal=True, th_a=a, th_b=b, Ra=TH_RA, Rh=TH_RH,
              ktau=list(KTAU14[:n] if ktau is None else ktau), T0=list(np.broadcast_to(np.asarray(T0, float), (n,))),
              T_lo=T_lo, T_hi=T_hi)
    return sp


def pilz6_thermal(N: int = 100, T0=79.0, q0=None, line_ref=(0.1, 0.4)) -> dict:
    """Thermal C2 variant (build-defined; parity unpinned by construction): the benchmark force task with
    the winding temperatures as state, starting hot (T0 = 79 C, one degree under the reference's 80 C
    limit).  Over the 2 s horizon the windings warm by 0.28 C at most (T_max 79.28 C): the bound stays
    inactive and the optimum equals the non-thermal one (tests/test_oracle_generic.py).  The instance with
    the bound active is C4 started hot (centauro(T0=79), tests/test_gpu_generic.py)."""
    return with_thermal(pilz6_bench(N=N, q0=q0, line_ref=line_ref), T0=T0)


def pilz6_batch_q0(batch: int, seed: int = 0, spread: float = 0.05, q0=None) -> np.ndarray:
    """C5 initial states: q0_i = q0 + U(-spread, spread) per joint, numpy default_rng(seed)."""
    base = pilz6_q0() if q0 is None else np.asarray(q0, float)
    rng = np.random.default_rng(seed)
    return base[None, :] + rng.uniform(-spread, spread, size=(batch, base.size))


def pilz6_bench(N: int = 100, q0=None, line_ref=(0.1, 0.4)) -> dict:
    """The benchmark instance of C2 (feasible fatigue floor, see BENCH_FLOOR)."""
    return pilz6_force(N=N, q0=q0, line_ref=line_ref, tau_floor=BENCH_FLOOR)


# ---------------------------------------------------------------- C4: Centauro thermal box lift
# Centauros_features.py:22-34 (limits of j_arm1_1..7, j_arm2_1..7)
CENT_Q_LO = [-3.312, 0.020, -2.552, -2.465, -2.569, -1.529, -2.565, -3.3458, -3.4258, -2.5614, -2.4794, -2.5394,
             -1.5154, -2.5554]
CENT_Q_HI = [1.615, 3.431, 2.566, 0.280, 2.562, 1.509, 2.569, 1.6012, -0.0138, 2.5606, 0.2886, 2.5546, 1.5156, 2.5686]
CENT_QD_LIM = [3.86, 3.86, 6.06, 6.06, 11.72, 11.72, 20.35] * 2
CENT_TAU_LIM = [147.0, 147.0, 147.0, 147.0, 55.0, 55.0, 28.32] * 2
_CQ0_FILE = os.path.join(HERE, "data", "centauro_q0.json")


def centauro_q0() -> np.ndarray:
    """IK start of the substitute arms (tools/centauro_ik.py: the problem of Centauro_functions.py:207-260)."""
    with open(_CQ0_FILE) as f:
        return np.array(json.load(f)["q0"], float)


def centauro(N: int = 40, T: float = 30.0, q0=None, T0=20.0, qd0=None, mass: float = 10.0,
             box_pos=(0.9, 0.0, 1.3), target_decimals: int = -1) -> dict:
    """C4: the thermal Centauro MPC of ``python/Centauro_script/RepeatedMPCwithThermal.py`` (Const1:
    full relative-pose constraints) on the substitute 7-DOF arms (tools/make_centauro_urdf.py; the
    Centauro URDF is not in the reference).

    x = [q(14), T(14)], u = [qd(14), F_L(3), F_R(3)] (L183-241, 376-391).  Per node k:
    tau = ID(q, qd, 0) + J_LA^T [F_L; 0] + J_RA^T [F_R; 0] within +-joint_torque_lim (L341-350);
    force / moment equilibrium = 0 for every k (mixed rows, L238-253); relative position
    R_L^T (p_R - p_L) and orientation error of R_L R_R^T held at their x_0 values for k >= 1 (state
    rows; the reference chains node k to node k-1, L255-272, and repeats the orientation rows,
    L274-296 -- the same feasible set); T_{k+1} = a T_k + b (Ra (tau / ktau)^2 + qd^2 / Rh), T in
    [0, 80] (L122-123, 365-402); cost 100 |p_box - box_pos|^2 + 100 qd^T qd + 10 |F_L|^2 + 10 |F_R|^2
    (L353-356; the temperature term of L357-359 reads the numeric T_0, a constant).
    target_decimals: round the relative-orientation target as the MPC restart does
    (RepeatedMPCwithThermal.py:485-486); the relative-position rows keep x_0's exact value (they chain).
    """
    h = T / N
    a, b = thermal_coeffs(h)
    n = 14
    tl = np.asarray(CENT_TAU_LIM, float)
    return dict(
        name="centauro", family="centauro",
        urdf=["centauro_substitute_arm1.urdf", "centauro_substitute_arm2.urdf"], frames=["mass1_ee", "mass2_ee"],
        frame="mass1_ee", N=N, h=h, n=n, nf=6, thermal=True,
        q0=list(centauro_q0() if q0 is None else q0), qd0=list(np.zeros(n) if qd0 is None else qd0),
        T0=list(np.broadcast_to(np.asarray(T0, float), (n,))), T_lo=0.0, T_hi=80.0,
        q_lo=list(CENT_Q_LO), q_hi=list(CENT_Q_HI),
        qd_lo=list(-np.asarray(CENT_QD_LIM)), qd_hi=list(CENT_QD_LIM),
        tau_lo=np.tile(-tl, (N, 1)), tau_hi=np.tile(tl, (N, 1)),
        th_a=a, th_b=b, Ra=TH_RA, Rh=TH_RH, ktau=list(KTAU14), wT=0.0,
        box_mg=9.81 * mass, p_des=list(box_pos), w_box=100.0, w_qd=100.0, wF=10.0,
        target_decimals=target_decimals,
    )


def centauro_u_init(spec: dict) -> np.ndarray:
    """Initial controls of the first Centauro solve: qd = 0, each hand carrying half the box,
    F = (0, 0, m g / 2) -- the reference's sol0 (RepeatedMPCwithThermal.py:148-151)."""
    return np.r_[np.zeros(14), [0.0, 0.0, spec["box_mg"] / 2] * 2]


def box_shared_fatigue(N: int = 100, T0=60.0, T_hi: float = 80.0, budget_mean: float = 60.1, **kw) -> dict:
    """C3 "shared fatigue budget" (BASELINE config 3; build-defined, no reference counterpart):
    the dual-arm box of box_dual with the winding temperature of all 12 joints as state (the a8 recursion of
    Tmodel_library.py:9-41 / RepeatedMPCwithThermal.py:371-376, h = T / N, kτ = the first six entries of the
    reference table for each arm), T in [0, T_hi], and one budget row per node shared by both arms:
    sum_j T_j <= 12 budget_mean."""
    sp = box_dual(N=N, **kw)
    a, b = thermal_coeffs(sp["h"])
    sp.update(name="box_shared_fatigue", thermal=True, th_a=a, th_b=b, Ra=TH_RA, Rh=TH_RH,
              ktau=list(KTAU14[:6]) * 2, wT=0.0, T0=list(np.broadcast_to(np.asarray(T0, float), (12,))),
              T_lo=0.0, T_hi=T_hi, T_budget=12.0 * budget_mean)
    return sp
