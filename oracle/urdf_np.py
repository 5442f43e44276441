"""ORACLE (test infrastructure only) — URDF → kinematic-tree model, Pinocchio semantics.

This module is part of the parity *checker*.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it;
the product path (``mpc_fatigue_amd``) parses URDF in C++ inside
``libmpcfatigue.so`` and never touches this file.

It restates what the reference does at
``src/casadi_pinocchio_bridge.hpp:60-63`` (``urdf::parseURDF`` then
``pinocchio::urdf::buildModel(urdf, model, verbose=true)`` -- no root joint, i.e. a
fixed base):

* the root link (no parent joint) is attached to the universe; its inertia never
  moves and is irrelevant to RNEA;
* every revolute / prismatic joint becomes a 1-DoF joint whose placement in its
  parent joint frame is ``(placement of the parent link in the parent joint) *
  origin(joint)``;
* children of ``fixed`` joints are merged into the parent joint's body: their
  spatial inertia is appended with the accumulated placement, and their link name
  becomes a BODY frame with that placement (this matters for
  ``urdf/pilz_robot_3DOF.urdf`` whose joints 4-6 are fixed, and for the
  ``end_effector`` link of ``urdf/pilz_robot_6DOF_first.urdf:279-293``);
* urdfdom stores child joints in a name-sorted map, so a link's children are
  visited in joint-name order (depth first);
* URDF ``rpy`` is fixed-axis X-Y-Z: ``R = Rz(yaw) Ry(pitch) Rx(roll)``;
* the link inertia tensor given in the ``<inertial><origin rpy>`` frame is
  rotated into the link frame, ``I = R I_urdf R^T``, com = origin.xyz;
* joint ``damping`` / ``friction`` are parsed by urdfdom but ignored by
  ``pinocchio::rnea`` (they are not part of the model's dynamics).
"""
from __future__ import annotations

import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

import numpy as np


def rpy_to_R(r: float, p: float, y: float) -> np.ndarray:
    cr, sr = np.cos(r), np.sin(r)
    cp, sp = np.cos(p), np.sin(p)
    cy, sy = np.cos(y), np.sin(y)
    Rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def _vec(s: str | None, default=(0.0, 0.0, 0.0)) -> np.ndarray:
    if s is None:
        return np.array(default, dtype=float)
    return np.array([float(v) for v in s.split()], dtype=float)


@dataclass
class Inertia:
    """Spatial inertia about the frame origin: mass, com (3), rotational inertia at com."""

    m: float = 0.0
    c: np.ndarray = field(default_factory=lambda: np.zeros(3))
    Ic: np.ndarray = field(default_factory=lambda: np.zeros((3, 3)))

    def transformed(self, R: np.ndarray, t: np.ndarray) -> "Inertia":
        # express an inertia given in frame B in frame A, with A_M_B = (R, t)
        return Inertia(self.m, R @ self.c + t, R @ self.Ic @ R.T)

    def __add__(self, o: "Inertia") -> "Inertia":
        m = self.m + o.m
        if m <= 0.0:
            return Inertia()
        c = (self.m * self.c + o.m * o.c) / m

        def shift(I: Inertia) -> np.ndarray:
            d = I.c - c
            return I.Ic + I.m * (np.dot(d, d) * np.eye(3) - np.outer(d, d))

        return Inertia(m, c, shift(self) + shift(o))


@dataclass
class Joint:
    name: str
    parent: int                 # index of the parent movable joint, -1 = universe
    R: np.ndarray               # placement rotation in parent joint frame
    t: np.ndarray               # placement translation in parent joint frame
    axis: np.ndarray            # unit axis in the joint frame
    jtype: str                  # "revolute" | "prismatic"
    inertia: Inertia
    lower: float = -np.inf
    upper: float = np.inf
    effort: float = np.inf
    velocity: float = np.inf


@dataclass
class Frame:
    name: str
    parent: int                 # movable joint index, -1 = universe
    R: np.ndarray
    t: np.ndarray


@dataclass
class Model:
    joints: list[Joint]
    frames: dict[str, Frame]
    gravity: np.ndarray = field(default_factory=lambda: np.array([0.0, 0.0, -9.81]))

    @property
    def nq(self) -> int:
        return len(self.joints)

    nv = nq


def parse_urdf(urdf: str) -> Model:
    root = ET.fromstring(urdf)
    links: dict[str, ET.Element] = {l.get("name"): l for l in root.findall("link")}
    joints_xml = root.findall("joint")
    child_of: dict[str, list[ET.Element]] = {}
    has_parent: set[str] = set()
    for j in sorted(joints_xml, key=lambda e: e.get("name")):
        p = j.find("parent").get("link")
        c = j.find("child").get("link")
        child_of.setdefault(p, []).append(j)
        has_parent.add(c)
    roots = [n for n in links if n not in has_parent]
    if len(roots) != 1:
        raise ValueError(f"URDF must have exactly one root link, found {roots}")

    def link_inertia(name: str) -> Inertia:
        inl = links[name].find("inertial")
        if inl is None:
            return Inertia()
        o = inl.find("origin")
        xyz = _vec(o.get("xyz") if o is not None else None)
        rpy = _vec(o.get("rpy") if o is not None else None)
        m = float(inl.find("mass").get("value"))
        ie = inl.find("inertia")
        g = {k: float(ie.get(k, "0")) for k in ("ixx", "ixy", "ixz", "iyy", "iyz", "izz")}
        I = np.array([[g["ixx"], g["ixy"], g["ixz"]],
                      [g["ixy"], g["iyy"], g["iyz"]],
                      [g["ixz"], g["iyz"], g["izz"]]])
        R = rpy_to_R(*rpy)
        return Inertia(m, xyz.copy(), R @ I @ R.T)

    joints: list[Joint] = []
    frames: dict[str, Frame] = {}
    frames[roots[0]] = Frame(roots[0], -1, np.eye(3), np.zeros(3))

    def visit(link: str, pj: int, R_l: np.ndarray, t_l: np.ndarray) -> None:
        # (R_l, t_l): placement of `link` in the frame of movable joint `pj`
        for j in child_of.get(link, []):
            o = j.find("origin")
            xyz = _vec(o.get("xyz") if o is not None else None)
            rpy = _vec(o.get("rpy") if o is not None else None)
            Rj = R_l @ rpy_to_R(*rpy)
            tj = R_l @ xyz + t_l
            child = j.find("child").get("link")
            jt = j.get("type")
            if jt == "fixed":
                frames.setdefault(j.get("name"), Frame(j.get("name"), pj, Rj, tj))
                frames.setdefault(child, Frame(child, pj, Rj, tj))
                if pj >= 0:
                    joints[pj].inertia = joints[pj].inertia + link_inertia(child).transformed(Rj, tj)
                visit(child, pj, Rj, tj)
            elif jt in ("revolute", "prismatic", "continuous"):
                if jt == "continuous":
                    # pinocchio models continuous joints with nq=2 (cos, sin); no
                    # reference URDF uses one, so it is rejected rather than guessed.
                    raise ValueError("continuous joints are not supported")
                a = j.find("axis")
                axis = _vec(a.get("xyz") if a is not None else None, (1.0, 0.0, 0.0))
                axis = axis / np.linalg.norm(axis)
                lim = j.find("limit")
                kw = {}
                if lim is not None:
                    for k in ("lower", "upper", "effort", "velocity"):
                        if lim.get(k) is not None:
                            kw[k] = float(lim.get(k))
                idx = len(joints)
                joints.append(Joint(j.get("name"), pj, Rj, tj, axis, jt,
                                    link_inertia(child), **kw))
                frames.setdefault(j.get("name"), Frame(j.get("name"), idx, np.eye(3), np.zeros(3)))
                frames.setdefault(child, Frame(child, idx, np.eye(3), np.zeros(3)))
                visit(child, idx, np.eye(3), np.zeros(3))
            else:
                raise ValueError(f"unsupported joint type {jt}")

    visit(roots[0], -1, np.eye(3), np.zeros(3))
    return Model(joints, frames)


def load_urdf_file(path: str) -> Model:
    with open(path) as f:
        return parse_urdf(f.read())
