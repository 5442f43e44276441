"""C-ABI tests that need no GPU: the library loads, exports every symbol declared
in include/mpcfatigue.h, and its host-side URDF ingestion reproduces the
oracle's (independent numpy) Pinocchio-semantics model exactly."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from mpc_fatigue_amd import _lib
from oracle import oracle as O
from oracle.urdf_np import load_urdf_file
from tests.conftest import ROOT, has_gpu

URDFS = ["pilz_robot_6DOF.urdf", "pilz_robot_3DOF.urdf", "pilz_robot_6DOF_first.urdf", "pilz_robot_6DOF_second.urdf"]


def header_functions():
    with open(os.path.join(ROOT, "include", "mpcfatigue.h")) as f:
        txt = f.read()
    return sorted(set(re.findall(r"\b(mf_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    L = _lib.lib()
    declared = header_functions()
    assert len(declared) >= 19
    for name in declared:
        assert hasattr(L, name), name
    assert set(_lib.EXPORTED_SYMBOLS) == set(declared)


@pytest.mark.parametrize("urdf", URDFS)
def test_urdf_ingestion_matches_oracle(urdf):
    path = os.path.join(ROOT, "mpc_fatigue_amd", "urdf", urdf)
    with open(path) as f:
        xml = f.read()
    m = _lib.Model(xml)
    ref = load_urdf_file(path)
    b = m.export()
    rb = O.model_blob(ref)
    assert b.shape == rb.shape
    np.testing.assert_allclose(b, rb, rtol=0, atol=1e-15)
    for name, fr in ref.frames.items():
        fid = m.frame_id(name)
        np.testing.assert_allclose(m.frame_record(fid), O.frame_arr(ref, name), atol=1e-15)


def test_unknown_frame_is_an_error_not_a_crash():
    xml = open(os.path.join(ROOT, "mpc_fatigue_amd", "urdf", "pilz_robot_6DOF.urdf")).read()
    m = _lib.Model(xml)
    with pytest.raises(_lib.MFError) as e:
        m.frame_id("no_such_link")
    assert e.value.code == -3 and "no_such_link" in str(e.value)


@pytest.mark.parametrize("xml,frag", [("<robot name='x'><link name='a'/>", "unterminated"),
                                      ("<robot><link name='a'/><link name='b'/></robot>", "root"),
                                      ("<notrobot/>", "robot")])
def test_bad_urdf_is_an_error(xml, frag):
    with pytest.raises(_lib.MFError) as e:
        _lib.Model(xml)
    assert e.value.code == -2 and frag in str(e.value)


@pytest.mark.skipif(has_gpu(), reason="checks the no-device failure mode")
def test_compute_without_device_fails_loudly():
    from mpc_fatigue_amd import pin
    xml = open(os.path.join(ROOT, "mpc_fatigue_amd", "urdf", "pilz_robot_6DOF.urdf")).read()
    idyn = pin.generate_inv_dyn(xml)
    with pytest.raises(_lib.MFError) as e:
        idyn(q=np.zeros(6), qdot=np.zeros(6), qddot=np.zeros(6))
    assert e.value.code == -4
