"""Solution CSV I/O in the reference format (Box_Pilz_6DOF.py:464-477) on the reference's own
committed solutions (tests/golden, copies of plotter/*solution.csv), CPU only."""
import os

import numpy as np
import pytest

from mpc_fatigue_amd.solution_io import read_solution_csv, write_solution_csv
from tests.conftest import GOLDEN


@pytest.mark.parametrize("name,N", [("G1_box_N50", 50), ("G2_box_N80", 80)])
def test_reference_csv_roundtrip(tmp_path, name, N):
    src = os.path.join(GOLDEN, f"{name}_solution.csv")
    sol = read_solution_csv(src)
    assert sol.size == 12 + 30 * N          # Box_Pilz_6DOF.py layout: (q, qd, F_L, F_R) x N + q_N
    np.testing.assert_array_equal(sol, np.loadtxt(src, delimiter=",").ravel())
    out = tmp_path / "solution.csv"
    write_solution_csv(str(out), sol)
    np.testing.assert_array_equal(read_solution_csv(str(out)), sol)   # bit-exact (repr)
    assert len(open(out).read().strip().splitlines()) == 1             # one row, as writerow(sol)
