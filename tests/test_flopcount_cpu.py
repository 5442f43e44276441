"""The op-counted FP64 work per node evaluation that bench.py's roofline.fp64 divides by the
eval phase's time: recounted from the device templates (tests/native/flopcount.cpp, counting scalars) and
compared with the committed profiles/fp64_opcount.json, so the figure cannot drift from the code."""
import json
import os
import sys

from tests.conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_fp64_opcount_matches_committed():
    import flopcount
    rec = flopcount.count()
    with open(os.path.join(ROOT, "profiles", "fp64_opcount.json")) as f:
        old = json.load(f)
    assert rec["fp64_ops_per_node_eval"] == old["fp64_ops_per_node_eval"]
    q, qd = rec["q_lanes"], rec["qd_lanes"]
    # the split sweep runs plain FP64 below joint v: each later q direction costs less; the qd class is uniform
    assert all(a > b for a, b in zip(q, q[1:])) and len(set(qd)) == 1
    assert q[-1] > qd[0]
    assert 100_000 < rec["fp64_ops_per_node_eval"] < 200_000
