"""Dump k_bk_compare's inputs and both factors (tests/test_gpu_bk.py's blocks) to gpurun_out/bk_probe.npz."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from mpc_fatigue_amd import _lib  # noqa: E402
from test_gpu_bk import M, _blocks  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 600
K = _blocks(np.random.default_rng(7), n)
R = np.zeros_like(K)
W = np.zeros_like(K)
meta = np.zeros((n, 2 * M + 6), np.int32)
_lib.check(_lib.lib().mf_debug_bk_compare(_lib.dptr(K), n, 0, _lib.dptr(R), _lib.dptr(W), _lib.iptr(meta)))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "bk_probe.npz"), K=K, R=R, W=W, meta=meta)
print("ok")
