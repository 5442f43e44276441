"""Diagnostic (GPU): IPOPT-mode C2 device solutions against the oracle's -- the 64-horizon headline fixture, the
16-horizon spread and the reference's 15 Nm instance -- with tests/c2check.compare's measures, no assertions."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    torch.cuda.init()
    from mpc_fatigue_amd import problems as PR
    from mpc_fatigue_amd.gocp import GOCP
    from oracle import generic as G
    from tests import c2check
    kw = dict(init_zero=True, filter=True, bound_relax=1e-8, max_iter=3000, max_soc=4)
    fx = np.load(os.path.join(ROOT, "tests", "golden", "c2_headline_ipopt_oracle.npz"))
    Q0, LR = fx["q0"], fx["line_ref"]
    g = GOCP(PR.pilz6_bench(N=100))
    r = g.solve(x0=Q0, line_ref=LR, **kw)
    rows = []
    for b in range(Q0.shape[0]):
        spec = PR.pilz6_bench(N=100, q0=Q0[b], line_ref=LR[b])
        c = c2check.compare(g, b, spec, r.w[b], float(r.obj[b]), fx["w"][b], float(fx["obj"][b]))
        c.update(b=b, st=(int(r.status[b]), int(fx["status"][b])), it=(int(r.iters[b]), int(fx["iters"][b])),
                 counters=g.counters(b))
        rows.append(c)
        print(json.dumps(c), flush=True)
    kinds = {k: sum(1 for c in rows if c["kind"] == k) for k in ("same", "mirror", "neighbour")}
    print("kinds", kinds, "max E0", max(c["E0"] for c in rows), "max dobj", max(c["dobj"] for c in rows),
          "max inner dq same/mirror", max([c["inner_dq"] for c in rows if c["kind"] != "neighbour"] + [0]), flush=True)
    for N in (60, 100):
        sp = PR.pilz6_force(N=N)
        g2 = GOCP(sp)
        r2 = g2.solve(x0=np.asarray(sp["q0"])[None], **kw)
        print("15Nm", N, "device", int(r2.status[0]), int(r2.iters[0]), g2.counters(0), flush=True)


if __name__ == "__main__":
    main()
