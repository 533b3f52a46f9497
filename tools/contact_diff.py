"""Diagnostic: per geom-pair contact counts, GPU forward_debug vs oracle, on fresh reset states;
plus the contact-count histogram of the bench (C3) workload.  usage: python tools/contact_diff.py"""
import os
import sys
from collections import Counter

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd"), os.path.join(ROOT, "tests")]
from oracle import oracle as O  # noqa: E402
from pnp_amd import _lib  # noqa: E402
from pnp_amd.engine import get_engine  # noqa: E402
import physics_states as PS  # noqa: E402
import bench  # noqa: E402

D = _lib.DBG


def dev(st, dt):
    return {k: torch.as_tensor(v.astype(np.int32) if k == "warn" else np.ascontiguousarray(v),
                               dtype=torch.int32 if k == "warn" else dt, device="cuda").contiguous()
            for k, v in st.items()}


def main():
    eng = get_engine()
    m = eng.model
    st = PS.reset_states(4, seed=7)
    dbg = eng.forward_debug(dev(st, torch.float64)).cpu().numpy()
    for b in range(4):
        f = O.forward_fields({k: st[k][b] for k in O.STATE_KEYS}, ["contact", "ncon"])
        n = int(f["ncon"][0])
        c = f["contact"].reshape(n, 30)
        ref = Counter((m.names_geom[int(r[27])], m.names_geom[int(r[28])]) for r in c)
        ng = int(dbg[b][D["COUNTS"]])
        gq = [dbg[b][D["CON"] + 16 * i: D["CON"] + 16 * (i + 1)] for i in range(ng)]
        gpu = Counter((m.names_geom[int(q[13])], m.names_geom[int(q[14])]) for q in gq)
        print(f"env {b}: gpu {ng} ref {n}")
        for k in sorted(set(ref) | set(gpu), key=str):
            if ref[k] != gpu[k]:
                print("   ", k, "gpu", gpu[k], "ref", ref[k])
                for r in c:
                    if (m.names_geom[int(r[27])], m.names_geom[int(r[28])]) == k:
                        print("      ref pos", np.round(r[:3], 6), "dist", r[12])
                for q in gq:
                    if (m.names_geom[int(q[13])], m.names_geom[int(q[14])]) == k:
                        print("      gpu pos", np.round(q[:3], 6), "dist", q[12])
    # bench workload contact counts
    st, ctrl = bench.step_inputs(eng, m, 0, 4096)
    for i in range(4):
        st["ctrl"] = ctrl[i]
        eng.step(st, 25)
    d = eng.forward_debug(st).cpu().numpy()
    nc = d[:, D["COUNTS"]].astype(int)
    ne = d[:, D["COUNTS"] + 1].astype(int)
    print("bench ncon hist", np.bincount(nc).nonzero()[0].tolist(), "max", nc.max(), "mean", nc.mean(),
          "nefc max", ne.max(), "warn", np.bincount(st["warn"].cpu().numpy()).tolist())
    w = np.nonzero(st["warn"].cpu().numpy())[0][:3]
    for b in w:
        ng = int(d[b][D["COUNTS"]])
        gq = [d[b][D["CON"] + 16 * i: D["CON"] + 16 * (i + 1)] for i in range(min(ng, 28))]
        print(" env", b, Counter((m.names_geom[int(q[13])], m.names_geom[int(q[14])]) for q in gq).most_common(12))


if __name__ == "__main__":
    main()
