"""How the bench's C3 states evolve over its timed steps: per checkpoint, the launch time and the
contact population (mean ncon / nefc, share of contacts on mesh geoms).  Exploratory (prints a
report).  usage: python tools/bench_drift.py [B] [steps]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
import bench  # noqa: E402
from pnp_amd import _lib  # noqa: E402
from pnp_amd.engine import get_engine  # noqa: E402

D = _lib.DBG
MESH = 7   # mjGEOM_MESH


def census(eng, st):
    m = eng.model
    dbg = eng.forward_debug(st).cpu().numpy()
    ncon = dbg[:, D["COUNTS"]].astype(int)
    nefc = dbg[:, D["COUNTS"] + 1].astype(int)
    mesh = total = 0
    pairs = {}
    for b in range(dbg.shape[0]):
        for c in range(ncon[b]):
            rec = dbg[b, D["CON"] + c * D["CON_STRIDE"]:D["CON"] + (c + 1) * D["CON_STRIDE"]]
            g1, g2 = int(rec[13]), int(rec[14])
            total += 1
            if m.geom_type[g1] == MESH or m.geom_type[g2] == MESH:
                mesh += 1
                key = (m.names_geom[g1], m.names_geom[g2])
                pairs[key] = pairs.get(key, 0) + 1
    top = sorted(pairs.items(), key=lambda kv: -kv[1])[:6]
    return ncon.mean(), nefc.mean(), mesh / max(total, 1), (ncon >= 48).mean(), top


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    eng = get_engine()
    st, ctrl = bench.step_inputs(eng, eng.model, 0, B)
    for i in range(steps + 1):
        if i % 10 == 0:
            nc, ne, fm, full, top = census(eng, st)
            print(f"step {i:3d}: ncon {nc:5.2f} nefc {ne:6.1f} mesh-contact share {fm:.3f} "
                  f"capped {full:.3f} warn {int(st['warn'].max())}", flush=True)
            cl = {k: v.clone() for k, v in st.items()}
            prof = eng.step_profile(cl, bench.NSUB).cpu().numpy().astype(np.float64) / bench.NSUB
            print("      cycles/sub-step " + " ".join(f"{n}={prof[:, j].mean():.0f}" for j, n in enumerate(eng.STAGES)
                                               if prof[:, j].mean() > 15000))
            for k, v in top:
                print(f"      {k[0]:>20s} - {k[1]:<20s} {v / B:.3f}/env")
        st["ctrl"] = ctrl[i % bench.NCTRL]
        torch.cuda.synchronize()
        t = time.time()
        eng.step(st, bench.NSUB)
        torch.cuda.synchronize()
        if i % 10 == 0:
            print(f"          launch {1e3 * (time.time() - t):.2f} ms", flush=True)


if __name__ == "__main__":
    main()
