"""Targeted BADQACC probe (CPU oracle).  MUJOCO_LOG.TXT:1-8 records three
BADQACC resets on cube3's angular dofs (24 / 25) in real MuJoCo; the round-5 census of the engine's
own workload found none.  This probe builds cube3 in the contact situations the box-box restatement's
assumptions leave open (oracle/collision.c A1 / A3 / A6) and steps them through the oracle with each
assumption changed (oracle.set_boxbox_variant bits: 1 near-parallel edge axes kept down to 1e-12,
2 round 5's edge tie margin, 4 no parallel-line guard on the edge closest points, 8 the edge contact
on box 2's edge), reporting per family and variant the largest |qacc| on cube3's dofs, the farthest
contact from cube3's centre (a lever arm on its angular dofs) and any non-finite normal or frame.
Families (cube3 on board1, shelf_pnp.xml:45-52,75; randomised, fixed seed):
  par_edge   cube3 on an edge (45 deg about y) lying on board1's front-top edge, its edge rotated by
             a small angle (1e-8 .. 1e-2 rad, log-uniform, random axis) away from parallel, pressed
             0 .. 5 mm into the corner
  leg_wedge  cube3 tilted (0 .. 45 deg) between board1's top and shelf_leg2, pressed 0 .. 5 mm into both
  cube_edge  cube1 moved onto board1 next to cube3, the two cubes' edges nearly parallel and touching
usage: python tools/badqacc_probe.py [n_per_family] [out.npz]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd"), os.path.join(ROOT, "tests")]
from oracle import oracle as O  # noqa: E402
from pnp_amd.model import load_model  # noqa: E402
import badqacc_states as BQ  # noqa: E402

VARIANTS = (0, 1, 2, 4, 8, 1 | 2 | 4 | 8)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    out = sys.argv[2] if len(sys.argv) > 2 else None
    m = load_model()
    d3 = int(m.jnt_dofadr[m.joint_id("cube3_joint")])
    a3 = int(m.jnt_qposadr[m.joint_id("cube3_joint")])
    rec = {}
    for fam in BQ.FAMILIES:
        st, info = BQ.family_states(m, fam, n, seed=17)
        for v in VARIANTS:
            O.set_boxbox_variant(v)
            qa, lever, bad, ncon = np.zeros(n), np.zeros(n), 0, np.zeros(n, int)
            for b in range(n):
                row = {k: st[k][b] for k in O.STATE_KEYS}
                f = O.forward_fields(row, ["qacc", "ncon", "contact"], model=m)
                k = int(f["ncon"][0])
                con = f["contact"].reshape(k, 30)
                qa[b] = np.abs(f["qacc"][d3:d3 + 6]).max() if np.isfinite(f["qacc"]).all() else np.inf
                c3 = st["qpos"][b, a3:a3 + 3]
                mine = [i for i in range(k) if BQ.touches_cube3(m, con[i])]
                ncon[b] = len(mine)
                lever[b] = max([np.linalg.norm(con[i, 0:3] - c3) for i in mine] + [0.0])
                bad += int(not np.isfinite(con[:, 0:12]).all())
            rec[(fam, v)] = (qa, lever, ncon)
            w = int(np.argmax(qa))
            print(f"{fam:10s} variant {v:2d}: max |qacc| cube3 {qa.max():.3e} (state {w}: {info[w]}), over 1e10 "
                  f"{int((qa > 1e10).sum())} of {n}; farthest cube3 contact {lever.max():.3f} m; non-finite contacts "
                  f"{bad}", flush=True)
    O.set_boxbox_variant(0)
    if out:
        np.savez(out, **{f"{f}_{v}_{k}": a for (f, v), t in rec.items() for k, a in zip(("qacc", "lever", "ncon"), t)})


if __name__ == "__main__":
    main()
