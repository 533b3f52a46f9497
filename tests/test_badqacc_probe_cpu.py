"""Targeted BADQACC probe on the CPU oracle (tools/badqacc_probe.py runs
the larger sweep): cube3 in the contact situations the box-box restatement's assumptions leave open
(tests/badqacc_states.py: near-parallel edges on board1's front edge, wedged between board1 and
shelf_leg2, cube1's edge on cube3's edge), stepped through the oracle with the restatement (variant
0) and with every probed assumption changed at once (15: near-parallel edge axes kept to 1e-12, round
5's edge tie margin, no parallel-line guard on the edge closest points, the edge contact on box 2's
edge).  Real MuJoCo reset cube3 for |qacc| > 1e10 three times (MUJOCO_LOG.TXT:1-8); here no state
comes near it: cube3's accelerations stay below 1e4, every contact lies on the cube (within its
half-diagonal of its centre: no far edge-edge point, no lever arm) and every normal and frame is
finite -- for the changed assumptions too, because near-parallel edges never win the axis
selection (a face axis is never worse there).  Measured (tools/badqacc_probe.py 1000): largest
|qacc| 4.9e2 (par_edge), 8.5e2 (leg_wedge), 1.2e1 (cube_edge), farthest contact 0.035 m."""
import numpy as np
import pytest

from oracle import oracle as O

import badqacc_states as BQ


@pytest.mark.parametrize("fam", BQ.FAMILIES)
def test_probe_family_stays_finite_and_local(model, fam):
    m = model
    d3 = int(m.jnt_dofadr[m.joint_id("cube3_joint")])
    a3 = int(m.jnt_qposadr[m.joint_id("cube3_joint")])
    st, info = BQ.family_states(m, fam, 40, seed=17)
    try:
        for v in (0, 15):
            O.set_boxbox_variant(v)
            worst = 0.0
            for b in range(40):
                f = O.forward_fields({k: st[k][b] for k in O.STATE_KEYS}, ["qacc", "ncon", "contact"], model=m)
                con = f["contact"].reshape(int(f["ncon"][0]), 30)
                assert np.isfinite(con[:, 0:13]).all() and np.isfinite(f["qacc"]).all(), (fam, v, b, info[b])
                qa = float(np.abs(f["qacc"][d3:d3 + 6]).max())
                worst = max(worst, qa)
                assert qa < 1e4, (fam, v, b, info[b], qa)
                c3 = st["qpos"][b, a3:a3 + 3]
                for row in con:
                    if BQ.touches_cube3(m, row):
                        assert np.linalg.norm(row[0:3] - c3) <= BQ.H * np.sqrt(3) + 0.005, (fam, v, b, row[0:3], c3)
            print(f"{fam} variant {v}: max |qacc| on cube3 {worst:.3e}")
    finally:
        O.set_boxbox_variant(0)
