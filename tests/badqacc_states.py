"""cube3 contact fixtures for the targeted BADQACC probe (test helper; tools/badqacc_probe.py,
tests/test_badqacc_probe_cpu.py, tests/test_boxbox_gpu.py): the situations the box-box
restatement's assumptions A1 / A3 / A6 (oracle/collision.c above box_box) leave open, around
board1 where MUJOCO_LOG.TXT:1-8's BADQACC resets hit cube3 (shelf_pnp.xml:45-52,75).  Randomised
with a fixed seed and kept only where cube3 touches what the family names, at most 5 mm deep:
  par_edge   cube3 at board1's front-top edge (x 1.35, z 0.41), rotated about y (0 .. 90 deg: edge or
             face towards the corner) and then by a small angle (1e-8 .. 1e-2 rad, log-uniform,
             random axis), so that its edges and the board's are parallel to within that angle
  leg_wedge  cube3 tilted up to 45 deg on board1 against shelf_leg2 (x 1.35-1.39, y 0.46-0.50)
  cube_edge  cube1 moved onto board1 onto cube3's top edge, edge on edge, within 1e-8 .. 1e-2 rad
             of parallel
"""
from __future__ import annotations

import numpy as np

import box_states as BS
import physics_states as PS

FAMILIES = ("par_edge", "leg_wedge", "cube_edge")
H = 0.02


def _rand_axis(rng):
    a = rng.normal(size=3)
    return a / np.linalg.norm(a)


def touches_cube3(model, con_row):
    g = model.geom_id("cube3_geom")
    return int(con_row[27]) == g or int(con_row[28]) == g


def _contacts(model, st, b):
    from oracle import oracle as O
    f = O.forward_fields({k: st[k][b] for k in O.STATE_KEYS}, ["ncon", "contact"], model=model)
    n = int(f["ncon"][0])
    return f["contact"].reshape(n, 30)


def family_states(model, fam, n, seed=17, max_tries=40):
    """n states of family `fam` (and a short description of each)."""
    m = model
    rng = np.random.default_rng(seed + FAMILIES.index(fam))
    a3 = int(m.jnt_qposadr[m.joint_id("cube3_joint")])
    a1 = int(m.jnt_qposadr[m.joint_id("cube1_joint")])
    g3, gb1, gl2, gc1 = (m.geom_id(x) for x in ("cube3_geom", "shelf_board1", "shelf_leg2", "cube1_geom"))
    out = PS.reset_states(n, seed=13, model=m)
    out["qpos"][:, 7:9] = 0.004
    info = []
    for b in range(n):
        for _ in range(max_tries * 100):
            st = {k: v[b:b + 1].copy() for k, v in out.items()}
            th = 10 ** rng.uniform(-8, -2)
            if fam == "par_edge":
                q = BS._qmul(BS._quat(_rand_axis(rng), th), BS._quat([0, 1, 0], rng.uniform(0, np.pi / 2)))
                c = [1.35 + rng.uniform(-0.03, 0.0), rng.uniform(-0.1, 0.1), 0.41 + rng.uniform(0.0, 0.03)]
                st["qpos"][0, a3:a3 + 3], st["qpos"][0, a3 + 3:a3 + 7] = c, q
                want = {(g3, gb1)}
                desc = f"theta {th:.1e}"
            elif fam == "leg_wedge":
                th = rng.uniform(0, np.pi / 4)
                q = BS._quat(_rand_axis(rng), th)
                c = [rng.uniform(1.36, 1.42), rng.uniform(0.40, 0.46), 0.41 + rng.uniform(0.012, 0.035)]
                st["qpos"][0, a3:a3 + 3], st["qpos"][0, a3 + 3:a3 + 7] = c, q
                want = {(g3, gb1), (g3, gl2)}
                desc = f"tilt {np.degrees(th):.1f} deg"
            else:
                c3 = np.array([1.45, 0.0, 0.41 + H])
                st["qpos"][0, a3:a3 + 3], st["qpos"][0, a3 + 3:a3 + 7] = c3, [1, 0, 0, 0]
                q = BS._qmul(BS._quat(_rand_axis(rng), th), BS._quat([0, 1, 0], np.pi / 4))
                c = c3 + [rng.uniform(-H, H), rng.uniform(-0.03, 0.03), H + H * np.sqrt(2) + rng.uniform(-0.004, 0.0)]
                st["qpos"][0, a1:a1 + 3], st["qpos"][0, a1 + 3:a1 + 7] = c, q
                want = {(g3, gc1)}
                desc = f"theta {th:.1e}"
            con = _contacts(m, st, 0)
            pairs = {tuple(sorted((int(x[27]), int(x[28])))) for x in con if touches_cube3(m, x)}
            deep = min([x[12] for x in con if touches_cube3(m, x)] + [0.0])
            if all(tuple(sorted(w)) in pairs for w in want) and deep > -0.005:
                for k in out:
                    out[k][b] = st[k][0]
                info.append(desc + f", depth {-deep * 1e3:.2f} mm")
                break
        else:
            raise RuntimeError(f"{fam}: no state found for slot {b}")
    return out, info
