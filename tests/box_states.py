"""Box-contact fixture states (test helper): one env per configuration, every other body at the
reference's reset (neutral arm, mocap home, cubes on their boards).  The configurations are the
box-box cases a box collider has to get right -- a cube resting flat, tilted onto an edge and onto a
corner, two cubes crossing edge to edge, the closed fingers' pad boxes pressed together -- and the
deep spawns the reference's reset random walk produces (envs/panda_env.py:146-158, tools/
badqacc_census.py): a cube inside a shelf leg (1 and 3.9 cm), inside a table leg on the floor,
two cubes overlapping, a cube half over a board edge.
"""
from __future__ import annotations

import numpy as np

import physics_states as PS

BOARD2_TOP = 0.71   # shelf_pnp.xml:51 (board2 z 0.7, half-height 0.01)
H = 0.02            # cube half-size


def _quat(axis, ang):
    a = np.asarray(axis, np.float64)
    a = a / np.linalg.norm(a)
    return np.concatenate([[np.cos(ang / 2)], a * np.sin(ang / 2)])


def _qmul(p, q):
    w0, x0, y0, z0 = p
    w1, x1, y1, z1 = q
    return np.array([w0 * w1 - x0 * x1 - y0 * y1 - z0 * z1, w0 * x1 + x0 * w1 + y0 * z1 - z0 * y1,
                     w0 * y1 + y0 * w1 + z0 * x1 - x0 * z1, w0 * z1 + z0 * w1 + x0 * y1 - y0 * x1])


def _rot(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def _low(q):
    """How far the cube's lowest point lies below its centre at orientation q."""
    return float(np.abs(_rot(q)[2]).sum() * H)


CASES = ("rest", "tilt_edge", "tilt_corner", "edge_edge", "pads", "leg_1cm", "leg_3p9cm", "cube_cube",
         "table_leg_floor", "board_edge")


def box_states(model, cases=CASES):
    """{case: env index} and the batch (one env per case)."""
    m = model
    n = len(cases)
    st = PS.reset_states(n, seed=13, model=m)
    st["qpos"][:, 7:9] = 0.004          # fingers 4 mm open (off the closed-pad knife edge), but "pads"
    adr = {c: int(m.jnt_qposadr[m.joint_id(f"{c}_joint")]) for c in ("cube1", "cube2", "cube3")}

    def put(b, cube, pos, q=(1.0, 0.0, 0.0, 0.0)):
        a = adr[cube]
        st["qpos"][b, a:a + 3] = pos
        st["qpos"][b, a + 3:a + 7] = q

    for b, c in enumerate(cases):
        # cube2 / cube3 out of cube1's way on their own boards unless the case moves them
        if c == "rest":
            put(b, "cube1", [1.45, 0.10, BOARD2_TOP + H - 2e-4])
        elif c == "tilt_edge":
            q = _quat([1, 0, 0], np.radians(30))
            put(b, "cube1", [1.45, 0.05, BOARD2_TOP + _low(q) - 5e-4], q)
        elif c == "tilt_corner":
            q = _quat([1, 1, 0], np.radians(35))
            put(b, "cube1", [1.45, -0.05, BOARD2_TOP + _low(q) - 5e-4], q)
        elif c == "edge_edge":
            ql = _quat([1, 0, 0], np.radians(45))                       # lower cube on an edge, top edge along x
            zl = BOARD2_TOP + _low(ql) - 2e-4
            put(b, "cube1", [1.45, -0.20, zl], ql)
            qu = _qmul(_quat([0, 0, 1], np.radians(45)), _quat([1, 0, 0], np.radians(45)))   # bottom edge along (1,1,0)
            put(b, "cube2", [1.45, -0.20, zl + H * np.sqrt(2) + _low(qu) - 5e-4], qu)
        elif c == "pads":
            st["qpos"][b, 7:9] = -0.002                                  # pad boxes pressed 4 mm together
            st["ctrl"][b, -2:] = 0.0
        elif c == "leg_1cm":
            put(b, "cube1", [1.40, 0.47, BOARD2_TOP + H - 2e-4])         # shelf_leg2: x in [1.35, 1.39]
        elif c == "leg_3p9cm":
            put(b, "cube1", [1.371, 0.48, BOARD2_TOP + H - 2e-4])
        elif c == "cube_cube":
            put(b, "cube1", [1.45, 0.20, BOARD2_TOP + H - 2e-4])
            put(b, "cube2", [1.46, 0.205, BOARD2_TOP + H - 2e-4])       # 3 cm / 3.5 cm overlap, axis aligned
        elif c == "table_leg_floor":
            put(b, "cube3", [1.07, 0.37, H - 2e-4])                     # table_leg1: [1.04, 1.10] x [0.34, 0.40]
        elif c == "board_edge":
            put(b, "cube1", [1.45, 0.505, BOARD2_TOP + H - 2e-4])       # half over board2's edge (|y| <= 0.5)
        else:
            raise KeyError(c)
    return {c: i for i, c in enumerate(cases)}, st
