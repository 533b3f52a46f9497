"""Known answers of the oracle's box-box collider (oracle/collision.c) on tests/box_states.py's
configurations, from the geometry alone: a cube pressed 0.2 mm flat into a board touches it at its
four bottom corners, 0.2 mm deep, normal along z; tilted onto an edge, at the edge's two ends; onto a
corner, at that corner; two cubes crossing edge to edge, at one point on both edges with the normal
along their cross product; spawned 1 cm / 3.9 cm inside a shelf leg or 3 cm inside another cube, the
four corners of the overlap face at that depth along the axis of least penetration."""
import collections

import numpy as np
import pytest

from oracle import oracle as O

import box_states as BS


@pytest.fixture(scope="module")
def contacts(model):
    idx, st = BS.box_states(model)
    out = {}
    for case, b in idx.items():
        f = O.forward_fields({k: st[k][b] for k in O.STATE_KEYS}, ["ncon", "contact", "geom_xpos"], model=model)
        n = int(f["ncon"][0])
        out[case] = (f["contact"].reshape(n, 30), f["geom_xpos"].reshape(-1, 3), st["qpos"][b])
    return out


def _pair(model, c, a, b):
    ga, gb = model.geom_id(a), model.geom_id(b)
    sel = ((c[:, 27] == ga) & (c[:, 28] == gb)) | ((c[:, 27] == gb) & (c[:, 28] == ga))
    return c[sel]


def _cube_corners(qpos, adr):
    p, q = qpos[adr:adr + 3], qpos[adr + 3:adr + 7]
    R = BS._rot(q)
    s = np.array([[i, j, k] for i in (-1, 1) for j in (-1, 1) for k in (-1, 1)], float) * BS.H
    return p + s @ R.T


def test_rest_four_corners(model, contacts):
    c, _, q = contacts["rest"]
    k = _pair(model, c, "shelf_board2", "cube1_geom")
    assert len(k) == 4
    np.testing.assert_allclose(k[:, 12], -2e-4, atol=1e-12)
    np.testing.assert_allclose(np.abs(k[:, 3:6]), [[0, 0, 1]] * 4, atol=1e-12)
    a = int(model.jnt_qposadr[model.joint_id("cube1_joint")])
    low = _cube_corners(q, a)
    low = low[low[:, 2] < q[a + 2]]
    # contact points halfway between the surfaces: the corners lifted by half the depth
    got = sorted(map(tuple, np.round(k[:, :2], 9)))
    assert got == sorted(map(tuple, np.round(low[:, :2], 9)))
    np.testing.assert_allclose(k[:, 2], BS.BOARD2_TOP - 1e-4, atol=1e-12)


@pytest.mark.parametrize("case,n", [("tilt_edge", 2), ("tilt_corner", 1)])
def test_tilted_cube_touches_at_its_lowest_feature(model, contacts, case, n):
    c, _, q = contacts[case]
    k = _pair(model, c, "shelf_board2", "cube1_geom")
    assert len(k) == n
    np.testing.assert_allclose(k[:, 12], -5e-4, atol=1e-12)
    a = int(model.jnt_qposadr[model.joint_id("cube1_joint")])
    cr = _cube_corners(q, a)
    low = cr[np.argsort(cr[:, 2])[:n]]
    np.testing.assert_allclose(sorted(map(tuple, k[:, :2])), sorted(map(tuple, low[:, :2])), atol=1e-12)


def test_edge_edge_single_contact(model, contacts):
    c, _, q = contacts["edge_edge"]
    k = _pair(model, c, "cube1_geom", "cube2_geom")
    assert len(k) == 1
    np.testing.assert_allclose(k[0, 12], -5e-4, atol=1e-9)
    # lower edge along x, upper along (1, 1, 0)/sqrt2: the normal is their cross product, +-z
    np.testing.assert_allclose(np.abs(k[0, 3:6]), [0, 0, 1], atol=1e-9)
    np.testing.assert_allclose(k[0, :2], [1.45, -0.20], atol=1e-9)


@pytest.mark.parametrize("case,a,b,depth,axis", [("leg_1cm", "shelf_leg2", "cube1_geom", 0.01, 0),
                                                  ("leg_3p9cm", "shelf_leg2", "cube1_geom", 0.039, 0),
                                                  ("cube_cube", "cube1_geom", "cube2_geom", 0.03, 0),
                                                  ("table_leg_floor", "table_leg1", "cube3_geom", 0.04 - 2e-4, 2)])
def test_deep_spawn_overlap_face(model, contacts, case, a, b, depth, axis):
    """A deep spawn's contacts: four, at the least-penetration axis, each at the overlap depth."""
    c, _, _ = contacts[case]
    k = _pair(model, c, a, b)
    assert len(k) == 4, (case, len(k))
    np.testing.assert_allclose(k[:, 12], -depth, atol=1e-9)
    e = np.zeros(3)
    e[axis] = 1
    np.testing.assert_allclose(np.abs(k[:, 3:6]), [e] * 4, atol=1e-12)


def test_pads_pressed_contact_census(model, contacts):
    """Pads pressed 4 mm together: every pad-pad pair the oracle reports is box-box with 4 points."""
    c, _, _ = contacts["pads"]
    per = collections.Counter((int(x), int(y)) for x, y in c[:, 27:29])
    boxes = {p: n for p, n in per.items() if model.geom_type[p[0]] == 6 and model.geom_type[p[1]] == 6 and
             model.body_weldid[model.geom_bodyid[p[0]]] != 0}
    assert len(boxes) >= 10 and set(boxes.values()) <= {1, 2, 3, 4}
