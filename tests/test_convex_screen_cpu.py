"""The compact tier's convex screen (csrc/collide_dev.h c_hull_beyond / c_convex_screen): a pair
it proves separated has no MPR contact.  Restated here in float32 numpy over the oracle's geom
frames (rounded to fp32, as the fp32 kernel sees them) and checked against the oracle's MPR
(oracle/convex.c through convex_probe) on every sphere / box / mesh -- mesh geom pair of settled,
reset and randomly posed arm states: whenever the screen says separated, MPR reports no
intersection; and the screen proves most far-apart pairs (it is useful, not vacuous)."""
import numpy as np
import pytest

from oracle import oracle as O
import physics_states as PS


def _aabb(m, g):
    t = int(m.geom_type[g])
    if t == 2:
        return np.zeros(3), np.full(3, float(m.geom_size[g][0]) if np.ndim(m.geom_size[g]) else float(m.geom_size[3 * g]))
    size = np.asarray(m.geom_size).reshape(-1, 3)[g]
    if t == 6:
        return np.zeros(3), size.astype(np.float64)
    mesh = int(m.geom_dataid[g])
    V = np.asarray(m.mesh_vert).reshape(-1, 3)[int(m.mesh_vertadr[mesh]):int(m.mesh_vertadr[mesh]) + int(m.mesh_vertnum[mesh])]
    lo, hi = V.min(0), V.max(0)
    return 0.5 * (lo + hi), 0.5 * (hi - lo)


def _hull_beyond(m, gx, gm_, gm, gb, margin):
    """float32 restatement of c_hull_beyond: mesh gm's vertices beyond a face of gb's box (or the
    sphere's plane) by margin + 1e-5."""
    f = np.float32
    mesh = int(m.geom_dataid[gm])
    n = int(m.mesh_vertnum[mesh])
    if n > 192:
        return False
    V = np.asarray(m.mesh_vert).reshape(-1, 3)[int(m.mesh_vertadr[mesh]):int(m.mesh_vertadr[mesh]) + n].astype(f)
    Rm, Rb = gm_[gm].reshape(3, 3).astype(f), gm_[gb].reshape(3, 3).astype(f)
    d = (gx[gm].astype(f)[None, :] + V @ Rm.T) - gx[gb].astype(f)[None, :]
    cb, hb = (a.astype(f) for a in _aabb(m, gb))
    mg = f(margin) + f(1e-5)
    if int(m.geom_type[gb]) == 2:
        cm, _ = _aabb(m, gm)
        w = gx[gm].astype(f) + Rm @ cm.astype(f) - gx[gb].astype(f)
        nn = f(w @ w)
        if not nn > f(1e-12):
            return False
        u = w / np.sqrt(nn)
        r = f(np.asarray(m.geom_size).reshape(-1, 3)[gb][0])
        return bool((d @ u).min() > r + mg)
    q = d @ Rb - cb[None, :]
    h = hb + mg
    return bool(((q.min(0) > h) | (q.max(0) < -h)).any())


def _screen(m, gx, gmat, g1, g2, margin):
    if _hull_beyond(m, gx, gmat, g2, g1, margin):
        return True
    return int(m.geom_type[g1]) == 7 and _hull_beyond(m, gx, gmat, g1, g2, margin)


def _states(model):
    """Arm poses swung through the scene, plus states with convex contacts: the hand pushed into
    cube1 and the fingers closed past each other (pads pressed)."""
    st = PS.reset_states(8, seed=3, model=model)
    rng = np.random.default_rng(4)
    st["qpos"][:4, :7] += rng.normal(size=(4, 7)) * 0.6     # arm swung through the scene
    st["qpos"][:, 7:9] = rng.uniform(-0.002, 0.04, size=(8, 2))
    sx, _ = O.site_kinematics(st["qpos"][4:6], model=model)
    a = int(model.jnt_qposadr[model.joint_id("cube1_joint")])
    st["qpos"][4:6, a:a + 3] = sx[:, model.site_id("ee_center_site")] + [0.0, 0.0, 0.075]
    st["qpos"][6:, 7:9] = -0.003
    return st


def test_screen_never_hides_an_mpr_contact(model):
    st = _states(model)
    t = np.asarray(model.geom_type)
    coll = (np.asarray(model.geom_contype) != 0) | (np.asarray(model.geom_conaffinity) != 0)
    has = (t != 7) | (np.asarray(model.geom_dataid) >= 0)   # (visual meshes carry no vertices)
    meshes = np.where((t == 7) & coll & has)[0]
    others = np.where(((t == 2) | (t == 6) | (t == 7)) & coll & has)[0]
    body = np.asarray(model.geom_bodyid)
    weld = np.asarray(model.body_weldid)
    par = np.asarray(model.body_parentid)
    ct, ca = np.asarray(model.geom_contype), np.asarray(model.geom_conaffinity)

    def is_pair(g1, g2):   # the engine's pair filter (phys_host.cpp: MuJoCo 2.3.3 mj_collision)
        if not (ct[g1] & ca[g2]) and not (ct[g2] & ca[g1]):
            return False
        w1, w2 = weld[body[g1]], weld[body[g2]]
        if w1 == w2:
            return False
        p1, p2 = weld[par[w1]], weld[par[w2]]
        return not (w1 != 0 and w2 != 0 and (w1 == p2 or w2 == p1))
    margin = 0.0
    proven = checked = hits = 0
    for b in range(st["qpos"].shape[0]):
        row = {k: st[k][b] for k in O.STATE_KEYS}
        _, gx, gmat = O.convex_probe(row, int(meshes[0]), int(meshes[1]), model=model)
        gx32, gm32 = gx.astype(np.float32).astype(np.float64), gmat.astype(np.float32).astype(np.float64)
        for g2 in meshes:
            for g1 in others:
                # (the engine's convex pairs put the mesh second: any index order)
                if g1 == g2 or (int(model.geom_type[g1]) == 7 and g1 > g2) or not is_pair(int(g1), int(g2)):
                    continue
                if not _screen(model, gx32, gm32, int(g1), int(g2), margin):
                    hits += O.convex_probe(row, int(g1), int(g2), model=model)[0] is not None
                    continue
                proven += 1
                hit, _, _ = O.convex_probe(row, int(g1), int(g2), model=model)
                checked += 1
                assert hit is None, (b, g1, g2, hit)
    assert checked > 50, (proven, checked)
    assert hits > 0, hits   # the states do hold convex contacts the screen must not hide
