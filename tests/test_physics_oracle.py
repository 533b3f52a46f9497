"""CPU checks of the fp64 mj_step oracle (oracle/physics.c, collision.c).

Dynamics parity against MuJoCo itself is unpinned: the reference's dynamics live in MuJoCo 2.3.3,
which is not installed, and the reference's tests hold no dynamics vectors.  So the
oracle is checked here against independent restatements and physical invariants instead:

* the CRBA mass matrix against the Jacobian sum sum_b J_b^T m_b J_b + J_r^T I J_r + armature;
* the RNE bias at rest against the gravity-only generalised force sum_b Jp_b^T m_b (-g);
* exact semi-implicit Euler free fall of the unconstrained dummy sphere;
* a cube sliding on a shelf board stops after about v^2 / (2 mu g);
* mj_checkPos / mj_checkVel reset the env and raise the warning bit (mj_resetData semantics);
* bit-identical results across worker-thread counts.
"""
import numpy as np
import pytest

from oracle import oracle as O
from pnp_amd import setconst

import physics_states as PS


def _row(st, b):
    return {k: st[k][b] for k in O.STATE_KEYS}


def _random_arm(model, n, seed):
    st = PS.reset_states(n, seed=seed, model=model)
    rng = np.random.default_rng(seed)
    lo, hi = model.jnt_range[:9, 0], model.jnt_range[:9, 1]
    st["qpos"][:, :9] = rng.uniform(lo, hi, size=(n, 9))
    return st


def test_mass_matrix_matches_jacobian_sum(model):
    st = _random_arm(model, 6, seed=11)
    raw = model.__dict__
    for b in range(6):
        f = O.forward_fields(_row(st, b), ["qM"], model=model)
        M = f["qM"].reshape(model.nv, model.nv)
        Mj = setconst.mass_matrix(raw, st["qpos"][b])
        assert np.abs(M - Mj).max() <= 1e-12 * max(1.0, np.abs(Mj).max())
        assert np.allclose(M, M.T, atol=0, rtol=0)


def test_bias_at_rest_is_gravity(model):
    st = _random_arm(model, 4, seed=12)
    raw = model.__dict__
    g = np.array([0.0, 0.0, -9.81])
    for b in range(4):
        f = O.forward_fields(_row(st, b), ["qfrc_bias"], model=model)
        Jp, _, _, _ = setconst.body_jacobians(raw, st["qpos"][b])
        want = np.zeros(model.nv)
        for i in range(1, model.nbody):
            want -= model.body_mass[i] * Jp[i].T @ g
        assert np.abs(f["qfrc_bias"] - want).max() <= 1e-10 * max(1.0, np.abs(want).max())


def test_dummy_free_fall_is_semi_implicit_euler(model):
    st = PS.reset_states(1, seed=0, model=model)
    a = int(model.jnt_qposadr[model.joint_id("obj_joint")])
    d = int(model.jnt_dofadr[model.joint_id("obj_joint")])
    st["qpos"][0, a:a + 3] = [2.0, 2.0, 3.0]          # far from every other geom
    st["qvel"][0, d:d + 3] = [0.1, -0.2, 0.3]
    z0, vz0 = 3.0, 0.3
    h = model.opt_timestep
    n = 20
    O.step(st, nsub=n, model=model)
    vz = vz0 - 9.81 * h * n
    z = z0 + h * sum(vz0 - 9.81 * h * k for k in range(1, n + 1))
    assert abs(st["qvel"][0, d + 2] - vz) < 1e-12
    assert abs(st["qpos"][0, a + 2] - z) < 1e-12
    assert abs(st["qpos"][0, a] - (2.0 + 0.1 * h * n)) < 1e-12
    assert st["time"][0] == pytest.approx(h * n, abs=1e-15)


def test_cube_on_shelf_stops_by_friction(model):
    st = PS.settled_states(1, seed=0, nsettle=100, model=model)
    j = model.joint_id("cube2_joint")
    a, d = int(model.jnt_qposadr[j]), int(model.jnt_dofadr[j])
    x0 = st["qpos"][0, a]
    v0 = 0.3
    st["qvel"][0, d] = v0
    O.step(st, nsub=60, model=model)
    assert abs(st["qvel"][0, d]) < 1e-3, "cube still sliding after 0.12 s"
    slide = st["qpos"][0, a] - x0
    coulomb = v0 ** 2 / (2 * 1.0 * 9.81)              # mu = 1 (max-mixed cube/shelf friction)
    assert 0.5 * coulomb < slide < 2.0 * coulomb
    assert st["warn"][0] == 0


def test_bad_qpos_resets_env_and_warns(model):
    st = PS.settled_states(2, seed=0, nsettle=10, model=model)
    st["qpos"][1, 3] = np.nan
    O.step(st, nsub=1, model=model)
    assert st["warn"][1] & 1                          # PNP_WARN_BADQPOS
    assert st["warn"][0] == 0
    assert np.isfinite(st["qpos"]).all()


def test_bad_qvel_resets_env_and_warns(model):
    st = PS.settled_states(1, seed=0, nsettle=10, model=model)
    st["qvel"][0, 12] = 1e11
    O.step(st, nsub=1, model=model)
    assert st["warn"][0] & 2                          # PNP_WARN_BADQVEL
    assert np.isfinite(st["qvel"]).all() and np.abs(st["qvel"]).max() < 1e3


def test_step_threads_bit_identical(model):
    st = PS.settled_states(8, seed=3, nsettle=20, model=model)
    PS.random_ctrl(st, model=model)
    a, b = PS.copy_state(st), PS.copy_state(st)
    O.step(a, nsub=5, nthreads=1, model=model)
    O.step(b, nsub=5, nthreads=4, model=model)
    for k in O.STATE_KEYS:
        assert np.array_equal(a[k], b[k]), k


def test_settled_scene_is_at_rest(model):
    st = PS.settled_states(4, seed=5, nsettle=250, model=model)
    for name in ("cube1_joint", "cube2_joint", "cube3_joint"):
        d = int(model.jnt_dofadr[model.joint_id(name)])
        assert np.abs(st["qvel"][:, d:d + 6]).max() < 5e-3, name
    assert (st["warn"] == 0).all()


# ---------------------------------------------------------------- convex (MPR) narrowphase
def _gid(model, name):
    return list(model.names_geom).index(name)


def test_mpr_matches_sat_on_resting_cube(model):
    """MPR (convex.c) on a box-box pair equals the exact SAT face-contact depth and normal."""
    st = PS.settled_states(2, seed=0, nsettle=100, model=model)
    for b in range(2):
        row = _row(st, b)
        f = O.forward_fields(row, ["contact", "ncon"], model=model)
        c = f["contact"].reshape(int(f["ncon"][0]), 30)
        g1, g2 = _gid(model, "shelf_board2"), _gid(model, "cube1_geom")
        sat = c[(c[:, 27] == g1) & (c[:, 28] == g2)]
        hit, _, _ = O.convex_probe(row, g1, g2, model=model)
        assert hit is not None and len(sat)
        assert abs(hit[0] - sat[:, 12].min()) < 1e-9
        assert np.allclose(hit[2], [0, 0, 1], atol=1e-9)


def _hand_in_cube(model):
    st = PS.reset_states(1, seed=0, model=model)
    sx, _ = O.site_kinematics(st["qpos"], model=model)
    a = int(model.jnt_qposadr[model.joint_id("cube1_joint")])
    st["qpos"][0, a:a + 3] = sx[0, model.site_id("ee_center_site")] + [0.0, 0.0, 0.075]   # into the palm
    return st


def test_mpr_depth_is_the_support_gap(model):
    """At MPR's termination the depth equals the Minkowski support gap along its direction,
    h(dir) = max_a a.dir - min_b b.dir, within mpr_tolerance."""
    st = _hand_in_cube(model)
    row = _row(st, 0)
    g_box, g_mesh = _gid(model, "cube1_geom"), 69           # the hand's collision mesh
    assert model.geom_type[g_mesh] == 7 and model.geom_type[g_box] == 6
    hit, gx, gm = O.convex_probe(row, g_box, g_mesh, model=model)
    assert hit is not None, "hand mesh and cube overlap"
    dist, pos, n = hit
    R = gm[g_box].reshape(3, 3)
    s = model.geom_size[g_box]
    corners = np.array([[i, j, k] for i in (-1, 1) for j in (-1, 1) for k in (-1, 1)]) * s
    wa = gx[g_box] + corners @ R.T
    mesh = int(model.geom_dataid[g_mesh])
    V = model.mesh_vert[model.mesh_vertadr[mesh]:model.mesh_vertadr[mesh] + model.mesh_vertnum[mesh]]
    wb = gx[g_mesh] + V @ gm[g_mesh].reshape(3, 3).T
    h = (wa @ n).max() - (wb @ n).min()
    assert np.isclose(np.linalg.norm(n), 1.0)
    assert -dist <= h + 1e-12 and h - (-dist) < 2e-6
    # the contact point lies between the two bodies' support planes along n
    assert (wb @ n).min() - 1e-9 <= pos @ n <= (wa @ n).max() + 1e-9


def test_mpr_separated_and_contact_list(model):
    st = _hand_in_cube(model)
    f = O.forward_fields(_row(st, 0), ["contact", "ncon"], model=model)
    c = f["contact"].reshape(int(f["ncon"][0]), 30)
    g_box = _gid(model, "cube1_geom")
    mesh_rows = c[(c[:, 27] == g_box) & np.isin(c[:, 28], np.nonzero(model.geom_type == 7)[0])]
    assert len(mesh_rows) >= 1 and np.all(mesh_rows[:, 12] < 0)        # box-mesh contacts present
    far = PS.reset_states(1, seed=0, model=model)
    hit, _, _ = O.convex_probe(_row(far, 0), g_box, 69, model=model)
    assert hit is None


def _pair_contacts(model, row, g1, g2):
    f = O.forward_fields(row, ["contact", "ncon"], model=model)
    c = f["contact"].reshape(int(f["ncon"][0]), 30)
    return c[(c[:, 27] == g1) & (c[:, 28] == g2)]


def test_multiccd_contact_fan(model):
    """multiccd (shelf_pnp.xml:5, mjc_Convex): the first contact of a convex pair is MPR's own
    (= the probe, = the single contact with the flag off); the perturbed runs add contacts on the
    flat faces, each farther than 1e-3 x min(rbound) from the pair's others, at most 5 per pair."""
    assert model.opt_multiccd == 1
    from pnp_amd.model import PandaModel
    off = PandaModel()   # (load_model() is the shared instance)
    off.opt_multiccd = 0
    off._desc = None
    st = PS.reset_states(1, seed=11, model=model)
    st["qpos"][:, 7:9] = 0.004
    sx, _ = O.site_kinematics(st["qpos"], model=model)
    a = int(model.jnt_qposadr[model.joint_id("cube1_joint")])
    st["qpos"][0, a:a + 3] = sx[0, model.site_id("ee_center_site")] + [0.0, 0.0, 0.075]   # into the palm
    row = _row(st, 0)
    g_box, g_mesh = _gid(model, "cube1_geom"), 69
    fan = _pair_contacts(model, row, g_box, g_mesh)
    one = _pair_contacts(off, row, g_box, g_mesh)
    assert len(one) == 1 and 2 <= len(fan) <= 5, (len(one), len(fan))
    assert np.array_equal(fan[0], one[0])
    hit, _, _ = O.convex_probe(row, g_box, g_mesh, model=model)
    assert abs(hit[0] - fan[0, 12]) < 1e-12 and np.allclose(hit[1], fan[0, :3], atol=1e-12)
    tol = 1e-3 * min(model.geom_rbound[g_box], model.geom_rbound[g_mesh])
    for i in range(len(fan)):
        for j in range(i):
            assert np.linalg.norm(fan[i, :3] - fan[j, :3]) > tol
    # every contact of the fan is a penetration along a unit normal with a completed frame
    assert np.all(fan[:, 12] < 0)
    fr = fan[:, 3:12].reshape(-1, 3, 3)
    assert np.allclose(np.einsum("nij,nkj->nik", fr, fr), np.eye(3), atol=1e-12)
    # across the scene's convex pairs: more contacts with the flag, never more than 5 per pair
    f_on = O.forward_fields(row, ["ncon"], model=model)["ncon"][0]
    f_off = O.forward_fields(row, ["ncon"], model=off)["ncon"][0]
    assert f_on > f_off


def test_meaninertia_is_the_mean_diagonal_of_M_at_qpos0(model):
    """stat.meaninertia (mj_setConst; scales the solvers' termination tests) = mean of diag(M) at
    qpos0 with armature -- the compiler's value (Jacobian-sum M, setconst.py) against the oracle's
    own CRBA at qpos0."""
    st = PS.reset_states(1, seed=0, model=model)
    st["qpos"][0] = model.qpos0
    M = O.forward_fields(_row(st, 0), ["qM"], model=model)["qM"].reshape(model.nv, model.nv)
    assert abs(model.stat_meaninertia - np.mean(np.diag(M))) <= 1e-12 * model.stat_meaninertia
    assert model.opt_noslip_tolerance == 1e-6 and model.opt_tolerance == 1e-8 and model.opt_iterations == 100


def _scale(model):
    return 1.0 / (model.stat_meaninertia * max(1, model.nv))


@pytest.mark.parametrize("kind", ["settled", "mesh"])
def test_noslip_stops_by_mujoco_rule(model, kind):
    """mj_solNoSlip's exit: sweep k ran only if sweep k-1's scaled improvement was >= noslip_tolerance,
    and the solver stopped after the first sweep below it (or at noslip_iterations)."""
    if kind == "settled":
        st = PS.settled_states(8, seed=0, nsettle=60, model=model)
    else:
        import test_step_gpu as T
        st = T.mesh_states(model)
    tol, cap = model.opt_noslip_tolerance, model.opt_noslip_iterations
    counts = []
    for b in range(st["qpos"].shape[0]):
        f = O.forward_fields(_row(st, b), ["noslip_improvement", "noslip_iter", "nefc"], model=model)
        n, imp = int(f["noslip_iter"][0]), f["noslip_improvement"]
        if int(f["nefc"][0]) == 0:
            assert n == 0
            continue
        assert 1 <= n <= cap
        assert all(imp[k] >= tol for k in range(n - 1))          # earlier sweeps did not stop it
        assert imp[n - 1] < tol or n == cap                       # the last one did, or the cap
        assert all(imp[k] == -1 for k in range(n, 8))             # no sweep past the exit
        counts.append(n)
    if kind == "settled":
        assert set(counts) == {1}      # settled contacts: the first sweep's improvement is ~1e-20
    else:
        assert max(counts) == cap and min(counts) == 1


def test_newton_stops_by_mujoco_rule(model):
    """mj_solNewton's exits on the mesh fixture: after the last step the scaled improvement or the
    scaled gradient is below tolerance (or the iteration cap); the scaled values are reported."""
    import test_step_gpu as T
    st = T.mesh_states(model)
    tol = model.opt_tolerance
    its = []
    for b in range(st["qpos"].shape[0]):
        f = O.forward_fields(_row(st, b), ["solver_iter", "solver_improvement", "solver_gradient", "nefc"],
                             model=model)
        it = int(f["solver_iter"][0])
        its.append(it)
        if it == 0 or it == model.opt_iterations:
            continue
        assert f["solver_improvement"][0] < tol or f["solver_gradient"][0] < tol, (b, f)
    assert max(its) >= 2      # the fixture makes Newton iterate
