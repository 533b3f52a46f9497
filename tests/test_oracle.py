"""CPU tests: the oracle against the reference's own known answers and golden vectors.

* home_wpt KAT: FK(ee_center_site, neutral q) = [1.23843967, 0, 0.49740014]
  (reference scripts/execute_pnp.py:38, test/reward_test.py:47; neutral pose panda_env.py:64-66).
* ik_golden.npz: outputs of the reference's JacobianIKController.solve (skills/ik_solver.py:35-101)
  run unmodified over the oracle's kinematics (tests/golden/make_golden.py).
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "ik_golden.npz")
NEUTRAL = np.array([0.00, 0.41, 0.00, -1.85, 0.00, 2.26, 0.79, 0.00, 0.00])
HOME_WPT = np.array([1.23843967, 0.0, 0.49740014])


def test_home_wpt_known_answer(model):
    q = model.qpos0.copy()
    q[:9] = NEUTRAL
    sx, _ = O.site_kinematics(q[None])
    ee = sx[0, model.site_id("ee_center_site")]
    # the reference prints the KAT with 8 decimals
    assert np.abs(ee - HOME_WPT).max() < 5e-9


def test_cube_and_target_sites_at_xml_positions(model):
    sx, sm = O.site_kinematics(model.qpos0[None])
    exp = {"cube1_site": [1.4, 0, 0.73], "cube2_site": [1.4, 0, 1.03], "cube3_site": [1.4, 0, 0.43],
           "target_cube1": [1.0, -0.1, 0.3], "target_cube2": [1.0, 0, 0.3], "target_cube3": [1.0, 0.1, 0.3]}
    for name, p in exp.items():
        assert np.allclose(sx[0, model.site_id(name)], p, atol=1e-12), name
        assert np.allclose(sm[0, model.site_id(name)], np.eye(3).ravel(), atol=1e-12)


def test_mat2quat_roundtrip():
    rng = np.random.default_rng(0)
    for _ in range(50):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        if q[0] < 0:
            q = -q
        w, x, y, z = q
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                      [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                      [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
        q2 = O.mat2quat(R)
        assert np.allclose(q2 * np.sign(q2[0] or 1), q, atol=1e-12)


def test_jacobian_matches_finite_differences(model):
    rng = np.random.default_rng(1)
    s = model.site_id("ee_center_site")
    for _ in range(5):
        q = model.qpos0.copy()
        q[:7] = rng.uniform(model.jnt_range[:7, 0] * 0.9, model.jnt_range[:7, 1] * 0.9)
        J = O.jac_site(q[None])[0]
        h = 1e-7
        for j in range(7):
            qp, qm = q.copy(), q.copy()
            qp[j] += h
            qm[j] -= h
            fd = (O.site_kinematics(qp[None])[0][0, s] - O.site_kinematics(qm[None])[0][0, s]) / (2 * h)
            assert np.allclose(J[:, j], fd, atol=1e-7)
        assert np.all(J[:, 7:] == 0)


@pytest.fixture(scope="module")
def golden():
    return np.load(GOLDEN, allow_pickle=False)


def test_golden_fixture_covers_cases(golden):
    tags = set(golden["tag"].tolist())
    assert {"ik_test", "waypoint/default", "ik_test/ik_test", "edge/unreachable",
            "edge/max_iters_0", "edge/q_outside_limits"} <= tags
    assert golden["converged"].sum() > 100 and (~golden["converged"]).sum() > 5


def test_oracle_matches_reference_ik_golden(golden):
    n = len(golden["tag"])
    for i in range(n):
        r = O.ik_dls(golden["q_init"][i][None], golden["target"][i][None], max_iters=int(golden["max_iters"][i]),
                     pos_thresh=float(golden["pos_thresh"][i]), damping=float(golden["damping"][i]),
                     step_limit=float(golden["step_limit"][i]))
        tag = golden["tag"][i]
        assert r["iterations"][0] == golden["iterations"][i], tag
        assert bool(r["flags"][0] & 1) == bool(golden["converged"][i]), tag
        assert bool(r["flags"][0] & 2) == bool(golden["success"][i]), tag
        np.testing.assert_allclose(r["q"][0], golden["q"][i], atol=1e-11, err_msg=tag)
        np.testing.assert_allclose(r["final_pos"][0], golden["final_pos"][i], atol=1e-11, err_msg=tag)
        assert abs(r["pos_error"][0] - golden["pos_error"][i]) < 1e-11


def test_reference_ik_test_scenario(golden):
    """test/ik_test.py:26-49 asserts |final - target| < 0.05; the golden run converges in 10."""
    i = list(golden["tag"]).index("ik_test")
    assert golden["converged"][i] and golden["iterations"][i] == 10
    assert np.linalg.norm(golden["final_pos"][i] - golden["target"][i]) < 0.05


def test_oracle_threads_agree(model):
    from pnp_amd import workloads
    idx = np.arange(64)
    q, d = workloads.ik_inputs(model, idx)
    qf = np.tile(model.qpos0, (64, 1))
    qf[:, :7] = q
    tgt = O.site_kinematics(qf)[0][:, model.site_id("ee_center_site")] + d
    a = O.ik_dls(q, tgt, nthreads=1)
    b = O.ik_dls(q, tgt, nthreads=4)
    for k in a:
        assert np.array_equal(a[k], b[k])
