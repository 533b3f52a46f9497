"""The engine's observation moments against the reference's own VecNormalize statistics (VERDICT
round 5, item 4): tests/golden/vecnormalize_200k.json holds sb3's running mean /
var of every observation column after the reference's 200k-step TQC run in real MuJoCo 2.3.3
(scripts/checkpoints/tqc_dense_vecnormalize_200000_steps.pkl, decoded by
tests/golden/make_vecnorm_fixture.py from the pickle's opcodes, never unpickled) -- the only
reference-held record of real-MuJoCo state at gym-step boundaries.  The reference's statistics mix
a learning policy's 667 episodes; the policy-independent moments are compared:

  * settled at gym-step boundaries (250 sub-steps after every action): the variances of ee_vel and
    of the cube's linear and angular velocity are ~0 in the reference (ee_vel 1e-8, cube velp
    <= 1.4e-7, velr <= 3e-6).  Run A (uniform random actions from reset -- TQC's learning_starts
    phase; its initial policy acts alike -- 512 envs x 80 gym steps, auto-reset) measured ee_vel
    2.6e-8 / 2.1e-8 / 3.8e-8 (the reference's order on every axis: asserted within 10x), cube velp
    1.3e-8 / 2.6e-9 / 2.7e-7 (within 30x), cube velr up to 2.8e-5 (the reference's cubes rest on
    the floor most of the run, ours on their boards under a random arm: asserted ~0 only,
    < 1e-4);
  * the gripper: finger width mean 0.0326 against 0.0289 and variance 1.91e-3 against 1.76e-3 --
    both above the largest variance a width inside the joint range [0, 0.08] could have at that
    mean, i.e. real MuJoCo squeezes the fingers past closed as this engine does (asserted: mean
    within 0.01, variance within 2x, both above the in-range bound);
  * the reset random walk (panda_env.py:146-158: each reset puts a cube at its current site plus
    U(+-0.02) x U(+-0.2)): run B, 512 envs x 167 one-step episodes (the reference's 4 workers ran
    ~167 episodes each), achieved_goal y variance 1.09 against 0.67 and x 0.0147 against 0.028
    (within 3x), mean height 0.097 m against 0.081 (the cubes walk off their boards to the floor:
    within 2x, inside floor-to-board).
Measured numbers are printed next to the reference's."""
import dataclasses
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = json.load(open(os.path.join(ROOT, "tests", "golden", "vecnormalize_200k.json")))
KEYS = ("observation", "achieved_goal")


def _moments(env, steps, seed):
    B = env.num_envs
    s, ss, n = {}, {}, 0

    def add(obs):
        nonlocal n
        for k in KEYS:
            x = obs[k].double()
            s[k] = s.get(k, 0) + x.sum(0)
            ss[k] = ss.get(k, 0) + (x * x).sum(0)
        n += B

    add(env.reset())
    g = torch.Generator(device="cuda").manual_seed(seed)
    for _ in range(steps):
        obs, *_ = env.step(torch.rand(B, 7, device="cuda", generator=g) * 2 - 1)
        add(obs)
    out = {}
    for k in KEYS:
        m = (s[k] / n).cpu().numpy()
        out[k] = (m, np.maximum((ss[k] / n).cpu().numpy() - m * m, 0.0))
    return out


def _ref(k):
    return np.array(REF["obs_rms"][k]["mean"]), np.array(REF["obs_rms"][k]["var"])


@pytest.mark.timeout(300)
def test_settled_moments_match_reference_vecnormalize():
    from pnp_amd.envs import BatchedFrankaShelfPNPEnv
    got = _moments(BatchedFrankaShelfPNPEnv(512, autoreset=True), 80, seed=3)
    m, v = got["observation"]
    rm, rv = _ref("observation")
    cols = REF["observation_columns"]
    for i in range(19):
        print(f"{cols[i]:14s} mean {m[i]: .4e} (ref {rm[i]: .4e})  var {v[i]:.3e} (ref {rv[i]:.3e}, ratio {v[i] / rv[i]:.2g})")
    ee, velp, velr = slice(3, 6), slice(13, 16), slice(16, 19)
    assert (v[ee] < 10 * rv[ee]).all() and (v[ee] > rv[ee] / 10).all(), (v[ee], rv[ee])
    assert (v[velp] < 30 * rv[velp]).all() and (v[velp] > rv[velp] / 30).all(), (v[velp], rv[velp])
    assert (v[velr] < 1e-4).all(), v[velr]
    # finger width: the moments match, and both exceed what a width inside [0, 0.08] allows
    w, rw = 6, 6
    assert abs(m[w] - rm[rw]) < 0.01 and rv[rw] / 2 < v[w] < 2 * rv[rw], (m[w], v[w], rm[rw], rv[rw])
    for mean, var in ((m[w], v[w]), (rm[rw], rv[rw])):
        assert var > mean * (0.08 - mean), (mean, var)


@pytest.mark.timeout(300)
def test_reset_random_walk_matches_reference_vecnormalize():
    from pnp_amd.envs import BatchedFrankaShelfPNPEnv, EnvConfig
    cfg = dataclasses.replace(EnvConfig(), max_episode_steps=1)
    got = _moments(BatchedFrankaShelfPNPEnv(512, autoreset=True, config=cfg), 167, seed=5)
    m, v = got["achieved_goal"]
    rm, rv = _ref("achieved_goal")
    print(f"achieved_goal mean {m} (ref {rm}), var {v} (ref {rv})")
    assert rv[1] / 3 < v[1] < 3 * rv[1] and rv[0] / 3 < v[0] < 3 * rv[0], (v, rv)
    assert 0.0199 <= m[2] <= 0.75 and rm[2] / 2 < m[2] < 2 * rm[2], (m, rm)
