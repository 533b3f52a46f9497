"""Diagnostic: fp64 env step vs oracle, per gym step: state and observation component errors."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
from oracle.env_oracle import EnvOracle  # noqa: E402
from pnp_amd.envs import BatchedFrankaShelfPNPEnv  # noqa: E402

B = 4
g = BatchedFrankaShelfPNPEnv(B, dtype=torch.float64, autoreset=False)
o = EnvOracle(B)
g.reset(); o.reset()
for nsub_total in (1,):
    pass
for k in range(3):
    a = np.random.default_rng(10 + k).uniform(-1, 1, size=(B, 7)).astype(np.float32).astype(np.float64)
    if os.environ.get("OPEN"):
        a[:, 6] = 1.0
    obs, r, *_ = g.step(torch.as_tensor(a, dtype=torch.float64))
    res = o.step(a)
    go = obs["observation"].cpu().numpy()
    ro = np.stack([x["obs"]["observation"] for x in res])
    print(f"step {k}: qpos {np.abs(g.state['qpos'].cpu().numpy() - o.st['qpos']).max():.2e} "
          f"qvel {np.abs(g.state['qvel'].cpu().numpy() - o.st['qvel']).max():.2e} "
          f"(|qvel| {np.abs(o.st['qvel']).max():.2e}) qkin {np.abs(g.env['qpos_kin'].cpu().numpy() - o.qpos_kin).max():.2e} "
          f"warm {np.abs(g.state['qacc_warmstart'].cpu().numpy() - o.st['qacc_warmstart']).max():.2e}")
    print("   obs err per comp", np.abs(go - ro).max(0).round(12))
    print("   reward err", np.abs(r.cpu().numpy() - np.array([x['reward'] for x in res])).max())
# same test on the plain step kernel: 250 sub-steps of the f64 kernel vs oracle from the same state
from oracle import oracle as O  # noqa: E402
st = {k: v.cpu().numpy().astype(np.uint32 if k == "warn" else np.float64) for k, v in g.state.items()}
gs = {k: v.clone() for k, v in g.state.items()}
for n in (1, 10, 50, 250):
    ref = {k: v.copy() for k, v in st.items()}
    O.step(ref, nsub=n, nthreads=8)
    gg = {k: v.clone() for k, v in gs.items()}
    g.engine.step(gg, n)
    print(f"pnp_step_f64 nsub {n}: qpos {np.abs(gg['qpos'].cpu().numpy() - ref['qpos']).max():.2e} "
          f"qvel {np.abs(gg['qvel'].cpu().numpy() - ref['qvel']).max():.2e}")
