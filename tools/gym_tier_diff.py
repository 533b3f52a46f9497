"""Diagnostic: gym steps starting in the compact tier vs the full tier; which envs differ, by how
much, and whether they were handed over (PNP_GYM_COMPACT=2 leaves the resume bits)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
from pnp_amd.envs import BatchedFrankaShelfPNPEnv  # noqa: E402


def make(B):
    g = BatchedFrankaShelfPNPEnv(B, autoreset=False)
    g.reset()
    g.state["qpos"][::3, 7:9] = -0.002
    return g


def main():
    B = 96
    envs = {m: make(B) for m in ("0", "1", "2")}
    rng = np.random.default_rng(21)
    for k in range(3):
        a = torch.as_tensor(rng.uniform(-1, 1, size=(B, 7)), dtype=torch.float32, device="cuda")
        res = {}
        for m, g in envs.items():
            os.environ["PNP_GYM_COMPACT"] = m
            st0 = {kk: v.clone() for kk, v in g.state.items()}
            obs, r, term, trunc, info = g.step(a)
            res[m] = (obs["observation"].clone(), r.clone(), {kk: v.clone() for kk, v in g.state.items()})
            if m == "2":
                w = g.state["warn"].to(torch.int64) & 0xFFFFFFFF
                hand = ((w >> 31) & 1).bool().cpu().numpy()
                sub = ((w >> 16) & 0xFFF).cpu().numpy()
                why = ((w >> 28) & 7).cpu().numpy()
                # restore mode-1 state into the diagnostic env so the next step starts equal
                for kk in g.state:
                    g.state[kk].copy_(envs["1"].state[kk])
                for kk in g.env:
                    g.env[kk].copy_(envs["1"].env[kk])
        torch.cuda.synchronize()
        o0, r0, s0 = res["0"]
        o1, r1, s1 = res["1"]
        dob = (o0 - o1).abs().max(1).values.cpu().numpy()
        dq = (s0["qpos"] - s1["qpos"]).abs().max(1).values.cpu().numpy()
        bad = np.nonzero((dob > 0) | (dq > 0))[0]
        print(f"step {k}: handed over {hand.sum()} envs {np.nonzero(hand)[0][:20]} at sub-steps {sub[hand][:20]} why {why[hand][:20]}")
        print(f"  differing envs {len(bad)}: {bad[:20]}  max dobs {dob.max():.3e} max dqpos {dq.max():.3e}")
        print(f"  differing & handed over: {np.intersect1d(bad, np.nonzero(hand)[0])[:20]}")
        # continue from equal states
        for kk in envs["0"].state:
            envs["0"].state[kk].copy_(envs["1"].state[kk])
        for kk in envs["0"].env:
            envs["0"].env[kk].copy_(envs["1"].env[kk])


if __name__ == "__main__":
    main()
