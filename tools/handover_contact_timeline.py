"""After the compact tier hands an env over (tools/gym_handover_census.py ... states.npz: the state
before the overflowing sub-step, the gym step's controls and mocap target in place), how long does
the env keep needing more than the compact tier's 20 contacts?  Steps the saved states on with
pnp_step one sub-step at a time (full tier first) up to the gym step's end and prints, every 10
sub-steps, how many envs are above 20 contacts at that state (forward_debug) and how many have
dropped back under 17 for good so far.  usage: python tools/handover_contact_timeline.py states.npz"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
os.environ["PNP_STEP_COMPACT"] = "0"
from pnp_amd import _lib  # noqa: E402
from pnp_amd.engine import get_engine  # noqa: E402

KEYS = ("qpos", "qvel", "ctrl", "mocap_pos", "mocap_quat", "qacc_warmstart", "time", "warn")


def main():
    d = np.load(sys.argv[1])
    n = len(d["env"])
    eng = get_engine()
    st = {}
    for k in KEYS:
        v = d[k]
        if k == "warn":
            st[k] = torch.as_tensor((v.astype(np.int64) & 0xFFFF).astype(np.int32), device="cuda")
        else:
            st[k] = torch.as_tensor(v, dtype=torch.float32, device="cuda").contiguous()
    k0 = d["k0"].astype(int)
    D = _lib.DBG
    last_heavy = np.full(n, -1)
    for s in range(250):
        ncon = eng.forward_debug(st)[:, D["COUNTS"]].cpu().numpy().astype(int)
        done = k0 + s >= 250           # this env's gym step has ended
        heavy = (ncon > 20) & ~done
        last_heavy[heavy] = s
        if s % 10 == 0:
            live = ~done
            print(f"+{s:3d} sub-steps: envs still in their gym step {int(live.sum())}, above 20 contacts "
                  f"{int(heavy.sum())}, 17-20 {int(((ncon > 16) & (ncon <= 20) & live).sum())}", flush=True)
        eng.step(st, 1)
    rem = 250 - k0
    print(f"sub-steps after the hand-over: {int(rem.sum())}; of them above 20 contacts at most "
          f"{int((last_heavy + 1).sum())} (up to each env's last heavy sub-step)")
    h, e = np.histogram(last_heavy + 1, bins=[0, 1, 10, 25, 50, 100, 150, 200, 251])
    print("sub-steps until the last one above 20 contacts:", {f"{a}-{b - 1}": int(c) for a, b, c in zip(e[:-1], e[1:], h)})


if __name__ == "__main__":
    main()
