"""How often the compact kernel hands envs over to the full kernel (step.hip resume protocol), on
the bench's gym workload (random actions) and C3 step workload.  For each step the state is
saved, stepped once with the compact kernel alone (PNP_STEP_COMPACT=2: handed-over envs keep
their resume bits = flag + sub-step), restored, and stepped normally.
usage: python tools/handover_stats.py [B] [gym_steps]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]


def report(tag, w, nsub):
    w = w.cpu().numpy().astype(np.uint32)
    flag = ((w >> 31) & 1) == 1
    sub = (w >> 16) & 0xFFF
    if flag.any():
        why = (w >> 28) & 7
        reasons = ", ".join(f"{n} {((why[flag] & bit) != 0).mean() * 100:.0f}%"
                            for n, bit in (("contacts", 1), ("rows/slots", 2), ("island blocks", 4)))
        print(f"{tag}: overflowing capacity: {reasons}")
        q = np.percentile(sub[flag], [0, 25, 50, 75, 100]).astype(int)
        print(f"{tag}: {flag.mean() * 100:5.1f}% envs handed over; sub-step of hand-over (of {nsub}) "
              f"min/q1/median/q3/max {q.tolist()}; full-kernel share of sub-steps "
              f"{(nsub - sub[flag]).sum() / (len(w) * nsub) * 100:.1f}%", flush=True)
    else:
        print(f"{tag}: no hand-over", flush=True)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    os.environ["PNP_GYM_COMPACT"] = "1"      # the opt-in compact gym path (env_host.h)
    os.environ["PNP_GYM_CHUNK"] = "250"      # one physics launch: resume bits survive to the end
    from pnp_amd.envs import BatchedFrankaShelfPNPEnv
    from pnp_amd.engine import get_engine
    from pnp_amd import _lib
    eng, D = get_engine(), _lib.DBG
    g = BatchedFrankaShelfPNPEnv(B, dtype=torch.float32, autoreset=True)
    g.reset()
    rng = np.random.default_rng(0)
    nsub = g.config.n_substeps * g.config.n_calls if hasattr(g, "config") else 250
    for k in range(nsteps):
        a = torch.as_tensor(rng.uniform(-1, 1, size=(B, 7)), dtype=torch.float32, device=g.device)
        saved = ({n: v.clone() for n, v in g.state.items()}, {n: v.clone() for n, v in g.env.items()})
        os.environ["PNP_STEP_COMPACT"] = "2"
        g.step(a)
        torch.cuda.synchronize()
        report(f"gym step {k}", g.state["warn"], nsub)
        for n, v in saved[0].items():
            g.state[n].copy_(v)
        for n, v in saved[1].items():
            g.env[n].copy_(v)
        os.environ["PNP_STEP_COMPACT"] = "1"
        g.step(a)
        d = eng.forward_debug(g.state).cpu().numpy()
        nc = d[:, D["COUNTS"]].astype(int)
        ne = d[:, D["COUNTS"] + 1].astype(int)
        print(f"  after step {k}: ncon percentiles 50/90/99/max {np.percentile(nc, [50, 90, 99, 100]).tolist()}, "
              f"nefc 50/90/99/max {np.percentile(ne, [50, 90, 99, 100]).tolist()}; "
              f"envs > 20 contacts {np.mean(nc > 20) * 100:.1f}%, > 24 {np.mean(nc > 24) * 100:.1f}%, "
              f"> 32 {np.mean(nc > 32) * 100:.1f}%", flush=True)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
