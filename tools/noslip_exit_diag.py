"""How many noslip sweeps MuJoCo 2.3.3 would run (diagnostic, CPU oracle).  mj_solNoSlip stops once
a sweep's scaled cost improvement falls below opt.noslip_tolerance (default 1e-6); this engine
always runs noslip_iterations (3) sweeps.  Prints, over C3-like settled states and the mesh-contact
fixture, each sweep's improvement and the sweeps MuJoCo would run.
usage: python tools/noslip_exit_diag.py [envs]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd"), os.path.join(ROOT, "tests")]
from oracle import oracle as O  # noqa: E402
from pnp_amd.model import load_model  # noqa: E402
import physics_states as PS  # noqa: E402

TOL = 1e-6


def report(name, m, st):
    imp = np.array([O.forward_fields({k: st[k][b] for k in O.STATE_KEYS}, ["noslip_improvement"], model=m)
                    ["noslip_improvement"][:3] for b in range(st["qpos"].shape[0])])
    runs = np.where(imp[:, 0] < TOL, 1, np.where(imp[:, 1] < TOL, 2, 3))
    print(f"{name}: {len(imp)} envs; improvement per sweep: median {np.median(imp, 0)}, max {imp.max(0)}")
    print(f"  sweeps MuJoCo would run: 1: {np.mean(runs == 1):.2f}  2: {np.mean(runs == 2):.2f}  3: {np.mean(runs == 3):.2f}")


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    m = load_model()
    report("settled (C3-like)", m, PS.settled_states(B, seed=0, nsettle=200, model=m))
    import test_step_gpu as T
    report("mesh-contact fixture", m, T.mesh_states(m))


if __name__ == "__main__":
    main()
