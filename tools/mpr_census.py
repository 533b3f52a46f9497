"""MPR work on the steady-state gym workload (CPU oracle; the kernels run the same iteration):
per env class (contacts 21-64: the full tier, > 64: the wide tier) the MPR runs per forward, support
pairs per run, discover / refine / penetration loop trips per run, runs that hit the penetration
cap, and the largest support count of one run (oracle/convex.c g_mpr counters).
usage: python tools/mpr_census.py [states.npz] [max_envs_per_class]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
from oracle import oracle as O  # noqa: E402
from pnp_amd.model import load_model  # noqa: E402


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "scratch", "steady_states.npz")
    cap = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    z = np.load(path)
    m = load_model()
    nc = z["ncon"]
    for label, sel in (("compact (<= 20)", nc <= 20), ("full (21-64)", (nc > 20) & (nc <= 64)), ("wide (> 64)", nc > 64)):
        idx = np.nonzero(sel)[0][:cap]
        O.mpr_stats(reset=True)
        per_env = []
        for b in idx:
            O.mpr_stats(reset=True)
            O.forward_fields({k: z[k][b] for k in O.STATE_KEYS}, ["ncon"], model=m)
            per_env.append(O.mpr_stats(reset=True))
        runs = np.array([s["runs"] for s in per_env], float)
        tot = {k: sum(s[k] for s in per_env) for k in per_env[0]}
        r = max(tot["runs"], 1)
        print(f"== {label}: {len(idx)} envs; MPR runs per forward mean {runs.mean():.1f} max {runs.max():.0f}; per run: "
              f"supports {tot['supports'] / r:.1f}, discover {tot['discover'] / r:.2f}, refine {tot['refine'] / r:.2f}, "
              f"penetration {tot['penetration'] / r:.2f}; capped runs {tot['capped']}; largest run "
              f"{max(s['max_supports_run'] for s in per_env)} supports", flush=True)
        w = int(np.argmax([s["supports"] for s in per_env]))
        print(f"   heaviest env {idx[w]}: {per_env[w]}")


if __name__ == "__main__":
    main()
