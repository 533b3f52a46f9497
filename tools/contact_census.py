"""Contact census of the gym workload on the CPU env oracle: random actions (C5's exploration
phase), per gym step the number of contacts of each env after the step and which geom pairs make
them.  usage: python tools/contact_census.py [envs] [gym_steps] [seed]"""
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
from oracle import oracle as O  # noqa: E402
from oracle.env_oracle import EnvOracle  # noqa: E402
from pnp_amd.model import load_model  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    mode = sys.argv[4] if len(sys.argv) > 4 else "uniform"   # uniform | saturated (constant +-1 per env)
    m = load_model()
    o = EnvOracle(B, model=m, nthreads=8)
    o.reset()
    rng = np.random.default_rng(seed)
    const = np.sign(rng.uniform(-1, 1, size=(B, 7)))
    counts = []
    pairs = collections.Counter()
    for k in range(n):
        a = const if mode == "saturated" else rng.uniform(-1, 1, size=(B, 7))
        o.step(a.astype(np.float32).astype(np.float64))
        row = []
        for b in range(B):
            f = O.forward_fields({kk: v[b] for kk, v in o.st.items()}, ["ncon", "contact"], model=m)
            nc = int(f["ncon"][0])
            row.append(nc)
            c = f["contact"].reshape(-1, 30)
            for g1, g2 in c[:, 27:29].astype(int):
                pairs[(str(m.names_geom[g1]) or g1,
                       str(m.names_geom[g2]) or g2)] += 1
        counts.append(row)
        print(f"gym step {k}: ncon per env {row}", flush=True)
    a = np.array(counts)
    print(f"max {a.max()}  mean {a.mean():.1f}  >20: {(a > 20).mean():.2f}  >32: {(a > 32).mean():.2f}  "
          f">48: {(a > 48).mean():.2f}  >64: {(a > 64).mean():.2f}")
    for p, c in pairs.most_common(25):
        print(f"  {p}: {c / a.size:.2f} per env-step")


if __name__ == "__main__":
    main()
