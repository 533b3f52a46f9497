"""Solver iteration counts under MuJoCo 2.3.3's exits (round 4: restated in the oracle and every
kernel tier).  mj_solNoSlip stops once a sweep's scaled cost improvement falls below
opt.noslip_tolerance (1e-6); mj_solNewton once scale (cost_old - cost) or scale |grad| falls below
opt.tolerance (1e-8), scale = 1 / (stat.meaninertia nv).  Prints, over C3-like settled states and
the mesh-contact fixture: the oracle's per-sweep improvement and sweep counts, and -- with a GPU --
the kernel's Newton iterations and sweeps (fp64 instantiation env by env against the oracle, and
the fp32 product kernel's distribution).
usage: python tools/noslip_exit_diag.py [envs]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd"), os.path.join(ROOT, "tests")]
from oracle import oracle as O  # noqa: E402
from pnp_amd.model import load_model  # noqa: E402
import physics_states as PS  # noqa: E402


def hist(x, n=4):
    x = np.asarray(x)
    return " ".join(f"{k}: {np.mean(x == k):.2f}" for k in range(n))


def report(name, m, st, eng=None):
    B = st["qpos"].shape[0]
    f = [O.forward_fields({k: st[k][b] for k in O.STATE_KEYS}, ["noslip_improvement", "noslip_iter", "solver_iter"],
                          model=m) for b in range(B)]
    imp = np.array([x["noslip_improvement"][:3] for x in f])
    ns = np.array([int(x["noslip_iter"][0]) for x in f])
    nw = np.array([int(x["solver_iter"][0]) for x in f])
    print(f"{name}: {B} envs")
    print(f"  oracle improvement per sweep (-1: not run): median {np.median(imp, 0)}, max {imp.max(0)}")
    print(f"  oracle noslip sweeps   {hist(ns)}")
    print(f"  oracle newton iters    mean {nw.mean():.2f} max {nw.max()}")
    if eng is None:
        return
    import torch
    from pnp_amd import _lib
    D = _lib.DBG
    for dt in (torch.float64, torch.float32):
        src = st if dt == torch.float64 else {k: (v if k == "warn" else v.astype(np.float32).astype(np.float64))
                                                for k, v in st.items()}
        g = {k: torch.as_tensor(v.astype(np.int32) if k == "warn" else np.ascontiguousarray(v),
                                dtype=torch.int32 if k == "warn" else dt, device="cuda").contiguous()
             for k, v in src.items()}
        dbg = eng.forward_debug(g).cpu().numpy()
        kns = dbg[:, D["NOSLIP_ITER"]].astype(int)
        knw = dbg[:, D["COUNTS"] + 2].astype(int)
        tag = "fp64" if dt == torch.float64 else "fp32"
        print(f"  kernel {tag} noslip sweeps {hist(kns)}   newton iters mean {knw.mean():.2f} max {knw.max()}")
        if dt == torch.float64:
            print(f"  kernel fp64 = oracle, env by env: noslip {np.mean(kns == ns):.3f}, newton {np.mean(knw == nw):.3f}")


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    m = load_model()
    eng = None
    try:
        import torch
        if torch.cuda.is_available():
            from pnp_amd.engine import get_engine
            eng = get_engine()
    except ImportError:
        pass
    report("settled (C3-like)", m, PS.settled_states(B, seed=0, nsettle=200, model=m), eng)
    import test_step_gpu as T
    report("mesh-contact fixture", m, T.mesh_states(m), eng)
    report("fresh resets (cubes landing)", m, PS.reset_states(32, seed=7, model=m), eng)


if __name__ == "__main__":
    main()
