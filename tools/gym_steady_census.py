"""Steady-state census of the fp32 gym workload (bench.py run_gym_steady's shape: 4096 envs, uniform
random actions, auto-reset): per gym step the envs starting in each tier, the hand-over queue's
counts and the wall time; every `every` steps the contact / row distribution (forward_debug through
the tiers), the finger opening and where the cubes are; optionally the state after the last step
(npz: the physics state, each env's tier and contact count) for tools/steady_stage_prof.py.  usage:
python tools/gym_steady_census.py [B] [steps] [every] [dump.npz]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
from pnp_amd import _lib  # noqa: E402
from pnp_amd.envs import BatchedFrankaShelfPNPEnv  # noqa: E402

D = _lib.DBG


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    every = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    dump = sys.argv[4] if len(sys.argv) > 4 else None
    g = BatchedFrankaShelfPNPEnv(B, autoreset=True)
    m = g.model
    g.reset()
    rng = np.random.default_rng(11)
    acts = torch.as_tensor(rng.uniform(-1, 1, size=(16, B, 7)), dtype=torch.float32, device="cuda")
    cube_z = [int(m.jnt_qposadr[m.joint_id(f"cube{i}_joint")]) + 2 for i in (1, 2, 3)]
    for k in range(n):
        t = g.env["tier"].to(torch.int64) & 3
        cnt = [int((t == i).sum()) for i in range(3)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.step(acts[k % 16])
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        q = _lib.env_queue_status()
        print(f"step {k + 1}: starts compact {cnt[0]} full {cnt[1]} wide {cnt[2]}; queue published {q['published']} "
              f"timeouts {q['timeouts']} fallback {q['fallback']}; {dt:.1f} ms", flush=True)
        if (k + 1) % every == 0:
            st = {kk: v for kk, v in g.state.items()}
            dbg = g.engine.forward_debug(st).cpu().numpy()
            nc, ne = dbg[:, D["COUNTS"]], dbg[:, D["COUNTS"] + 1]
            pct = lambda x: np.percentile(x, [50, 90, 99, 100]).astype(int).tolist()
            qp = g.state["qpos"].double().cpu().numpy()
            fw = qp[:, 7] + qp[:, 8]
            cz = qp[:, cube_z]
            el = g.env["elapsed"].cpu().numpy()
            print(f"  contacts p50/90/99/max {pct(nc)}; rows {pct(ne)}; > 20 contacts {int((nc > 20).sum())}, > 64 "
                  f"{int((nc > 64).sum())}, > 100 {int((nc > 100).sum())}; fingers closed (< 1 mm) {int((fw < 1e-3).sum())}, "
                  f"squeezed past closed {int((fw < -1e-4).sum())}; cubes on the floor (z < 0.03) {int((cz < 0.03).sum())} of "
                  f"{cz.size}; episode step p50 {int(np.median(el))}", flush=True)
            big = np.argsort(-nc)[:5]
            for b in big:
                con = dbg[b, D["CON"]:D["CON"] + 16 * int(nc[b])].reshape(int(nc[b]), 16)
                pairs = {}
                for g1, g2 in con[:, 13:15].astype(int):
                    key = (str(m.names_body[m.geom_bodyid[g1]]), str(m.names_body[m.geom_bodyid[g2]]))
                    pairs[key] = pairs.get(key, 0) + 1
                top = sorted(pairs.items(), key=lambda x: -x[1])[:6]
                print(f"    env {b}: {int(nc[b])} contacts, {int(ne[b])} rows, fingers {fw[b] * 1e3:.2f} mm; by body pair {top}",
                      flush=True)

    if dump:
        dbg = g.engine.forward_debug({kk: v for kk, v in g.state.items()}).cpu().numpy()
        out = {k: v.cpu().numpy() for k, v in g.state.items()}
        out.update(tier=(g.env["tier"].to(torch.int64) & 3).cpu().numpy(), ncon=dbg[:, D["COUNTS"]],
                   nefc=dbg[:, D["COUNTS"] + 1])
        np.savez(dump, **out)
        print(f"state after step {n} -> {dump}", flush=True)


if __name__ == "__main__":
    main()
