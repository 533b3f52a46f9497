"""BADQACC census: does the reference's reset random walk reproduce
MUJOCO_LOG.TXT:1-8 (real MuJoCo: BADQACC on cube3's angular dofs 24 / 25 at t = 1.15-1.57 s, i.e.
0.6-1.1 s into an episode, initial_time 0.5 s)?

The walk (panda_env.py:146-158): every reset re-centres each cube on its CURRENT site position and
adds U(+-0.02) in x and U(+-0.2) in y, z kept (shelf_pnp.py:23-24).  Over episodes the cubes drift,
into the shelf legs (shelf_pnp.xml:45-48: x in [1.35, 1.39] u [1.61, 1.65], |y| in [0.46, 0.50],
z in [0, 1.01]; the cubes start at x = 1.4, :61-77), off the boards, and -- once fallen -- along
the floor, into the table legs (:30-35).

The census runs B envs of the batched device env (pnp_env_reset / pnp_env_step: the product
kernels) through E episodes of S gym steps, every env reset at every episode start (so the walk
runs E times), and records per episode and cube:
  * the spawn: penetration depth into each static box (shelf legs, boards, table legs / top, the
    floor) and into the other cubes (all spawn with identity orientation: axis-aligned boxes),
    and whether anything supports it (board / table top / floor under its centre at its height);
  * a spawn probe: the first `probe` physics sub-steps from the reset state, one launch each (ctrl
    and mocap as reset), max |qacc| over each cube's dofs -- the transient a deep spawn causes;
  * every bad-state warning bit (BADQPOS / BADQVEL / BADQACC: the engine resets that env like
    mj_resetData) with its gym step, and the max |qacc_warmstart| (qacc of the last sub-step) over
    the cube dofs after each gym step;
  * --far: after each gym step, the contacts of a forward at the new state (forward_debug, the
    full tier's 48 contacts) that involve a cube, and how far each lies from that cube's centre --
    a box-box edge-edge contact of nearly parallel edges placed far along the edge lines would put
    a huge lever arm on the cube's angular dofs (one candidate for the reference's BADQACC on
    cube3's angular dofs 24 / 25).
Events are saved (spawn state + actions, --out) for replay on the fp64 CPU oracle.

usage: python tools/badqacc_census.py [--envs B] [--episodes E] [--steps S] [--policy small|uniform]
                                      [--probe N] [--dtype f32|f64] [--far] [--out file.npz]
"""
import argparse
import collections
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
from oracle import oracle as O  # noqa: E402
from pnp_amd.envs import BatchedFrankaShelfPNPEnv  # noqa: E402

CUBES = ("cube1", "cube2", "cube3")
HALF = 0.02   # cube half-size (shelf_pnp.xml:63,69,75)
BAD = {1: "BADQPOS", 2: "BADQVEL", 4: "BADQACC"}


def static_boxes(m):
    """Static box geoms (weld body 0) as axis-aligned boxes: names, centres, half-sizes."""
    f = O.forward_fields({k: v[0] for k, v in O.new_state(1, model=m).items()}, ["geom_xpos", "geom_xmat"], model=m)
    gx, gm = f["geom_xpos"].reshape(-1, 3), f["geom_xmat"].reshape(-1, 3, 3)
    names, ctr, half = [], [], []
    for g in range(m.ngeom):
        if m.geom_type[g] != 6 or m.body_weldid[m.geom_bodyid[g]] != 0:
            continue
        if not (m.geom_contype[g] or m.geom_conaffinity[g]):
            continue
        R = gm[g]
        h = np.abs(R) @ m.geom_size[g]      # axis-aligned extent (exact for the scene's unrotated boxes)
        names.append(str(m.names_geom[g]))
        ctr.append(gx[g])
        half.append(h)
    return np.array(names), np.array(ctr), np.array(half)


def aabb_depth(c1, h1, c2, h2):
    """Penetration depth of axis-aligned boxes (min overlap over the axes; <= 0: apart)."""
    ov = h1 + h2 - np.abs(c1 - c2)
    return ov.min(-1)


def classify(pos, names, ctr, half):
    """pos [B, 3 cubes, 3] at spawn -> per cube: deepest static penetration (depth, box name),
    deepest cube-cube penetration, supported flag."""
    B = pos.shape[0]
    h = np.full(3, HALF)
    d_st = aabb_depth(pos[:, :, None, :], h, ctr[None, None], half[None, None])   # [B, 3, nbox]
    k = d_st.argmax(-1)
    dmax = np.take_along_axis(d_st, k[..., None], -1)[..., 0]
    dfloor = HALF - pos[..., 2]                                                  # floor plane z = 0
    dcc = np.full((B, 3), -1.0)
    for i in range(3):
        for j in range(3):
            if i != j:
                dcc[:, i] = np.maximum(dcc[:, i], aabb_depth(pos[:, i], h, pos[:, j], h))
    # supported: a static box top (or the floor) within 1 mm under the cube's bottom face, whose
    # xy extent contains the cube's centre
    bottom = pos[..., 2] - HALF
    top = ctr[:, 2] + half[:, 2]
    inside = ((np.abs(pos[:, :, None, 0] - ctr[None, None, :, 0]) <= half[None, None, :, 0]) &
              (np.abs(pos[:, :, None, 1] - ctr[None, None, :, 1]) <= half[None, None, :, 1]))
    on = inside & (np.abs(bottom[..., None] - top[None, None]) < 1e-3)
    supported = on.any(-1) | (np.abs(bottom) < 1e-3)
    return dict(static_depth=dmax, static_box=names[k], floor_depth=dfloor, cube_depth=dcc, supported=supported)


def policy_actions(kind, rng, B):
    if kind == "uniform":
        return rng.uniform(-1, 1, size=(B, 7))
    # TQC's initial policy (train.py:88, log_std_init -3): a near-zero mean, std e^-3 = 0.05
    return np.clip(rng.normal(0.0, np.exp(-3.0), size=(B, 7)), -1, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--episodes", type=int, default=40)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--policy", default="small", choices=("small", "uniform"))
    ap.add_argument("--probe", type=int, default=25)
    ap.add_argument("--dtype", default="f32", choices=("f32", "f64"))
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--far", action="store_true", help="contact-distance check after every gym step")
    args = ap.parse_args()
    dt = torch.float32 if args.dtype == "f32" else torch.float64
    B = args.envs
    g = BatchedFrankaShelfPNPEnv(B, dtype=dt, autoreset=False)
    m = g.model
    eng = g.engine
    names, ctr, half = static_boxes(m)
    qadr = [int(m.jnt_qposadr[m.joint_id(f"{c}_joint")]) for c in CUBES]
    dadr = [int(m.jnt_dofadr[m.joint_id(f"{c}_joint")]) for c in CUBES]
    rng = np.random.default_rng(args.seed)
    cube_geoms = [m.geom_id(f"{c}_geom") for c in CUBES]
    far_max = 0.0
    far_n = 0
    t0 = time.time()
    rows = []          # per (episode, env, cube)
    events = []        # bad-state warnings
    replay = collections.defaultdict(list)
    g.reset()
    for ep in range(args.episodes):
        if ep:
            g.reset()
        g.state["warn"].zero_()
        q = g.state["qpos"].double().cpu().numpy()
        pos = np.stack([q[:, a:a + 3] for a in qadr], 1)
        cl = classify(pos, names, ctr, half)
        spawn = {k: v.cpu().clone() for k, v in g.state.items()}
        # spawn probe: the first sub-steps from the reset state, one launch each
        pst = {k: v.clone() for k, v in g.state.items()}
        pmax = np.zeros((B, 3))
        pwarn = np.zeros(B, np.int64)
        for _ in range(args.probe):
            eng.step(pst, 1)
            qa = pst["qacc_warmstart"].double().abs().cpu().numpy()
            for i, d in enumerate(dadr):
                pmax[:, i] = np.maximum(pmax[:, i], qa[:, d:d + 6].max(1))
        pwarn = (pst["warn"].to(torch.int64) & 0xFFFF).cpu().numpy()
        acts = [policy_actions(args.policy, rng, B) for _ in range(args.steps)]
        smax = np.zeros((B, 3))
        first_bad = np.full(B, -1)
        bad_bits = np.zeros(B, np.int64)
        for k, a in enumerate(acts):
            g.step(torch.as_tensor(a, dtype=dt, device=g.device))
            w = (g.state["warn"].to(torch.int64) & 0x7).cpu().numpy()
            new = (w != 0) & (first_bad < 0)
            first_bad[new] = k
            bad_bits |= w
            qa = g.state["qacc_warmstart"].double().abs().cpu().numpy()
            for i, d in enumerate(dadr):
                smax[:, i] = np.maximum(smax[:, i], qa[:, d:d + 6].max(1))
            if args.far:
                fd, fn = far_contacts(eng, g, cube_geoms, qadr)
                far_max = max(far_max, fd)
                far_n += fn
        for b in np.nonzero(first_bad >= 0)[0]:
            ev = dict(episode=ep, env=int(b), step=int(first_bad[b]), bits=int(bad_bits[b]),
                      time_window=[0.5 + 0.5 * first_bad[b], 0.5 + 0.5 * (first_bad[b] + 1)],
                      spawn=[dict(cube=CUBES[i], pos=pos[b, i].tolist(), static_depth=float(cl["static_depth"][b, i]),
                                  static_box=str(cl["static_box"][b, i]), cube_depth=float(cl["cube_depth"][b, i]),
                                  floor_depth=float(cl["floor_depth"][b, i]), supported=bool(cl["supported"][b, i]))
                             for i in range(3)],
                      probe_qacc=pmax[b].tolist(), probe_warn=int(pwarn[b]))
            events.append(ev)
            print("EVENT", json.dumps(ev), flush=True)
            for kk, v in spawn.items():
                replay[kk].append(v[b].double().numpy() if kk != "warn" else v[b].numpy())
            replay["actions"].append(np.stack([a[b] for a in acts]))
            replay["episode"].append(ep)
            replay["env"].append(int(b))
        for i in range(3):
            rows.append(np.stack([np.full(B, ep), np.arange(B), np.full(B, i), pos[:, i, 0], pos[:, i, 1], pos[:, i, 2],
                                  cl["static_depth"][:, i], cl["cube_depth"][:, i], cl["floor_depth"][:, i],
                                  cl["supported"][:, i], pmax[:, i], smax[:, i], pwarn != 0,
                                  (bad_bits & 4) != 0], 1))
        nbad = int((first_bad >= 0).sum())
        print(f"episode {ep}: spawn in a static box {int((cl['static_depth'] > 1e-4).sum())}, in a cube "
              f"{int((cl['cube_depth'] > 1e-4).sum())}, unsupported {int((~cl['supported']).sum())} (of {3 * B} cubes); "
              f"probe max|qacc| {pmax.max():.3g}; step max|qacc| {smax.max():.3g}; bad-state envs {nbad}; "
              + (f"cube contacts farthest from the cube centre {far_max:.4f} m, beyond 0.05 m: {far_n}; " if args.far else "") +
              f"{time.time() - t0:.0f} s", flush=True)
    R = np.concatenate(rows)
    cols = ["episode", "env", "cube", "x", "y", "z", "static_depth", "cube_depth", "floor_depth", "supported",
            "probe_qacc", "step_qacc", "probe_warn", "badqacc"]
    summarize(R, cols, names, events)
    if args.out:
        np.savez_compressed(args.out, census=R, columns=np.array(cols), events=json.dumps(events),
                            **{f"replay_{k}": np.array(v) for k, v in replay.items()})


def far_contacts(eng, g, cube_geoms, qadr):
    """After a gym step: (the largest distance from a cube contact to that cube's centre, the number
    of such contacts beyond 0.05 m) over the envs' current contacts (forward_debug, full tier)."""
    from pnp_amd import _lib
    D = _lib.DBG
    dbg = eng.forward_debug(g.state).double().cpu().numpy()
    n = dbg[:, D["COUNTS"]].astype(int)
    q = g.state["qpos"].double().cpu().numpy()
    far, cnt = 0.0, 0
    K = int(n.max()) if n.size else 0
    if K == 0:
        return far, cnt
    con = dbg[:, D["CON"]:D["CON"] + 16 * K].reshape(-1, K, 16)
    valid = np.arange(K)[None] < n[:, None]
    for cg, a in zip(cube_geoms, qadr):
        hit = valid & ((con[..., 13] == cg) | (con[..., 14] == cg))
        d = np.linalg.norm(con[..., 0:3] - q[:, None, a:a + 3], axis=-1)
        d = np.where(hit, d, 0.0)
        far = max(far, float(d.max()))
        cnt += int((d > 0.05).sum())
        for e, k in zip(*np.nonzero(d > 0.05)):
            r = con[e, k]
            print(f"  far contact: env {e}, geoms {int(r[13])}-{int(r[14])}, {d[e, k]:.4f} m from the cube centre, "
                  f"dist {r[12]:.3g}, pos {np.round(r[0:3], 4)}, normal {np.round(r[3:6], 4)}", flush=True)
    return far, cnt


def summarize(R, cols, names, events):
    c = {k: i for i, k in enumerate(cols)}
    deep = R[:, c["static_depth"]] > 1e-4
    cc = R[:, c["cube_depth"]] > 1e-4
    fl = R[:, c["z"]] < 0.1
    uns = R[:, c["supported"]] == 0
    print(f"\ncube spawns: {len(R)}; penetrating a static box {deep.sum()} ({deep.mean():.3%}), a cube {cc.sum()}, "
          f"unsupported {uns.sum()} ({uns.mean():.3%}), on the floor {fl.sum()} ({fl.mean():.3%})")
    for lab, sel in (("all", np.ones(len(R), bool)), ("static-box spawn", deep), ("cube-cube spawn", cc),
                     ("unsupported", uns), ("floor", fl)):
        if sel.any():
            p = R[sel, c["probe_qacc"]]
            s = R[sel, c["step_qacc"]]
            print(f"  {lab:18s} n={sel.sum():7d}  probe max|qacc| p50 {np.median(p):.3g} p99 {np.quantile(p, 0.99):.3g} "
                  f"max {p.max():.3g}; after-step |qacc| max {s.max():.3g}")
    if deep.any():
        d = R[deep, c["static_depth"]]
        print(f"  static penetration depth: p50 {np.median(d):.4f} m, max {d.max():.4f} m")
    for cube in range(3):
        sel = R[:, c["cube"]] == cube
        print(f"  cube{cube + 1}: floor {fl[sel].mean():.2%}, static-box spawn {deep[sel].mean():.2%}, "
              f"|y| p50 {np.median(np.abs(R[sel, c['y']])):.3f} max {np.abs(R[sel, c['y']]).max():.3f}")
    print(f"bad-state events: {len(events)}")
    by = collections.Counter((e["step"], e["bits"]) for e in events)
    for (st, bits), n in sorted(by.items()):
        print(f"  gym step {st} (t in [{0.5 + 0.5 * st}, {1.0 + 0.5 * st}] s): {n} envs, bits "
              f"{'|'.join(v for k, v in BAD.items() if bits & k)}")


if __name__ == "__main__":
    main()
