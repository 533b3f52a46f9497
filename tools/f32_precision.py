"""fp32 step precision on identical inputs, per kinematic tree (diagnostic; tests/test_step_gpu.py
asserts the bar).  The fp64 oracle is fed the fp32-rounded state (north_star: "a single step on
identical (qpos, qvel, ctrl)"), so input rounding is not counted as kernel error.

Per fixture and tree (arm 0:9, cube1..3, dummy): relative error of the stepped velocity change
dqvel = qvel' - qvel (scale: the tree's own max |dqvel_ref|, floored at h*|g|), of M dqacc from
forward_debug (scale: max |M qacc_ref| over the tree, floored at the tree's weight force), and the
fp64 kernel's error for reference.   usage: python tools/f32_precision.py [nsub]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd"), os.path.join(ROOT, "tests")]
from oracle import oracle as O  # noqa: E402
from pnp_amd import _lib  # noqa: E402
from pnp_amd.engine import get_engine  # noqa: E402
import physics_states as PS  # noqa: E402

D = _lib.DBG
TREES = {"arm": slice(0, 9), "cube1": slice(9, 15), "cube2": slice(15, 21), "cube3": slice(21, 27),
         "dummy": slice(27, 33)}


def round32(st):
    return {k: (v.copy() if k == "warn" else v.astype(np.float32).astype(np.float64)) for k, v in st.items()}


def dev(st, dt):
    return {k: (torch.as_tensor(v.astype(np.int32), device="cuda") if k == "warn" else
                torch.as_tensor(np.ascontiguousarray(v), dtype=dt, device="cuda").contiguous()) for k, v in st.items()}


def host(g):
    return {k: v.cpu().numpy().astype(np.uint32 if k == "warn" else np.float64) for k, v in g.items()}


def fixtures(model):
    import test_step_gpu as T
    sc = PS.settled_states(24, seed=0, nsettle=60, model=model)
    PS.random_ctrl(sc, model=model)
    sc["qvel"] += np.random.default_rng(3).normal(size=sc["qvel"].shape) * 0.05
    fr = PS.reset_states(16, seed=7, model=model)
    fr["qpos"][:, 7:9] = 0.004
    pr = PS.reset_states(12, seed=11, model=model)
    pr["qpos"][:, 7:9] = -np.linspace(0.001, 0.004, 12)[:, None]
    pr["ctrl"][:, -2:] = 0.0
    pr["qvel"] += np.random.default_rng(5).normal(size=pr["qvel"].shape) * 0.02
    return {"scene": sc, "fresh": fr, "mesh_scene": T.mesh_states(model), "pressed": pr}


def main():
    nsub = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    eng = get_engine()
    m = eng.model
    nv, h = m.nv, float(m.opt_timestep)
    g = float(np.linalg.norm(m.opt_gravity))
    for name, st in fixtures(m).items():
        st = round32(st)
        ref = PS.copy_state(st)
        O.step(ref, nsub=nsub, nthreads=8, model=m)
        res = {}
        for dt in (torch.float32, torch.float64):
            gg = host(eng.step(dev(st, dt), nsub))
            dq_r, dq_g = ref["qvel"] - st["qvel"], gg["qvel"] - st["qvel"]
            e = {}
            for t, sl in TREES.items():
                scale = np.maximum(np.abs(dq_r[:, sl]).max(axis=1), h * g * nsub)
                e[t] = float((np.abs(dq_g[:, sl] - dq_r[:, sl]).max(axis=1) / scale).max())
            res[dt] = e
            res[(dt, "warn")] = bool(np.array_equal(gg["warn"], ref["warn"]))
        # the tests' measure: dqvel error in the tree's kinetic-energy norm ||v||_M = sqrt(v' M_t v),
        # relative to ||dqvel_ref||_M floored at the gravity step of the tree's mass, h |g| sqrt(m_t)
        g32 = host(eng.step(dev(st, torch.float32), nsub))
        mn = {t: 0.0 for t in TREES}
        for b in range(st["qpos"].shape[0]):
            M = O.forward_fields({k: st[k][b] for k in O.STATE_KEYS}, ["qM"], model=m)["qM"].reshape(nv, nv)
            for t, sl in TREES.items():
                Mt = M[sl, sl]
                root = int(m.body_rootid[int(m.dof_bodyid[sl.start])])
                mt = float(m.body_subtreemass[root])
                dr = ref["qvel"][b, sl] - st["qvel"][b, sl]
                de = g32["qvel"][b, sl] - ref["qvel"][b, sl]
                nrm = lambda v: float(np.sqrt(max(v @ Mt @ v, 0.0)))
                mn[t] = max(mn[t], nrm(de) / max(nrm(dr), h * g * nsub * np.sqrt(mt)))
        dbg = eng.forward_debug(dev(st, torch.float32)).cpu().numpy()
        fe = {t: 0.0 for t in TREES}
        fe_nt = {t: 0.0 for t in TREES}
        B = st["qpos"].shape[0]
        for b in range(B):
            f = O.forward_fields({k: st[k][b] for k in O.STATE_KEYS}, ["qM", "qacc", "qacc_newton", "ncon"], model=m)
            M = f["qM"].reshape(nv, nv)
            for t, sl in TREES.items():
                mt = M[sl, sl].diagonal().max()
                for key, qa, qr in (("qacc", dbg[b, D["QACC"]:D["QACC"] + nv], f["qacc"]),
                                    ("newton", dbg[b, D["QACC_NEWTON"]:D["QACC_NEWTON"] + nv], f["qacc_newton"])):
                    fr_ = M @ qr
                    scale = max(np.abs(fr_[sl]).max(), mt * g)
                    err = np.abs((M @ (qa - qr))[sl]).max() / scale
                    tgt = fe if key == "qacc" else fe_nt
                    tgt[t] = max(tgt[t], float(err))
        fmt = lambda d: " ".join(f"{t}={v:.2e}" for t, v in d.items())
        print(f"[{name}] B={B} nsub={nsub}")
        print(f"  dqvel f32 : {fmt(res[torch.float32])}  warn_eq={res[(torch.float32, 'warn')]}")
        print(f"  dqvel f32 M-norm: {fmt(mn)}")
        print(f"  dqvel f64 : {fmt(res[torch.float64])}  warn_eq={res[(torch.float64, 'warn')]}")
        print(f"  M dqacc f32 (after noslip): {fmt(fe)}")
        print(f"  M dqacc f32 (Newton)      : {fmt(fe_nt)}", flush=True)


if __name__ == "__main__" and not os.environ.get("DATA_SOLVE"):
    main()


def data_vs_solver(name, st, eng, m):
    """Where the fp32 constrained-acceleration error comes from: re-solve the Newton problem in
    fp64 on the host from the fp32 kernel's own intermediates (qM, efc_J, efc_D, efc_aref,
    qacc_smooth; the oracle's active set) -- if that matches the oracle, the error is the fp32
    solver's; if not, it is in the data the solver is handed."""
    nv = m.nv
    st = round32(st)
    dbg = eng.forward_debug(dev(st, torch.float32)).cpu().numpy()
    worst = {"data_solve": 0.0, "kernel": 0.0, "aref": 0.0, "J": 0.0, "D": 0.0, "M": 0.0, "smooth": 0.0}
    for b in range(st["qpos"].shape[0]):
        f = O.forward_fields({k: st[k][b] for k in O.STATE_KEYS},
                             ["qM", "efc_J", "efc_D", "efc_aref", "qacc_smooth", "qacc_newton", "efc_type", "nefc", "ncon"],
                             model=m)
        ne = int(f["nefc"][0])
        g = dbg[b]
        if int(g[D["COUNTS"] + 1]) != ne:
            continue
        Mr, Jr = f["qM"].reshape(nv, nv), f["efc_J"].reshape(ne, nv)
        Mg = g[D["QM"]:D["QM"] + nv * nv].reshape(nv, nv)
        Jg = g[D["EFC_J"]:D["EFC_J"] + ne * nv].reshape(ne, nv)
        Dg, ag = g[D["EFC_D"]:D["EFC_D"] + ne], g[D["EFC_AREF"]:D["EFC_AREF"] + ne]
        sg = g[D["QACC_SMOOTH"]:D["QACC_SMOOTH"] + nv]
        qn = f["qacc_newton"]
        act = (Jr @ qn - f["efc_aref"] < 0) | (f["efc_type"] == 0)

        def solve(M, J, Dd, ar, a0):
            H = M + (J[act].T * Dd[act]) @ J[act]
            return np.linalg.solve(H, M @ a0 + J[act].T @ (Dd[act] * ar[act]))
        q_data = solve(Mg, Jg, Dg, ag, sg)
        # noslip (3 pyramid-pair Gauss-Seidel sweeps, oracle/physics.c solve_noslip) on the host in
        # fp64, fed (a) the oracle's own data, (b) the kernel's fp32 data and Newton result
        ty = f["efc_type"]
        pairs = [i for i in range(ne) if ty[i] == 6][::2]

        def noslip(M, J, Dd, ar, a0, qn_):
            jar = J @ qn_ - ar
            f0 = np.where((jar < 0) | (ty == 0), -Dd * jar, 0.0)
            A = J @ np.linalg.solve(M, J.T)
            bb = J @ a0 - ar
            f_ = f0.copy()
            for _ in range(3):
                for j in pairs:
                    r0, r1 = bb[j] + A[j] @ f_, bb[j + 1] + A[j + 1] @ f_
                    a00, a01, a10, a11 = A[j, j], A[j, j + 1], A[j + 1, j], A[j + 1, j + 1]
                    bc0, bc1 = r0 - (a00 * f_[j] + a01 * f_[j + 1]), r1 - (a10 * f_[j] + a11 * f_[j + 1])
                    mid = 0.5 * (f_[j] + f_[j + 1])
                    K1, K0 = a00 + a11 - a01 - a10, mid * (a00 - a11) + bc0 - bc1
                    y = 0.0 if K1 < 1e-15 else min(max(-K0 / K1, -mid), mid)
                    f_[j], f_[j + 1] = mid + y, mid - y
            return np.linalg.solve(M, M @ a0 + J.T @ f_)
        q_ref_ns = noslip(Mr, Jr, f["efc_D"], f["efc_aref"], f["qacc_smooth"], qn)
        q_dat_ns = noslip(Mg, Jg, Dg, ag, sg, g[D["QACC_NEWTON"]:D["QACC_NEWTON"] + nv])
        q_kern_ns = g[D["QACC"]:D["QACC"] + nv]
        # one kernel input at a time into the oracle's noslip (which input drives the error)
        qng = g[D["QACC_NEWTON"]:D["QACC_NEWTON"] + nv]
        subs = {"aref": (Mr, Jr, f["efc_D"], ag, f["qacc_smooth"], qn), "D": (Mr, Jr, Dg, f["efc_aref"], f["qacc_smooth"], qn),
                "J": (Mr, Jg, f["efc_D"], f["efc_aref"], f["qacc_smooth"], qn),
                "smooth": (Mr, Jr, f["efc_D"], f["efc_aref"], sg, qn), "newton": (Mr, Jr, f["efc_D"], f["efc_aref"], f["qacc_smooth"], qng),
                "M": (Mg, Jr, f["efc_D"], f["efc_aref"], f["qacc_smooth"], qn)}
        for key, args in subs.items():
            qx = noslip(*args)
            for i, (tn, tsl) in enumerate(TREES.items()):
                mt = Mr[tsl, tsl].diagonal().max()
                sc_t = max(np.abs((Mr @ q_ref_ns)[tsl]).max(), mt * 9.81)
                kk = f"sub_{key}_{tn}"
                worst[kk] = max(worst.get(kk, 0.0), np.abs((Mr @ (qx - q_ref_ns))[tsl]).max() / sc_t)
        for i, (tn, tsl) in enumerate(TREES.items()):
            mt = Mr[tsl, tsl].diagonal().max()
            sc_t = max(np.abs((Mr @ q_ref_ns)[tsl]).max(), mt * 9.81)
            worst.setdefault("ns_data_" + tn, 0.0)
            worst.setdefault("ns_kern_" + tn, 0.0)
            worst["ns_data_" + tn] = max(worst["ns_data_" + tn], np.abs((Mr @ (q_dat_ns - q_ref_ns))[tsl]).max() / sc_t)
            worst["ns_kern_" + tn] = max(worst["ns_kern_" + tn], np.abs((Mr @ (q_kern_ns - q_ref_ns))[tsl]).max() / sc_t)
        q_kern = g[D["QACC_NEWTON"]:D["QACC_NEWTON"] + nv]
        sl = slice(0, 9)
        scale = np.abs((Mr @ qn)[sl]).max()
        worst["data_solve"] = max(worst["data_solve"], np.abs((Mr @ (q_data - qn))[sl]).max() / scale)
        worst["kernel"] = max(worst["kernel"], np.abs((Mr @ (q_kern - qn))[sl]).max() / scale)
        worst["aref"] = max(worst["aref"], np.abs(ag - f["efc_aref"]).max() / np.abs(f["efc_aref"]).max())
        worst["J"] = max(worst["J"], np.abs(Jg - Jr).max() / np.abs(Jr).max())
        worst["D"] = max(worst["D"], (np.abs(Dg - f["efc_D"]) / np.abs(f["efc_D"])).max())
        worst["M"] = max(worst["M"], np.abs(Mg - Mr).max() / np.abs(Mr).max())
        worst["smooth"] = max(worst["smooth"], np.abs(Mr @ (sg - f["qacc_smooth"])).max() / np.abs(Mr @ f["qacc_smooth"]).max())
        # per-row aref error by type, rows of the weld (equality)
        if b == 0:
            e = f["efc_type"] == 0
            print(f"  [{name}] env0 weld rows aref ref {f['efc_aref'][e]}\n      gpu-ref {ag[e] - f['efc_aref'][e]}")
    print(f"  [{name}] arm M dqacc: host fp64 solve of the kernel's fp32 data {worst['data_solve']:.2e}, "
          f"kernel {worst['kernel']:.2e}; data rel errors: aref {worst['aref']:.2e} J {worst['J']:.2e} "
          f"D {worst['D']:.2e} M {worst['M']:.2e} M qacc_smooth {worst['smooth']:.2e}", flush=True)
    print(f"  [{name}] after noslip, host fp64 noslip on the kernel's data: " +
          " ".join(f"{k[8:]}={v:.2e}" for k, v in worst.items() if k.startswith("ns_data_")))
    for key in ("aref", "D", "J", "smooth", "newton", "M"):
        print(f"  [{name}] after noslip, oracle data but the kernel's {key:7s}: " +
              " ".join(f"{k.split('_')[-1]}={v:.2e}" for k, v in worst.items() if k.startswith(f"sub_{key}_")))
    print(f"  [{name}] after noslip, kernel:                              " +
          " ".join(f"{k[8:]}={v:.2e}" for k, v in worst.items() if k.startswith("ns_kern_")), flush=True)


if __name__ == "__main__" and os.environ.get("DATA_SOLVE"):
    eng = get_engine()
    for nm, s in fixtures(eng.model).items():
        if nm != "pressed":
            data_vs_solver(nm, s, eng, eng.model)
