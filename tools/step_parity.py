"""Exploratory GPU-vs-oracle comparison of mj_step stages (prints a report; tests/ hold the
asserted versions).  usage: python tools/step_parity.py [B]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd"), os.path.join(ROOT, "tests")]
from oracle import oracle as O  # noqa: E402
from pnp_amd import _lib  # noqa: E402
from pnp_amd.engine import get_engine  # noqa: E402
import physics_states as PS  # noqa: E402

D = _lib.DBG


def to_dev(st, dt):
    out = {}
    for k, v in st.items():
        if k == "warn":
            out[k] = torch.as_tensor(v.astype(np.int32), device="cuda")
        else:
            out[k] = torch.as_tensor(v, dtype=dt, device="cuda").contiguous()
    return out


def oracle_forward(st, b, fields):
    return O.forward_fields({k: st[k][b] for k in O.STATE_KEYS}, fields)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    t0 = time.time()
    st = PS.settled_states(B, seed=0, nsettle=50)
    PS.random_ctrl(st)
    st["qvel"] += np.random.default_rng(3).normal(size=st["qvel"].shape) * 0.05
    print(f"states ready in {time.time() - t0:.1f}s", flush=True)
    eng = get_engine()
    m = eng.model
    nv = m.nv
    for dt in (torch.float64, torch.float32):
        dbg = eng.forward_debug(to_dev(st, dt)).cpu().numpy()
        torch.cuda.synchronize()
        errs = {k: 0.0 for k in ("qM", "bias", "act", "qacc_smooth", "qacc", "efc_force", "efc_pos")}
        cnt_mis = 0
        for b in range(B):
            f = oracle_forward(st, b, ["qM", "qfrc_bias", "qfrc_actuator", "qacc_smooth", "qacc", "ncon", "nefc",
                                       "efc_force", "efc_pos", "solver_iter"])
            g = dbg[b]
            ncon, nefc, it = int(g[D["COUNTS"]]), int(g[D["COUNTS"] + 1]), int(g[D["COUNTS"] + 2])
            if ncon != int(f["ncon"][0]) or nefc != int(f["nefc"][0]):
                cnt_mis += 1
                print(f"  env {b}: ncon {ncon} vs {int(f['ncon'][0])}, nefc {nefc} vs {int(f['nefc'][0])}")
                continue
            rel = lambda a, r: np.abs(a - r).max() / max(1.0, np.abs(r).max())
            errs["qM"] = max(errs["qM"], rel(g[D["QM"]:D["QM"] + nv * nv], f["qM"]))
            errs["bias"] = max(errs["bias"], rel(g[D["BIAS"]:D["BIAS"] + nv], f["qfrc_bias"]))
            errs["act"] = max(errs["act"], rel(g[D["ACT"]:D["ACT"] + nv], f["qfrc_actuator"]))
            errs["qacc_smooth"] = max(errs["qacc_smooth"], rel(g[D["QACC_SMOOTH"]:D["QACC_SMOOTH"] + nv], f["qacc_smooth"]))
            errs["qacc"] = max(errs["qacc"], rel(g[D["QACC"]:D["QACC"] + nv], f["qacc"]))
            errs["efc_force"] = max(errs["efc_force"], rel(g[D["EFC_FORCE"]:D["EFC_FORCE"] + nefc], f["efc_force"]))
            errs["efc_pos"] = max(errs["efc_pos"], rel(g[D["EFC_POS"]:D["EFC_POS"] + nefc], f["efc_pos"]))
        if dt == torch.float32:
            for b in range(min(B, 4)):
                f = oracle_forward(st, b, ["qacc", "qacc_smooth", "qacc_newton"])
                gn = dbg[b][D["QACC_NEWTON"]:D["QACC_NEWTON"] + nv]
                en = np.abs(gn - f["qacc_newton"])
                print(f"  env {b}: newton x err arm {en[:9].max():.2e} cubes {en[9:27].max():.2e} dummy {en[27:33].max():.2e}")
                g = dbg[b][D["QACC"]:D["QACC"] + nv]
                e = np.abs(g - f["qacc"])
                k = int(e.argmax())
                print(f"  env {b}: worst dof {k} ({m.names_jnt[m.dof_jntid[k]]}) gpu {g[k]:.6g} ref {f['qacc'][k]:.6g}; "
                      f"per-tree max err: arm {e[:9].max():.2e} c1 {e[9:15].max():.2e} c2 {e[15:21].max():.2e} "
                      f"c3 {e[21:27].max():.2e} dummy {e[27:33].max():.2e}")
        print(dt, "count mismatches", cnt_mis, {k: f"{v:.2e}" for k, v in errs.items()},
              "gpu iters", dbg[:, D["COUNTS"] + 2].mean(), flush=True)
    # one and ten steps
    for nsub in (1, 10):
        ref = PS.copy_state(st)
        O.step(ref, nsub=nsub, nthreads=8)
        for dt in (torch.float64, torch.float32):
            g = to_dev(st, dt)
            eng.step(g, nsub)
            torch.cuda.synchronize()
            dq = np.abs(g["qpos"].double().cpu().numpy() - ref["qpos"]).max()
            dv = np.abs(g["qvel"].double().cpu().numpy() - ref["qvel"]).max() / max(1, np.abs(ref["qvel"]).max())
            print(f"nsub {nsub} {dt}: max|dqpos| {dq:.2e}  rel dqvel {dv:.2e}  warn {g['warn'].cpu().numpy().max()}",
                  flush=True)
    # timing of the fp32 kernel
    for B2, nsub in ((4096, 10),):
        big = {k: torch.cat([v] * (B2 // B)) for k, v in to_dev(st, torch.float32).items()}
        eng.step(big, 1)
        torch.cuda.synchronize()
        t = time.time()
        eng.step(big, nsub)
        torch.cuda.synchronize()
        t = time.time() - t
        print(f"B={B2} nsub={nsub}: {t * 1e3:.1f} ms -> {B2 * nsub / t / 1e6:.3f} M env-steps/s", flush=True)




def profile_stages(B=4096, nsub=10, bench_inputs=False):
    eng = get_engine()
    if bench_inputs:
        import bench
        big, ctrl = bench.step_inputs(eng, eng.model, 0, B)
        big["ctrl"] = ctrl[0]
    else:
        st = PS.settled_states(64, seed=0, nsettle=50)
        PS.random_ctrl(st)
        big = {k: torch.cat([v] * (B // 64)) for k, v in to_dev(st, torch.float32).items()}
    keep = {k: v.clone() for k, v in big.items()}
    prof = eng.step_profile(big, nsub).cpu().numpy().astype(np.float64)
    nc = eng.N_STAGE_CYCLES
    tot = prof[:, :16].sum(1).mean()
    for rep in range(3):                         # the timed (non-profiling) kernel on the same inputs
        st2 = {k: v.clone() for k, v in keep.items()}
        torch.cuda.synchronize()
        t = time.time()
        eng.step(st2, nsub)
        torch.cuda.synchronize()
        t = time.time() - t
        print(f"step_kernel B={B} nsub={nsub}: {t * 1e3:.2f} ms -> {B * nsub / t / 1e6:.3f} M env-steps/s; "
              f"implied resident waves {B * nsub * tot / nsub / t / 2.4e9:.0f} (at 2.4 GHz)")
    print(f"per env per sub-step: {tot / nsub:.0f} cycles")
    for k, name in enumerate(eng.STAGES):
        if k < nc or name.startswith("aux"):
            if name.startswith("aux") and not prof[:, k].any():
                continue
            print(f"  {name:18s} {prof[:, k].mean() / nsub:10.0f} cycles  {100 * prof[:, k].mean() / tot:5.1f}%")
        else:
            print(f"  {name:18s} {prof[:, k].mean() / nsub:10.2f} per env-sub-step (max {prof[:, k].max() / nsub:.2f})")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "prof":
        profile_stages(bench_inputs=len(sys.argv) > 3 and sys.argv[3] == "bench")
    else:
        main()
