"""Stage profile of the gym workload: B FrankaShelfPNPDense envs driven by random (or saturated
constant +-1) actions for a few fused gym steps, then the reached states are stepped 25 sub-steps
with the per-stage shader clocks (pnp_step_profile) and timed with plain pnp_step; prints the
per-env contact distribution and the stage cycles.  PNP_STEP_COMPACT=0 profiles the full kernel
alone.  usage: python tools/gym_profile.py [B] [gym_steps] [uniform|saturated]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
from pnp_amd.engine import Engine, get_engine  # noqa: E402
from pnp_amd.envs import BatchedFrankaShelfPNPEnv  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    mode = sys.argv[3] if len(sys.argv) > 3 else "uniform"
    torch.cuda.set_device(0)
    eng = get_engine()
    env = BatchedFrankaShelfPNPEnv(B, engine=eng, autoreset=False)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(3)
    const = torch.sign(torch.rand(B, 7, device="cuda", generator=g) * 2 - 1)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for k in range(n):
        a = const if mode == "saturated" else torch.rand(B, 7, device="cuda", generator=g) * 2 - 1
        ev0.record()
        env.step(a)
        ev1.record()
        torch.cuda.synchronize()
        print(f"gym step {k}: {ev0.elapsed_time(ev1):.1f} ms", flush=True)
    warn = env.state["warn"]
    print(f"envs with CONTACTFULL: {int(((warn & 8) != 0).sum())} / {B}", flush=True)
    st0 = {k: v.clone() for k, v in env.state.items()}
    st0["warn"].zero_()
    nsub = 25
    times = []
    for _ in range(3):
        st = {k: v.clone() for k, v in st0.items()}
        ev0.record()
        eng.step(st, nsub)
        ev1.record()
        torch.cuda.synchronize()
        times.append(ev0.elapsed_time(ev1))
    ms = float(np.median(times))
    print(f"pnp_step x{nsub} on the reached states: {ms:.2f} ms -> {B * nsub / ms / 1e3:.3f} M env-steps/s "
          f"(PNP_STEP_COMPACT={os.environ.get('PNP_STEP_COMPACT', '1')})", flush=True)
    st = {k: v.clone() for k, v in st0.items()}
    prof = eng.step_profile(st, nsub).cpu().numpy().astype(np.float64)
    names = Engine.STAGES
    ic = names.index("n_con")
    ncon = prof[:, ic] / nsub
    q = np.percentile(ncon, [50, 90, 99, 100])
    print(f"contacts per env (mean over the sub-steps): p50 {q[0]:.1f} p90 {q[1]:.1f} p99 {q[2]:.1f} max {q[3]:.1f}; "
          f"> 20: {(ncon > 20).mean():.3f}  > 32: {(ncon > 32).mean():.3f}  > 40: {(ncon > 40).mean():.3f}")
    tot = prof[:, :Engine.N_STAGE_CYCLES].sum(0) / (B * nsub)
    allc = tot[:16].sum()
    print(f"per env per sub-step: {allc:.0f} cycles")
    for i in range(Engine.N_STAGE_CYCLES):
        print(f"  {names[i]:22s} {tot[i]:8.0f} cycles  {100 * tot[i] / allc:5.1f}%")
    for i in range(Engine.N_STAGE_CYCLES, len(names)):
        v = prof[:, i] / nsub
        if names[i].startswith("n_"):
            print(f"  {names[i]:22s} {v.mean():8.2f} per env-sub-step (max {v.max():.2f})")
    # heavy vs light envs: cycles per sub-step and the top stages of each bucket
    for lo, hi in ((0, 20), (20, 32), (32, 48), (48, 97)):
        sel = (ncon > lo) & (ncon <= hi)
        if sel.any():
            per = prof[sel, :Engine.N_STAGE_CYCLES].mean(0) / nsub
            c = per[:16].sum()
            top = sorted(range(Engine.N_STAGE_CYCLES), key=lambda i: -per[i])[:8]
            print(f"  envs with {lo} < contacts <= {hi}: {sel.mean():.3f} of envs, {c:.0f} cycles per sub-step; "
                  + ", ".join(f"{names[i]} {per[i]:.0f}" for i in top))
            cnt = prof[sel].mean(0) / nsub
            sub = ("noslip_W", "noslip_lists", "newton_gradient", "newton_hessian", "newton_converge",
                   "n_noslip_sweep", "n_efc", "n_newton_iter", "n_convex")
            print("      " + ", ".join(f"{k} {cnt[names.index(k)]:.1f}" for k in sub))
    # the slowest envs (the gym step's span is the slowest env's sub-step chain): every stage
    tot_env = prof[:, :16].sum(1)
    for b in np.argsort(-tot_env)[:4]:
        per = prof[b] / nsub
        top = sorted(range(Engine.N_STAGE_CYCLES), key=lambda i: -per[i])[:12]
        print(f"  slow env {b}: {per[:16].sum():.0f} cycles per sub-step, {ncon[b]:.1f} contacts; "
              + ", ".join(f"{names[i]} {per[i]:.0f}" for i in top))
        print("      " + ", ".join(f"{k} {per[names.index(k)]:.1f}" for k in names[Engine.N_STAGE_CYCLES:]
                                   if k.startswith("n_")))


if __name__ == "__main__":
    main()
