"""Where the fused learner's chain kernels spend their time (GPU; a diagnostic build of libpnp.so
with PNP_DEFS=-DPNP_TQC_STAMPS=1, loaded with PNP_LIB): thread 0 of one workgroup per kernel stamps
the shader clock after every layer (csrc/tqc_fused.hip tqc_stamp) into columns 240..255 of the
workspace's per-row records 0..3, which nothing reads.  Printed per kernel: cycles from the kernel's
start at each stamp, the step between stamps, and the clock (GHz) over the workgroup's lifetime.
usage: PNP_LIB=... python tools/tqc_stamps.py [steps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
from pnp_amd.envs import BatchedFrankaShelfPNPEnv, EnvConfig  # noqa: E402
from pnp_amd.tqc import TQC, TQCConfig  # noqa: E402

M_SM, HID = 24, 256
KERNELS = ("tqc_fwd (slab 0, job 3: actor(next_obs) + target critic 0)", "tqc_critic_bwd (slab 0, critic 0)",
           "tqc_pi_critic (slab 0, critic 0)", "tqc_actor_bwd (slab 0)")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    env = BatchedFrankaShelfPNPEnv(64, config=EnvConfig(n_substeps=2, n_calls=2))
    a = TQC(env, TQCConfig(fused=True))
    a.total_timesteps = 10 ** 6
    a.reset()
    for _ in range(12):
        a.collect_step()
    a.train(n)
    torch.cuda.synchronize()
    B = a.cfg.batch_size
    ws = a._fws
    for r, name in enumerate(KERNELS):
        o = (M_SM * B + r) * HID + 240
        v = ws[o:o + 16].cpu().tolist()
        st = [x for x in v[:15] if x > 0]
        steps = [st[0]] + [st[i] - st[i - 1] for i in range(1, len(st))]
        print(f"{name}: {len(st)} stamps, total {st[-1]:.0f} cycles, clock {v[15] / 10:.2f} GHz")
        print("   at   " + " ".join(f"{x:7.0f}" for x in st))
        print("   step " + " ".join(f"{x:7.0f}" for x in steps))
    wgrad_stamps(a)


def wgrad_stamps(a):
    """the critic pass's weight-gradient workgroups: (start, product done, end, loads landed), 100 MHz ticks"""
    import numpy as np
    B = a.cfg.batch_size
    base = 25 * B * HID + (B // 16) * 8
    v = a._fws[base:base + 4096].cpu().numpy().reshape(-1, 4)
    v = v[v[:, 2] > 0]
    t0 = v[:, 0].min()
    st, pd, en = (v[:, 0] - t0) * 0.01, (v[:, 1] - v[:, 0]) * 0.01, (v[:, 2] - v[:, 0]) * 0.01   # us
    ld = (v[:, 3] - v[:, 0]) * 0.01
    print(f"wgrad loads landed (wave 0) p10/50/90/max {np.percentile(ld, [10, 50, 90, 100]).round(2).tolist()} us")
    print(f"wgrad (critic pass): {len(v)} workgroups; span {(v[:, 2].max() - t0) * 0.01:.2f} us; start offsets "
          f"p10/50/90/max {np.percentile(st, [10, 50, 90, 100]).round(2).tolist()} us; product "
          f"{np.percentile(pd, [10, 50, 90, 100]).round(2).tolist()} us; whole workgroup "
          f"{np.percentile(en, [10, 50, 90, 100]).round(2).tolist()} us")


if __name__ == "__main__":
    main()
