"""Generator of tests/golden/vecnormalize_200k.json: the observation statistics sb3's VecNormalize
held after the reference's own TQC run (train.py, 200k steps) -- the only reference-held record of
real-MuJoCo state at gym-step boundaries.

The file is a pickle; it is NOT unpickled (nothing in it is executed or imported): pickletools.genops
walks its opcodes as data, and the float64 payloads of the RunningMeanStd arrays (numpy's
_reconstruct + __setstate__ with raw bytes, SHORT_BINBYTES / BINBYTES operands) and the BINFLOAT
counts are decoded with numpy.frombuffer / the opcode's own float.  The array a payload belongs to
is named by the SHORT_BINUNICODE keys that precede it (obs_rms: achieved_goal, desired_goal,
observation -- each a RunningMeanStd with mean, var, count; then old_obs, the last observations of
the 4 SubprocVecEnv workers).  Runs in the build container only (/root/reference is absent on the
GPU box); the JSON it writes is the committed fixture.
usage: python tests/golden/make_vecnorm_fixture.py"""
import json
import os
import pickletools

import numpy as np

SRC = "/root/reference/scripts/checkpoints/tqc_dense_vecnormalize_200000_steps.pkl"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "vecnormalize_200k.json")


def main():
    data = open(SRC, "rb").read()
    keys, arrays, floats = [], [], []
    for op, arg, pos in pickletools.genops(data):
        if op.name in ("SHORT_BINUNICODE", "BINUNICODE"):
            keys.append((pos, arg))
        elif op.name in ("SHORT_BINBYTES", "BINBYTES") and len(arg) % 8 == 0 and len(arg) >= 8:
            arrays.append((pos, np.frombuffer(arg, dtype="<f8").tolist()))
        elif op.name == "BINFLOAT":
            floats.append((pos, arg))

    def after(name, start=0):
        return next(p for p, k in keys if k == name and p > start)

    # the key strings are memoised after their first use (later RunningMeanStd fields refer back to
    # them), so the arrays are taken in order: after "obs_rms" the mean / var payloads of
    # achieved_goal (3), desired_goal (3) and observation (19), and the three BINFLOAT counts
    rms = after("obs_rms")
    arr = [a for q, a in arrays if q > rms]
    cnt = [v for q, v in floats if q > rms]
    out = {"source": "scripts/checkpoints/tqc_dense_vecnormalize_200000_steps.pkl (pickletools.genops, never unpickled)",
           "obs_rms": {}}
    for i, (key, n) in enumerate((("achieved_goal", 3), ("desired_goal", 3), ("observation", 19))):
        mean, var = arr[2 * i], arr[2 * i + 1]
        assert len(mean) == n and len(var) == n, (key, len(mean), len(var))
        out["obs_rms"][key] = {"mean": mean, "var": var, "count": cnt[i]}
    p = after("old_obs")
    old = [np.array(a) for q, a in arrays if q > p]
    out["old_obs"] = {"achieved_goal": old[0].reshape(4, 3).tolist(), "desired_goal": old[1].reshape(4, 3).tolist(),
                      "observation": old[2].reshape(4, 19).tolist()}
    # the observation's 19 columns (panda_env.py _get_obs:279-301)
    out["observation_columns"] = ["ee_pos_x", "ee_pos_y", "ee_pos_z", "ee_vel_x", "ee_vel_y", "ee_vel_z", "fingers_width",
                                  "obj_pos_x", "obj_pos_y", "obj_pos_z", "obj_rot_x", "obj_rot_y", "obj_rot_z",
                                  "obj_velp_x", "obj_velp_y", "obj_velp_z", "obj_velr_x", "obj_velr_y", "obj_velr_z"]
    with open(OUT, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out["obs_rms"]["observation"]))


if __name__ == "__main__":
    main()
