"""Drop-in for scripts/execute_pnp.py (BASELINE config C1): the pick-and-place behaviour-tree demo
on the single-env facade (reference scripts/execute_pnp.py:22-124).

    python -m pnp_amd.execute_pnp [--env FrankaShelfPNPDense-v0] [--max-tick 3000] [--sim-steps 5]
                                  [--task-sequence cube1,cube2,cube3] [--no-render]

Same flow as the reference: reset, 20 gym steps with the gripper opening, pick / place tasks from
the current site poses (build_pick_place_tasks, same offsets and the same scipy quaternions --
xyzw handed over as MuJoCo wxyz), build_pnp_tree(retry_pick=1), then ticks
with ``--sim-steps`` extra mj_step calls each until the tree succeeds.  Success is the tree's,
as in the reference (no placement check); ``run()`` also reports where the objects ended up.
Rendering is not part of this engine (``--render`` is refused).
"""
from __future__ import annotations

import argparse
import time

import numpy as np
from scipy.spatial.transform import Rotation as R

from .bt import Status, build_pnp_tree
from .envs import make

HOME_WPT = np.array([1.23843967, 0.0, 0.49740014])   # execute_pnp.py:38 (= FK at the neutral pose)


def build_pick_place_tasks(env):
    """execute_pnp.py:22-43."""
    u = env.unwrapped
    tasks = []
    for name in u.task_sequence:
        obj_pos = u._utils.get_site_xpos(u.model, u.data, f"{name}_site").copy()
        target_pos = u._utils.get_site_xpos(u.model, u.data, f"target_{name}").copy()
        obj_y = obj_pos[1]
        pick_meta = {
            "id": hash(name) % 10000,
            "delta_q": R.from_euler("y", -90, degrees=True).as_quat().tolist(),
            "approach_wpt1": obj_pos + np.array([-0.2, -obj_y, 0.05]),
            "obj_pos": obj_pos + np.array([0.015, 0.0, 0.0]),
            "approach_wpt2": obj_pos + np.array([0.0, 0.0, 0.06]),
        }
        place_meta = {
            "approach_wpt1": obj_pos + np.array([-0.20, -obj_y, 0.05]),
            "home_wpt": HOME_WPT.copy(),
            "rotate_back_quat": R.from_euler("y", 90, degrees=True).as_quat().tolist(),
            "approach_wpt2": target_pos + np.array([0.0, 0.0, 0.06]),
        }
        tasks.append({"pick_meta": pick_meta, "place_meta": place_meta})
    return tasks


def run_on(env, max_tick=3000, sim_steps=5, record_reward=False, skills=None):
    """execute_pnp.py:79-114 on an env that has been reset and given its task sequence: 20 gym
    steps with the gripper opening, the pick / place tasks from the current site poses,
    build_pnp_tree(retry_pick=1), then ticks with ``sim_steps`` extra mj_step's each until the tree
    succeeds.  ``skills``: the skill classes the tree builds (pnp_amd.bt.DEFAULT_SKILLS).
    Returns (success, ticks, rewards)."""
    u = env.unwrapped
    open_act = np.zeros(env.action_space.shape, dtype=np.float32)
    open_act[-1] = 1.0
    for _ in range(20):
        env.step(open_act)
    tasks = build_pick_place_tasks(env)
    tree = build_pnp_tree(env, [{"obj_meta": t["pick_meta"], "place_meta": t["place_meta"]} for t in tasks],
                          retry_pick=1, skills=skills)
    success, ticks, rewards = False, 0, []
    for t in range(max_tick):
        tree.tick()
        u._mujoco.mj_step(u.model, u.data, nstep=sim_steps)   # = sim_steps x mj_step(nstep=1)
        ticks = t + 1
        if record_reward:
            o = u._get_obs()
            rewards.append(float(u.compute_reward(o["achieved_goal"], o["desired_goal"], {})))
        if tree.root.status == Status.SUCCESS:
            success = True
            break
    return success, ticks, np.asarray(rewards)


def run(env_id="FrankaShelfPNPDense-v0", max_tick=3000, sim_steps=5, task_sequence=None, verbose=True,
        record_reward=False, env_index=0):
    """execute_pnp.py:46-124 without rendering.  Returns a dict: success, ticks, wall seconds,
    final object / target positions; with record_reward, also the step reward after every tick
    (_get_obs + compute_reward at the tick's end state, as test/reward_test.py:69-74 records it).
    ``env_index``: the env's Philox counter (the reset draws of env i of a batched run)."""
    env = make(env_id, env_index=env_index)
    env.reset()
    u = env.unwrapped
    u.task_sequence[:] = list(task_sequence) if task_sequence else ["cube1", "cube2", "cube3"]
    t0 = time.perf_counter()
    success, ticks, rewards = run_on(env, max_tick, sim_steps, record_reward)
    wall = time.perf_counter() - t0
    obj = {n: u._utils.get_site_xpos(u.model, u.data, f"{n}_site").copy() for n in u.task_sequence}
    tgt = {n: u._utils.get_site_xpos(u.model, u.data, f"target_{n}").copy() for n in u.task_sequence}
    if verbose:
        if success:
            print(f"[ok] Pick + Place + Home SUCCESS after {ticks} ticks ({wall:.1f} s)")
        else:
            print("[x] Pick + Place + Home did not succeed within limit")
        for n in u.task_sequence:
            print(f"    {n}: at {np.round(obj[n], 3)}, target {np.round(tgt[n], 3)}, "
                  f"distance {np.linalg.norm(obj[n] - tgt[n]):.3f} m")
    # the env's sticky warning bits (MuJoCo's data.warning): bad-state resets (1, 2, 4) and a full
    # contact / constraint buffer (8, 16: the physics dropped contacts MuJoCo would keep)
    warn = int(u.data.warn) & 0xFFFF
    env.close()
    return {"success": success, "ticks": ticks, "wall_s": wall, "objects": obj, "targets": tgt,
            "rewards": rewards, "warn": warn}


def main(argv=None):
    ap = argparse.ArgumentParser("Debug Pick and Place and Home")
    ap.add_argument("--env", default="FrankaShelfPNPDense-v0")
    ap.add_argument("--render", action="store_true")
    ap.add_argument("--no-render", dest="render", action="store_false")
    ap.add_argument("--max-tick", type=int, default=3000)
    ap.add_argument("--sim-steps", type=int, default=5)
    ap.add_argument("--fps", type=int, default=30)
    ap.add_argument("--task-sequence", type=str, default=None)
    args = ap.parse_args(argv)
    if args.render:
        raise SystemExit("rendering is not part of this engine: run with --no-render (the default)")
    seq = [s.strip() for s in args.task_sequence.split(",")] if args.task_sequence else None
    r = run(args.env, args.max_tick, args.sim_steps, seq)
    return 0 if r["success"] else 1


if __name__ == "__main__":
    raise SystemExit(main())
