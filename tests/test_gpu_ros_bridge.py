"""The ROS-message adapters on the HIP path, end to end: the batched env's
outputs go out as the messages the reference loop consumed and come back through the reference's
own callbacks into the drop-in FFMP methods, whose every call is a HIP launch — and must give the
env's own verdicts.

  env lidar row -> lidar_to_ranges (LaserScan.ranges) -> ranges_to_scan_data (laser_callback,
      /root/reference/src/train.py:145-150) -> FFMP.is_collision2 / FFMP.rewarder2
      (ffmp.py:108-117, :179-188; ffmp_scan_collision_f64 / ffmp_reward_done kernels)
  env frame -> frame_to_image (mono8) -> image_to_map (temporal_bev_image_callback, :116-121)
      -> FFMP.is_collision / FFMP.rewarder (ffmp.py:85-105, :167-176; ffmp_footprint_collision)
  env pose -> pose_to_odometry -> odometry_to_pose (robot_position_extractor, :157-165) ->
      relative_goal (relative_goal_calculator, :174-180) -> the `relative_goal_info` argument

At the reference's map size (G = 100, 5 m, 0.05 m cells) with 180 beams, in a crowded world so that
lidar and footprint collisions, goals and sensors inside discs all occur.  The env's collision is
footprint OR lidar; the bridge's verdicts must compose to it exactly, and its rewards
equal the env's float32 rewards, for every env and step — except that a beam starting inside a
disc (-inf in the env) has no LaserScan encoding (it goes out as 0.0, which laser_callback drops),
so for those envs only the footprint / combined verdicts are compared (documented in
ros_adapters.lidar_to_ranges)."""
import contextlib
import io

import numpy as np
import pytest
import torch

from flow_field_based_motion_planner_amd import env as envmod
from flow_field_based_motion_planner_amd import ros_adapters as R
from flow_field_based_motion_planner_amd.config import FFMPConfig
from flow_field_based_motion_planner_amd.vec_env import FFMPVec

pytestmark = pytest.mark.gpu

N, STEPS = 40, 24
CFG = FFMPConfig(grid=100, n_obst=14, n_beams=180, moving=True, autoreset=False, obst_rmax=0.45, obst_vmax=1.5,
                 start_clear=-0.3, goal_clear=0.05, goal_min=0.3, goal_max=1.2, world_half=2.5, max_steps=200,
                 seed=61)


def _f32(x) -> np.float32:
    return np.float32(x)


def test_env_messages_through_the_reference_callbacks_into_ffmp():
    env = FFMPVec(N, CFG, device="cuda:0")
    ffmp = envmod.FFMP(verbose=False)          # the reference's 100 x 100 / 5 m footprint
    envmod._reset_global_d0()
    env.reset()
    rng = np.random.default_rng(5)
    d0 = {}                                     # per env: the d0 its is_first rewarder2 call stored
    seen = {"lidar_col": 0, "foot_col": 0, "foot_only": 0, "goal": 0, "inside": 0, "first_calls": 0}
    stamp = 0.0

    def rel_goal(i):
        pose = env.pose[i].cpu().numpy()
        odo = R.pose_to_odometry(float(pose[0]), float(pose[1]), float(pose[2]), stamp)
        x, y, yaw, _ = R.odometry_to_pose(odo)
        gx, gy = (float(v) for v in env.goal[i].cpu().numpy())
        return R.relative_goal(x, y, yaw, gx, gy)

    def scan_of(i):
        return R.ranges_to_scan_data(R.lidar_to_ranges(env.lidar[i].cpu().numpy(), CFG.lidar_range))

    def first_calls(ids):
        # the reference loop's is_first iteration on the reset observation: rewarder2 stores the
        # episode-start distance in the module global (ffmp.py:139-141); the env keeps it per env
        for i in ids:
            rel = rel_goal(i)
            with contextlib.redirect_stdout(io.StringIO()):
                ffmp.rewarder2(scan_of(i), rel, True)
            d0[i] = envmod._PRE_RELATIVE_GOAL_DIST
            assert d0[i] == float(env.d0[i]), (i, d0[i], float(env.d0[i]))
            seen["first_calls"] += 1

    first_calls(range(N))
    for s in range(STEPS):
        stamp += CFG.dt
        env.step(torch.as_tensor(rng.integers(0, 28, N), device="cuda:0"))
        torch.cuda.synchronize()
        lidar = env.lidar.cpu().numpy()
        frames = env.state_m[:, 1].cpu().numpy()
        col, goal, done, trunc = (getattr(env, k).cpu().numpy() for k in ("collision", "is_goal", "done", "truncated"))
        reward = env.reward.cpu().numpy()
        state_g = env.state_g.cpu().numpy()
        for i in range(N):
            row = lidar[i]
            inside = bool(np.isneginf(row).any())
            lidar_col = bool(((row != 0) & (row.astype(np.float64) < CFG.robot_r)).any())  # the env's rule
            scan = scan_of(i)
            rel = rel_goal(i)
            assert abs(rel[0] - state_g[i, 0]) <= 1e-5 and abs(R._wrap_pi(rel[1] - state_g[i, 1])) <= 1e-5, i
            # occupancy: frame -> mono8 image -> the callback's float map -> FFMP.is_collision
            img_map = R.image_to_map(R.frame_to_image(frames[i]))          # (1, G, G) float32 0..255
            local_map = np.transpose(img_map, (1, 2, 0)).astype(np.int32)  # the env's (G, G, 1) int32
            foot_col = ffmp.is_collision(local_map)
            assert bool(col[i]) == (foot_col or lidar_col), (s, i, foot_col, lidar_col)
            ros_col = ffmp.is_collision2(scan)
            if not inside:
                assert ros_col == lidar_col, (s, i)
            envmod._PRE_RELATIVE_GOAL_DIST = d0[i]   # this env's episode (the global is shared)
            r2, done2, goal2 = ffmp.rewarder2(scan, rel, False)
            assert goal2 == bool(goal[i]) and done2 == (ros_col or goal2), (s, i)
            r1, done1 = ffmp.rewarder(local_map, rel, False)
            assert done1 == (foot_col or goal2), (s, i)
            # rewards: the bridge call whose collision source is the env's own verdict
            if not foot_col and not inside:
                assert _f32(r2) == reward[i], (s, i, r2, reward[i])
            if not lidar_col:
                assert _f32(r1) == reward[i], (s, i, r1, reward[i])
            assert _f32(ffmp.reward_calculator(rel, bool(col[i]), bool(goal[i]), False)) == reward[i], (s, i)
            assert bool(done[i]) == (bool(col[i]) or bool(goal[i]) or bool(trunc[i]))
            seen["lidar_col"] += lidar_col
            seen["foot_col"] += foot_col
            seen["foot_only"] += foot_col and not lidar_col
            seen["goal"] += bool(goal[i])
            seen["inside"] += inside
        ended = np.flatnonzero(done)
        if len(ended):  # the episode manager's reset of finished envs (train.py:611-664)
            m = torch.zeros(N, dtype=torch.bool, device="cuda:0")
            m[torch.as_tensor(ended, device="cuda:0")] = True
            env.reset(mask=m)
            torch.cuda.synchronize()
            first_calls(ended.tolist())
    assert seen["lidar_col"] > 0 and seen["foot_col"] > 0 and seen["goal"] > 0 and seen["inside"] > 0, seen
    print(seen)
