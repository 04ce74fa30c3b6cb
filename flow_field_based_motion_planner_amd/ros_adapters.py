"""ROS-message adapters: the batched env's tensors <-> the messages the reference loop consumed
and produced (src/train.py:82-165), for a sim-to-real bridge.

No rospy here (not installed; nothing runs a ROS graph): messages are duck-typed — any object
with the fields rospy messages have works, and `Msg` is a minimal stand-in for tests.  The
conversions keep the reference's exact semantics:

  laser_callback (:145-150)          ranges_to_scan_data: keep r with `r != inf and r` — NaN
                                     is kept, 0.0 and +inf are dropped — appended to a list
                                     that starts as [None] (:97) and grows across callbacks
  temporal_bev_image_callback        image_to_map: mono8 image (H, W) -> float32 (1, H, W),
    (:116-121)                       raw 0..255 (kornia.image_to_tensor(keepdim=True).float())
  robot_position_extractor           odometry_to_pose: (x, y, yaw) with yaw from the quaternion
    (:157-165)                       (tf euler_from_quaternion, axes 'sxyz'), stamp -> seconds
  pose_array_callback (:126-132)     pose_array_to_start_goal: poses[0], poses[1]
  relative_goal_calculator           relative_goal: [sqrt(dx^2 + dy^2), pi_to_pi(atan2(dy, dx)
    (:167-180)                       - yaw)] in float64, the `relative_goal_info` rewarder2 takes
  cmd_vel_publisher (:134-143)       action_to_twist: RobotAction.cmd[a] -> linear.x, angular.z

and the other direction, env -> messages: lidar_to_ranges, frame_to_image, pose_to_odometry.
Host-side (numpy): a bridge talks to one robot at a time.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .config import action_table


class Msg:
    """Minimal attribute bag standing in for a rospy message (nested via keyword dicts)."""

    def __init__(self, **kw):
        for k, v in kw.items():
            setattr(self, k, Msg(**v) if isinstance(v, dict) else v)

    def __repr__(self):
        return f"Msg({', '.join(f'{k}={v!r}' for k, v in vars(self).items())})"


# ----------------------------------------------------------------------------- sensor -> env
def ranges_to_scan_data(ranges: Sequence[float], scan_data: Optional[List] = None) -> List:
    """laser_callback (train.py:145-150): append every range that is `!= inf` and truthy."""
    out = [None] if scan_data is None else scan_data
    for r in ranges:
        if r != float("inf") and r:
            out.append(r)
    return out


def image_to_map(img: np.ndarray) -> np.ndarray:
    """temporal_bev_image_callback (train.py:116-121): mono8 (H, W) -> float32 (1, H, W), 0..255."""
    a = np.asarray(img)
    if a.ndim == 2:
        a = a[None]
    elif a.ndim == 3:
        a = np.transpose(a, (2, 0, 1))  # HWC -> CHW, as kornia.image_to_tensor
    else:
        raise ValueError("image must be (H, W) or (H, W, C)")
    return a.astype(np.float32)


def quaternion_to_yaw(x: float, y: float, z: float, w: float) -> float:
    """Yaw of tf.transformations.euler_from_quaternion([x, y, z, w]) (static 'sxyz' axes):
    atan2(M[1,0], M[0,0]) of the normalised rotation matrix, 0 in gimbal lock or for a
    (near-)zero quaternion (tf returns the identity matrix there).  tf is not installed here,
    so this restates its published algorithm (ulp-level agreement; parity unpinned)."""
    eps = 4.0 * float(np.finfo(float).eps)  # tf's _EPS
    n = x * x + y * y + z * z + w * w
    if n < eps:
        return 0.0
    s = 2.0 / n
    m10 = s * (x * y + z * w)
    m00 = 1.0 - s * (y * y + z * z)
    if math.sqrt(m00 * m00 + m10 * m10) > eps:
        return math.atan2(m10, m00)
    return 0.0


def odometry_to_pose(msg) -> Tuple[float, float, float, float]:
    """robot_position_extractor (train.py:157-165): (x, y, yaw, stamp seconds)."""
    p = msg.pose.pose.position
    q = msg.pose.pose.orientation
    st = msg.header.stamp
    t = float(st.to_sec()) if hasattr(st, "to_sec") else float(st.secs) + 1e-9 * float(st.nsecs)
    return float(p.x), float(p.y), quaternion_to_yaw(q.x, q.y, q.z, q.w), t


def pose_array_to_start_goal(msg) -> Tuple[Tuple[float, float], Tuple[float, float]]:
    """pose_array_callback (train.py:126-132): start = poses[0], goal = poses[1] (x, y)."""
    s, g = msg.poses[0].position, msg.poses[1].position
    return (float(s.x), float(s.y)), (float(g.x), float(g.y))


def _wrap_pi(a: float) -> float:
    """ROSNode.pi_to_pi (train.py:167-172): subtract 2pi while >= pi, then add 2pi while <= -pi
    (so both +pi and -pi end at +pi); iterative on purpose — a remainder differs in the last bits."""
    two_pi = 2 * math.pi
    while a >= math.pi:
        a -= two_pi
    while a <= -math.pi:
        a += two_pi
    return a


def relative_goal(x: float, y: float, yaw: float, goal_x: float, goal_y: float) -> np.ndarray:
    """relative_goal_calculator (train.py:174-180) on a pose (e.g. from odometry_to_pose) and the
    goal of pose_array_to_start_goal: float64 [dist, orientation], the `relative_goal_info` that
    FFMP.rewarder / rewarder2 consume (train.py:536, :577)."""
    dx, dy = goal_x - x, goal_y - y
    return np.array([math.sqrt(dx * dx + dy * dy), _wrap_pi(math.atan2(dy, dx) - yaw)])


def action_to_twist(action: int) -> Msg:
    """cmd_vel_publisher(commander(a)) (train.py:134-143, :668-673)."""
    v, w = action_table()[int(action)]
    return Msg(linear={"x": v, "y": 0.0, "z": 0.0}, angular={"x": 0.0, "y": 0.0, "z": w})


# ----------------------------------------------------------------------------- env -> messages
def lidar_to_ranges(lidar_row: np.ndarray, range_max: float) -> List[float]:
    """One env's lidar (L,) as LaserScan.ranges: no return (+inf) stays inf (dropped by
    laser_callback), a beam starting inside a disc (-inf) becomes 0.0 (also dropped, as
    is_collision2 skips falsy ranges), everything else is the float32 range."""
    r = np.asarray(lidar_row, dtype=np.float32)
    out = np.where(np.isneginf(r), 0.0, r).astype(np.float64)
    out = np.where(out > range_max, np.inf, out)
    return [float(v) for v in out]


def frame_to_image(frame: np.ndarray) -> np.ndarray:
    """One (G, G) occupancy frame (0/255 float) as a mono8 image (H = G rows)."""
    f = np.asarray(frame)
    if f.ndim != 2:
        raise ValueError("frame must be (G, G)")
    return np.clip(f, 0, 255).astype(np.uint8)


def yaw_to_quaternion(yaw: float) -> Tuple[float, float, float, float]:
    """(x, y, z, w) of a rotation by `yaw` about z (tf quaternion_from_euler(0, 0, yaw))."""
    return 0.0, 0.0, math.sin(0.5 * yaw), math.cos(0.5 * yaw)


def pose_to_odometry(x: float, y: float, yaw: float, stamp: float) -> Msg:
    qx, qy, qz, qw = yaw_to_quaternion(yaw)
    secs = int(math.floor(stamp))
    return Msg(header={"stamp": {"secs": secs, "nsecs": int(round((stamp - secs) * 1e9))}},
               pose={"pose": {"position": {"x": x, "y": y, "z": 0.0},
                              "orientation": {"x": qx, "y": qy, "z": qz, "w": qw}}})
