"""Mirror of src/gym_ffmp/envs/ffmp.py: module constants + the FFMP class."""
from ...env import (FFMP, GOAL_THRESHOLHD, MAP_CHANNELS, MAP_GRID_NUM, MAP_RANGE,  # noqa: F401
                    MAP_RESOLUTION, ROBOT_RSIZE)
from .robot.config import RobotAction, RobotPose, RobotState, RobotVelocity  # noqa: F401
