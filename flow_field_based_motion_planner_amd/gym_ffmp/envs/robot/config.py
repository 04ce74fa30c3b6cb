"""Robot model of src/gym_ffmp/envs/robot/config.py:6-58.

The 28 commands are the product of the literal speed lists (never computed:
0.6 != 3*0.2 in binary), cmd[7*vi + wi] = (V[vi], W[wi])."""
from ....config import CMD_V, CMD_W


class RobotPose(object):
    def __init__(self, x, y, yaw):
        self.x = x
        self.y = y
        self.yaw = yaw


class RobotVelocity(object):
    def __init__(self, linear_v, angular_v):
        self.linear_v = linear_v
        self.angular_v = angular_v


class RobotState(object):
    def __init__(self, x, y, yaw, linear_v, angular_v):
        self.robot_position = RobotPose(x, y, yaw)
        self.robot_velocity = RobotVelocity(linear_v, angular_v)


class RobotAction(object):
    def __init__(self):
        self.cmd = [RobotVelocity(v, w) for v in CMD_V for w in CMD_W]

    def commander(self, i):
        return self.cmd[i]
