"""SE(3) helpers of R/path_planner/utils/transformation.py:7-93 (numpy)."""
import math

import numpy as np


def eulerAnglesToRotationMatrix(theta):
    R_x = np.array([[1, 0, 0], [0, math.cos(theta[0]), -math.sin(theta[0])],
                    [0, math.sin(theta[0]), math.cos(theta[0])]])
    R_y = np.array([[math.cos(theta[1]), 0, math.sin(theta[1])], [0, 1, 0],
                    [-math.sin(theta[1]), 0, math.cos(theta[1])]])
    R_z = np.array([[math.cos(theta[2]), -math.sin(theta[2]), 0], [math.sin(theta[2]), math.cos(theta[2]), 0],
                    [0, 0, 1]])
    return np.dot(R_z, np.dot(R_y, R_x))


def rotationMatrixToEulerAngles(R):
    sy = math.sqrt(R[0, 0] * R[0, 0] + R[1, 0] * R[1, 0])
    if not sy < 1e-6:
        return np.array([math.atan2(R[2, 1], R[2, 2]), math.atan2(-R[2, 0], sy), math.atan2(R[1, 0], R[0, 0])])
    return np.array([math.atan2(-R[1, 2], R[1, 1]), math.atan2(-R[2, 0], sy), 0])


def states2SE3(states):
    x, y, z, roll, pitch, yaw = states
    T = np.diag([1.0, 1.0, 1.0, 1.0])
    T[:3, :3] = eulerAnglesToRotationMatrix([roll, pitch, yaw])
    T[:3, 3] = [x, y, z]
    return T


def SE32states(T):
    s = np.zeros(6)
    s[3:] = rotationMatrixToEulerAngles(T[:3, :3])
    s[:3] = T[:3, 3]
    return s


def xyz2homo(xyz):
    return np.concatenate([xyz, np.ones([len(xyz), 1])], axis=1)
