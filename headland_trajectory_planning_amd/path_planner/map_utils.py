"""Orchard map helpers of R/path_planner/utils/map_utils.py used by the
notebooks' warm-start cells (create_tree_rows :45-61, get_base_pose :228-271).
Random draws are made exactly as the reference makes them (one
np.random.uniform per row, even when l_std = 0)."""
import numpy as np

NEAR_SIDE = 1
FAR_SIDE = 2
LEAVE_POSE = 1
ENTER_POSE = 2


def plot_arrow(x, y, yaw, plt=None, length=1.0, width=0.5, fc="r", ec="k"):
    """Heading arrow(s) on a matplotlib axes (map_utils.py:14-31); plotting only."""
    if not isinstance(x, float):
        for ix, iy, iyaw in zip(x, y, yaw):
            plot_arrow(float(ix), float(iy), float(iyaw), plt, length, width, fc, ec)
        return
    plt.arrow(x, y, length * np.cos(yaw), length * np.sin(yaw), fc=fc, ec=ec, head_width=width, head_length=width)
    plt.plot(x, y)


def create_tree_rows(row_num, row_width, row_lengths, slope_angle=0, l_std=0.0):
    tree_rows = []
    delta_x = row_width * np.tan(slope_angle)
    for i in range(row_num):
        if isinstance(row_lengths, (list, np.ndarray)):
            row_length = row_lengths[i]
        else:
            row_length = row_lengths
        y = row_width * i
        x = delta_x * i
        x += np.random.uniform(-l_std, l_std)
        tree_rows.append(np.array([[x, y], [x + row_length, y]]))
    return np.array(tree_rows)


def get_base_pose(row_id, map_tree_rows, min_offset, side=NEAR_SIDE, pose_type=LEAVE_POSE):
    near_side_end = [(map_tree_rows[row_id, 0, 0] + map_tree_rows[row_id + 1, 0, 0]) / 2,
                     (map_tree_rows[row_id, 0, 1] + map_tree_rows[row_id + 1, 0, 1]) / 2]
    far_side_end = [(map_tree_rows[row_id, 1, 0] + map_tree_rows[row_id + 1, 1, 0]) / 2,
                    (map_tree_rows[row_id, 1, 1] + map_tree_rows[row_id + 1, 1, 1]) / 2]
    row_yaw = np.arctan2(far_side_end[1] - near_side_end[1], far_side_end[0] - near_side_end[0])
    if pose_type == LEAVE_POSE:
        pose_yaw = row_yaw if side == FAR_SIDE else row_yaw + np.pi
        extend_dir = 1
    else:
        pose_yaw = row_yaw + np.pi if side == FAR_SIDE else row_yaw
        extend_dir = -1
    end = near_side_end if side == NEAR_SIDE else far_side_end
    pos = end + np.array([np.cos(pose_yaw), np.sin(pose_yaw)]) * min_offset * extend_dir
    return np.array([pos[0], pos[1], pose_yaw])
