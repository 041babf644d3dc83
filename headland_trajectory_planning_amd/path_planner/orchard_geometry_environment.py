"""OrchardGeometryEnvironment of R/path_planner/orchard_geometry_environment.py
(shapely-free).

Tree rows, point obstacles and the field polygon are built as the reference's
GEOS buffers (geom.buffer_segment_flat / buffer_point_square) and exterior
points (get_map_exterior_pts :288-334).  Random draws (np.random.uniform in
check_side_of_a_point / create_headland_countour_lines) are made in the same
order so seeded notebooks reproduce.  check_path_feasibility answers the
reference's predicate on the host; the batched search evaluates the same
predicate on the GPU (libhtp.so, hastar_core.h).
"""
import math

import numpy as np

from .geom import Polygon, buffer_point_square, buffer_segment_flat, convex_intersects, ring_of, simple_contains


class OrchardGeometryEnvironment(object):
    NEAR_SIDE = 1
    FAR_SIDE = -1

    def __init__(self, map_tree_rows, obstacles, contour_points=[], tree_width=0.2, headland_width=7,
                 obstacle_dim=0.3):
        self.map_tree_rows = np.asarray(map_tree_rows, dtype=np.float64)
        self.tree_width = tree_width
        self.headland_width = headland_width
        self.tree_polys = self.create_row_polygons(tree_width)
        self.obstacle_polys = self.create_obstacle_polygons(obstacles, obstacle_dim)
        self.field_range_poly = self.create_field_polygon(headland_width, contour_points)
        self.contour_points = contour_points
        self.obs_poly_list = self.obstacle_polys + self.tree_polys

    def update_tree_width(self, new_tree_width):
        self.tree_polys = self.create_row_polygons(new_tree_width)
        self.obs_poly_list = self.obstacle_polys + self.tree_polys

    def check_side_of_a_point(self, point):
        """:49-64 (consumes len(rows) uniform draws)."""
        row_centers = np.mean(self.map_tree_rows[:, :, :], axis=1)
        epsilon = np.random.uniform(-0.5, 0.5, size=(len(row_centers),))
        self._center_line_coeff = np.polyfit(row_centers[:, 0] + epsilon, row_centers[:, 1], deg=1)
        k, b = self._center_line_coeff[0], self._center_line_coeff[1]
        origin_sign = np.sign(0 * k + b - 0)
        row_side_judge = np.sign(point[0] * k + b - point[1])
        return self.NEAR_SIDE if origin_sign == row_side_judge else self.FAR_SIDE

    def create_headland_countour_lines(self, field_range_poly):
        """:66-91."""
        row_centers = np.mean(self.map_tree_rows[:, :, :], axis=1)
        contour_points = ring_of(field_range_poly)
        epsilon = np.random.uniform(-0.5, 0.5, size=(len(row_centers),))
        self._center_line_coeff = np.polyfit(row_centers[:, 0] + epsilon, row_centers[:, 1], deg=1)
        k, b = self._center_line_coeff[0], self._center_line_coeff[1]
        self._origin_sign = np.sign(0 * k + b - 0)
        judges = np.sign(contour_points[:, 0] * k + b - contour_points[:, 1])
        near = np.where(judges == self._origin_sign)
        far = np.where((judges > self._origin_sign) | (judges < self._origin_sign))
        return contour_points[near], contour_points[far]

    def get_row_ids_between_start_and_end(self, start_pose, end_pose):
        """:93-127."""
        near_row_xs = self.map_tree_rows[:, 0, 0]
        near_row_ys = self.map_tree_rows[:, 0, 1]
        far_row_xs = self.map_tree_rows[:, 1, 0]
        far_row_ys = self.map_tree_rows[:, 1, 1]
        row_id = np.argmin(np.abs(start_pose[1] - near_row_ys))
        near = abs(start_pose[0] - near_row_xs[row_id]) < abs(start_pose[0] - far_row_xs[row_id])
        check_side_ys = np.copy(near_row_ys) if near else np.copy(far_row_ys)
        check_side_xs = np.copy(near_row_xs) if near else np.copy(far_row_xs)
        start_y, end_y = start_pose[1], end_pose[1]
        if start_y > end_y:
            idx = np.where((check_side_ys > end_y) & (check_side_ys < start_y))[0]
        else:
            idx = np.where((check_side_ys > start_y) & (check_side_ys < end_y))[0]
        return check_side_xs, check_side_ys, idx

    def get_intermediate_contour_points(self, safety_distance, start_point, xs, ys):
        """:147-163."""
        side = self.check_side_of_a_point(start_point)
        offset = -safety_distance if side == self.NEAR_SIDE else safety_distance
        return np.vstack((xs[:] + offset, ys[:])).T

    def _sorted_row_ends(self, start_pose, end_pose):
        xs, ys, idx = self.get_row_ids_between_start_and_end(start_pose, end_pose)
        iy, ix = ys[idx], xs[idx]
        order = np.argsort(np.abs(iy - start_pose[1]))
        return ix[order], iy[order]

    def get_topology_waypoints_for_headland_transition(self, start_pose, end_pose, drive_row_offset):
        """:165-197."""
        ix, iy = self._sorted_row_ends(start_pose, end_pose)
        cp = self.get_intermediate_contour_points(drive_row_offset, start_pose[:2], ix, iy)
        return np.vstack((start_pose[:2], cp[1:], end_pose[:2]))

    def get_topology_waypoints(self, start_pose, end_pose, drive_row_offset):
        """:199-248."""
        ix, iy = self._sorted_row_ends(start_pose, end_pose)
        cp = self.get_intermediate_contour_points(drive_row_offset, start_pose[:2], ix, iy)
        return np.vstack((np.asarray(start_pose[:2]), cp, np.asarray(end_pose[:2])))

    def get_which_side_of_pose(self, pose):
        k, b = self._center_line_coeff[0], self._center_line_coeff[1]
        return self.NEAR_SIDE if np.sign(k * pose[0] + b - pose[1]) == self._origin_sign else self.FAR_SIDE

    def create_row_polygons(self, tree_width):
        """:277-286: flat-capped buffer of each row segment."""
        out = []
        for row in self.map_tree_rows:
            if len(row) != 2:
                raise NotImplementedError("[HA*] tree rows must be 2-point segments")
            out.append(buffer_segment_flat(row[0], row[1], tree_width / 2))
        return out

    def get_map_exterior_pts(self, headland_width):
        """:288-334."""
        row_width = np.mean(np.diff(self.map_tree_rows[:, 0, 1]))
        near_angle = self.get_headland_angle(self.NEAR_SIDE)
        far_angle = self.get_headland_angle(self.FAR_SIDE)
        delta_x_near = abs(headland_width / math.sin(near_angle))
        delta_x_far = abs(headland_width / math.sin(far_angle))
        near = np.array([row[0] for row in self.map_tree_rows])
        near[:, 0] -= delta_x_near
        up = np.argmax(near[:, 1])
        near[up, 1] += row_width
        delta_x = 0 if np.abs(np.sin(near_angle)) < 1e-5 else row_width / np.tan(near_angle)
        near[up, 0] += delta_x
        low = np.argmin(near[:, 1])
        near[low, 1] -= row_width
        near[low, 0] -= delta_x
        far = [row[1] for row in self.map_tree_rows]
        far.reverse()
        far = np.array(far)
        far[:, 0] += delta_x_far
        up = np.argmax(far[:, 1])
        delta_x = 0 if np.abs(np.sin(far_angle)) < 1e-5 else row_width / np.tan(far_angle)
        far[up, 1] += row_width
        far[up, 0] += delta_x
        low = np.argmin(far[:, 1])
        far[low, 1] -= row_width
        far[low, 0] -= delta_x
        return np.concatenate((near, far))

    def create_field_polygon(self, headland_width, contour_points):
        if len(contour_points) == 0:
            return Polygon(self.get_map_exterior_pts(headland_width))
        return Polygon(np.asarray(contour_points, dtype=np.float64))

    def create_obstacle_polygons(self, obstacles, obstacle_dim):
        return [buffer_point_square(float(o[0]), float(o[1]), obstacle_dim) for o in obstacles]

    def check_path_feasibility(self, car_model, path, boundary_check=True, aux_check=False):
        """:423-458 (nearest-then-intersects == any intersects)."""
        path = np.asarray(path, dtype=np.float64)
        path = path.reshape(-1, path.shape[-1])[:, :3]
        body, aux = car_model.get_path_poly(path)
        for poly in self.obs_poly_list:
            if convex_intersects(body, ring_of(poly)).any():
                return False
        field = ring_of(self.field_range_poly)
        if boundary_check and not simple_contains(field, body).all():
            return False
        if aux_check:
            for a in aux:
                for poly in self.obs_poly_list:
                    if convex_intersects(a, ring_of(poly)).any():
                        return False
                if boundary_check and not simple_contains(field, a).all():
                    return False
        return True

    def get_headland_angle(self, side):
        """:463-472."""
        side_idx = 0 if side == self.NEAR_SIDE else 1
        xs = self.map_tree_rows[:, side_idx, 0]
        if np.std(xs) < 0.01:
            return np.pi / 2
        k = np.polyfit(xs, self.map_tree_rows[:, side_idx, 1], deg=1)[0]
        return math.atan(k)
