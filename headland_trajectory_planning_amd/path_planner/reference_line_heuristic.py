"""ReferenceLineHeuristic of R/path_planner/reference_line_heuristic.py (shapely-free).

Same constructor and attributes (guided_path, way_points, segment_lanes,
search_lengths, default_search_length).  `segment_lanes` are the GEOS
round-cap buffers of each waypoint segment (geom.buffer_segment_round);
`guided_lane` (their union) is represented by the list itself.  The hybrid A*
kernel consumes these through path_planner.hybrid_a_star_search.lower_problem;
the host methods below answer the same queries for host-side callers.
"""
import math

import numpy as np

from .geom import (angle_wrap, buffer_segment_round, convex_contains_point, convex_intersects, ring_of,
                   union_contains)


class ReferenceLineHeuristic(object):
    ACCEPT_PATH_DEVIATION = 2
    DRIVE_ROW_OFFSET = 5.0
    LARGE_SEARCH_LENGTH = 1.0
    LANE_HALF_WIDTH = 6

    def __init__(self, waypoints, goal_pose, car_model, obstacle_polys=[], default_search_length=1.5):
        self.default_search_length = default_search_length
        self.goal_pose = goal_pose
        self.car_model = car_model
        self.guided_path, self.guided_lane, self.way_points, self.segment_lanes = self.get_guide_line(
            np.asarray(waypoints, dtype=np.float64))
        self.search_lengths = self.create_segment_lengths(self.segment_lanes, obstacle_polys)

    def get_guide_line(self, waypoints):
        """reference_line_heuristic.py:50-82."""
        segment_lanes = []
        step = 0.1
        way_xs, way_ys, way_yaws = np.array([]), np.array([]), np.array([])
        for i in range(1, len(waypoints)):
            x_end, x_start = waypoints[i, 0], waypoints[i - 1, 0]
            y_end, y_start = waypoints[i, 1], waypoints[i - 1, 1]
            dist = np.hypot(x_end - x_start, y_end - y_start)
            num = int(dist / step)
            xs = np.linspace(x_start, x_end, num)
            ys = np.linspace(y_start, y_end, num)
            way_xs = np.append(way_xs, xs)
            way_ys = np.append(way_ys, ys)
            segment_lanes.append(buffer_segment_round(waypoints[i - 1], waypoints[i], self.LANE_HALF_WIDTH))
            yaw = math.atan2(y_end - y_start, x_end - x_start)
            way_yaws = np.append(way_yaws, np.ones_like(xs) * yaw)
        delta_ss = np.hypot(np.diff(way_xs), np.diff(way_ys))
        way_ss = np.zeros_like(way_xs)
        way_ss[1:] = np.cumsum(delta_ss)
        guided_path = np.array([way_xs, way_ys, way_yaws, way_ss]).T
        return guided_path, segment_lanes, waypoints, segment_lanes

    def create_segment_lengths(self, segment_lanes, obs_polys):
        """reference_line_heuristic.py:84-96 (nearest-then-intersects == any intersects)."""
        search_lengths = np.ones(len(segment_lanes)) * self.default_search_length
        if len(search_lengths) > 4:
            if len(obs_polys) == 0:
                search_lengths[2:len(search_lengths) - 1] = self.LARGE_SEARCH_LENGTH
            else:
                for i in range(2, len(search_lengths) - 1):
                    lane = ring_of(segment_lanes[i])[None]
                    if not any(convex_intersects(lane, ring_of(o))[0] for o in obs_polys):
                        search_lengths[i] = self.LARGE_SEARCH_LENGTH
        return search_lengths

    def check_path_feasibility(self, car_model, path):
        """reference_line_heuristic.py:105-118: guided_lane contains the footprint union."""
        path = np.asarray(path, dtype=np.float64)
        body, _ = car_model.get_path_poly(path.reshape(-1, path.shape[-1])[:, :3])
        return bool(union_contains([ring_of(s) for s in self.segment_lanes], body).all())

    def get_search_length(self, pose):
        """reference_line_heuristic.py:120-129 (the last containing segment wins)."""
        out = self.default_search_length
        for i, seg in enumerate(self.segment_lanes):
            if convex_contains_point(ring_of(seg), pose[0], pose[1]):
                out = self.search_lengths[i]
        return out

    def calculate_state_cost(self, pose):
        """reference_line_heuristic.py:131-158."""
        dists = np.hypot(self.guided_path[:, 0] - pose[0], self.guided_path[:, 1] - pose[1])
        m = np.argmin(dists)
        distance_to_path = dists[m] * 100
        yaw_difference = abs(angle_wrap(self.guided_path[m][2] - pose[2]))
        if distance_to_path > self.ACCEPT_PATH_DEVIATION:
            distance_to_path = 100
        dist_to_goal = self.guided_path[-1, -1] - self.guided_path[m, -1]
        return distance_to_path + yaw_difference * 0.2 + dist_to_goal * 5
