"""CarModel of R/path_planner/car_model.py (shapely-free).

Same constructor, attributes and kinematic helpers; polygons are
`geom.Polygon` rings (`.exterior.xy` / `.exterior.coords` like shapely).
`get_path_poly` returns the per-pose footprint rings instead of their
shapely union -- the union is only ever used through intersects/contains
predicates, which hold for the union iff they hold footprint by footprint
(see geom.py / hybrid_a_star_search.py).
"""
import math

import numpy as np

from .geom import Polygon, angle_wrap, place, ring_of


class CarModel:
    def __init__(self, max_steer=0.55, wheel_base=1.9, axle_to_front=2.85, axle_to_back=0.5, width=1.48,
                 head_out=0.542, head_side=0.44, body_vertices=[], aux_poly_features=[], with_aux=False):
        self.MAX_STEER = max_steer
        self.WHEEL_BASE = wheel_base
        self.aux_polys = []
        self.AXLE_TO_FRONT = axle_to_front
        self.AXLE_TO_BACK = axle_to_back
        self.WIDTH = width
        self.HEAD_OUT = head_out
        self.HEAD_SIDE = head_side
        self.curvature = math.tan(self.MAX_STEER) / self.WHEEL_BASE   # car_model.py:34
        self.with_aux = with_aux
        self.body_vertices = body_vertices
        self.get_car_poly(aux_poly_features)

    def get_car_poly(self, aux_poly_features):
        """car_model.py:75-144."""
        body = np.array([[-self.AXLE_TO_BACK, -self.AXLE_TO_BACK, self.AXLE_TO_FRONT, self.AXLE_TO_FRONT,
                          -self.AXLE_TO_BACK],
                         [self.WIDTH / 2, -self.WIDTH / 2, -self.WIDTH / 2, self.WIDTH / 2, self.WIDTH / 2]])
        self.car_poly = Polygon(body.T)
        if self.with_aux:
            parts = self.get_aux_shapely_polys(aux_poly_features)
            if len(parts) > 0:
                self.aux_polys = parts

    @staticmethod
    def get_aux_shapely_polys(aux_polys):
        """car_model.py:146-162: feature = [[x, y] of the left-top vertex, height, width]."""
        out = []
        for f in aux_polys:
            p1 = [f[0][0], f[0][1]]
            p2 = [f[0][0] + f[2], f[0][1]]
            p3 = [f[0][0] + f[2], f[0][1] - f[1]]
            p4 = [f[0][0], f[0][1] - f[1]]
            out.append(Polygon(np.array([p1, p2, p3, p4], dtype=np.float64)))
        return out

    def get_path_poly(self, path, skip=1):
        """car_model.py:39-73 -> (body rings (P,k,2) at every `skip`-th pose,
        [aux rings at every 2nd pose for each implement])."""
        path = np.asarray(path, dtype=np.float64)
        body = place(ring_of(self.car_poly), path[0:len(path):skip, :3])
        aux = [place(ring_of(a), path[0:len(path):2, :3]) for a in self.aux_polys]
        return body, aux

    def get_car_poly_in_odom(self, odom_x, odom_y, odom_yaw):
        """car_model.py:178-200."""
        pose = np.array([[odom_x, odom_y, odom_yaw]])
        car = Polygon(place(ring_of(self.car_poly), pose)[0])
        return car, [Polygon(place(ring_of(a), pose)[0]) for a in self.aux_polys]

    def calculate_motion_path(self, init_pose, motion_command, delta_yaw, step):
        """car_model.py:202-234."""
        steer_angle, speed_direction = motion_command[0], motion_command[1]
        search_length = delta_yaw / self.curvature
        num_steps = round(search_length / step)
        yaw_step = speed_direction * step / self.WHEEL_BASE * math.tan(steer_angle)
        init_yaw = angle_wrap(init_pose[-1] + yaw_step)
        yaws = np.linspace(init_yaw, init_yaw + yaw_step * (num_steps + 1), num_steps + 1)
        yaws = angle_wrap(yaws)
        xs = init_pose[0] + np.cumsum(step * np.cos(yaws[:-1]) * speed_direction)
        ys = init_pose[1] + np.cumsum(step * np.sin(yaws[:-1]) * speed_direction)
        path = np.vstack([init_pose, np.vstack([xs, ys, yaws[1:]]).T])
        curvature = 0
        if abs(motion_command[0]) > 0.00001:
            curvature = math.tan(motion_command[0]) / self.WHEEL_BASE
        ks = np.ones((len(path), 1)) * curvature
        dirs = np.ones((len(path), 1)) * motion_command[1]
        return np.hstack((path, ks, dirs))

    def calculate_motion_path_new(self, init_pose, motion_dir, steer_dir, turning_radius, delta_yaw, step_size=0.1):
        """car_model.py:236-269: a circular arc of radius max(R_min, turning_radius) sampled in closed form;
        rows [x, y, yaw, k, dir], the init pose repeated as the first row (as the reference does)."""
        turning_radius = max(1.0 / self.curvature, turning_radius)
        steer_angle = math.atan(self.WHEEL_BASE / turning_radius) * steer_dir
        arc_length = abs(delta_yaw * turning_radius)
        num_steps = int(arc_length / step_size)
        actual_step_size = arc_length / num_steps
        yaw_step = motion_dir * actual_step_size / self.WHEEL_BASE * math.tan(steer_angle)
        init_x, init_y = init_pose[0], init_pose[1]
        init_yaw = angle_wrap(init_pose[-1])
        yaws = angle_wrap(np.linspace(init_yaw, init_yaw + yaw_step * num_steps, num_steps + 1))
        xs = init_x + turning_radius * (np.sin(yaws) - np.sin(init_yaw)) * steer_dir
        ys = init_y - turning_radius * (np.cos(yaws) - np.cos(init_yaw)) * steer_dir
        path = np.vstack([init_pose, np.vstack([xs, ys, yaws]).T])
        curvature = 0
        if abs(steer_angle) > 0.00001:
            curvature = math.tan(steer_angle) / self.WHEEL_BASE
        ks = np.ones((len(path), 1)) * curvature
        dirs = np.ones((len(path), 1)) * motion_dir
        return np.hstack((path, ks, dirs))

    def get_turn_radius(self, max_steer_angle=None):
        if max_steer_angle is None:
            return 1 / self.curvature
        return self.WHEEL_BASE / math.tan(max_steer_angle)

    def get_steer_angle(self, curvature):
        return min(math.atan(self.WHEEL_BASE * curvature), self.MAX_STEER)
