"""Vehicle geometry for OBCA (R/obca_py/car_model_obca.py, R/path_planner/car_model.py).

shapely is not a dependency: polygons are `Polygon2D` objects exposing the
`.exterior.xy` / `.exterior.coords` surface the optimizer reads
(R/obca_py/optimizer.py:174-183), closing vertex included like shapely.
"""
import math

import numpy as np


class _Ring:
    def __init__(self, pts):
        closed = np.vstack([pts, pts[:1]])
        self.xy = (closed[:, 0].copy(), closed[:, 1].copy())
        self.coords = [tuple(p) for p in closed]


class Polygon2D:
    def __init__(self, pts):
        pts = np.asarray(pts, dtype=np.float64)
        if pts.shape[0] > 1 and np.all(pts[0] == pts[-1]):
            pts = pts[:-1]
        self.exterior = _Ring(pts)


def angle_wrap(angle):
    return (angle + math.pi) % (2 * math.pi) - math.pi


class CarModel:
    """car_model.py:10-37 / car_model_obca.py:14-41 constructor surface."""

    def __init__(self, max_steer=0.55, wheel_base=1.9, axle_to_front=2.85, axle_to_back=0.5, width=1.48,
                 head_out=0.542, head_side=0.44, body_vertices=[], aux_poly_features=[], with_aux=False):
        self.MAX_STEER = max_steer
        self.WHEEL_BASE = wheel_base
        self.AXLE_TO_FRONT = axle_to_front
        self.AXLE_TO_BACK = axle_to_back
        self.WIDTH = width
        self.HEAD_OUT = head_out
        self.HEAD_SIDE = head_side
        self.curvature = math.tan(self.MAX_STEER) / self.WHEEL_BASE
        self.with_aux = with_aux
        self.body_vertices = body_vertices
        self.aux_polys = []
        body = np.array([[-axle_to_back, width / 2], [-axle_to_back, -width / 2],
                         [axle_to_front, -width / 2], [axle_to_front, width / 2]])
        self.car_poly = Polygon2D(body)
        if with_aux:
            self.aux_polys = [Polygon2D(p) for p in self.get_aux_polys(aux_poly_features)]

    @staticmethod
    def get_aux_polys(features):
        """car_model.py:146-162: [[x, y] of left-top vertex, height, width]."""
        out = []
        for f in features:
            (x, y), h, w = f[0], f[1], f[2]
            out.append(np.array([[x, y], [x + w, y], [x + w, y - h], [x, y - h]], dtype=np.float64))
        return out

    def get_turn_radius(self, max_steer_angle=None):
        if max_steer_angle is None:
            return 1 / self.curvature
        return self.WHEEL_BASE / math.tan(max_steer_angle)
