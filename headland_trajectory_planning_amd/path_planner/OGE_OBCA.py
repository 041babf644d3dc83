"""orchard_environment_OBCA of R/path_planner/OGE_OBCA.py: the convex
obstacle set the OBCA optimizer receives (create_boundary_polygons :306-373,
cover_side_points :171-262, get_obstacle_tree_rows :477-591,
get_obstacles_for_OBCA :593-677), shapely-free.  `rdp` (Ramer-Douglas-Peucker,
third-party `rdp` package, unpinned) is restated below."""
import math

import numpy as np

from .orchard_geometry_environment import OrchardGeometryEnvironment


def shortest_distance(x1, y1, a, b, c):
    return np.abs((a * x1 + b * y1 + c)) / (math.sqrt(a * a + b * b))


def point_along_centerline(A, B, d):
    M = (A + B) / 2.0
    L = np.linalg.norm(B - A)
    N = np.array([(B[1] - A[1]) / L, -(B[0] - A[0]) / L])
    return M + N * d


def point_side_of_line(A, B, C):
    return np.sign((B[0] - A[0]) * (C[1] - A[1]) - (B[1] - A[1]) * (C[0] - A[0]))


def points_along_rectangles(A, B, d):
    extra = point_along_centerline(A, B, d)
    return extra + (A - B) / 2, extra - (A - B) / 2


def _pldist(point, start, end):
    """rdp.pldist: distance of `point` to the line through start, end."""
    if np.all(np.equal(start, end)):
        return np.linalg.norm(point - start)
    e, s = end - start, start - point
    return np.divide(np.abs(np.linalg.norm(e[0] * s[1] - e[1] * s[0])), np.linalg.norm(end - start))


def rdp(M, epsilon=0):
    """rdp.rdp_rec: keep the farthest point (first on ties) while it is > epsilon off the chord."""
    M = np.asarray(M, dtype=np.float64)
    dmax, index = 0.0, -1
    for i in range(1, M.shape[0]):
        d = _pldist(M[i], M[0], M[-1])
        if d > dmax:
            index, dmax = i, d
    if dmax > epsilon:
        r1 = rdp(M[:index + 1], epsilon)
        r2 = rdp(M[index:], epsilon)
        return np.vstack((r1[:-1], r2))
    return np.vstack((M[0], M[-1]))


class orchard_environment_OBCA(OrchardGeometryEnvironment):
    MIN_ROW_WIDTH = 0.5
    SAFETY_BOUND = 0.2

    def __init__(self, map_tree_rows, obstacles, contour_points=[], tree_width=0.5, headland_width=7,
                 obstacle_dim=0.3):
        super().__init__(map_tree_rows, obstacles, contour_points=contour_points, tree_width=tree_width,
                         headland_width=headland_width, obstacle_dim=obstacle_dim)
        self.row_width = np.abs(np.mean(np.diff(self.map_tree_rows[:, 0, 1])))

    def cover_side_points(self, contour_points, side, width=2):
        """:171-262."""
        std_x = np.std(contour_points[:, 0])
        shift = -width if side == self.NEAR_SIDE else width
        if std_x < 1e-3 or len(contour_points) == 2:
            up, down = np.argmax(contour_points[:, 1]), np.argmin(contour_points[:, 1])
            eu, ed = np.copy(contour_points[up]), np.copy(contour_points[down])
            eu[0] += shift
            ed[0] += shift
            return [np.array([eu, contour_points[up], contour_points[down], ed])]
        k, b = np.polyfit(contour_points[:, 1], contour_points[:, 0], deg=1)
        if side == self.NEAR_SIDE:
            cond = contour_points[:, 0] - k * contour_points[:, 1] - b >= 0
        else:
            cond = contour_points[:, 0] - k * contour_points[:, 1] - b <= 0
        idxs = np.where(cond)[0]
        side_points = contour_points[idxs]
        dists = shortest_distance(side_points[:, 0], side_points[:, 1], 1, -k, -b)
        if dists.mean() < 0.1:
            far = contour_points[idxs[np.argmax(dists)], :]
            b_max = far[0] - k * far[1]
            max_y, min_y = np.max(contour_points[:, 1]), np.min(contour_points[:, 1])
            ux, dx = max_y * k + b_max, min_y * k + b_max
            return [np.array([[ux + shift, max_y], [ux, max_y], [dx, min_y], [dx + shift, min_y]])]
        out = []
        dist_signed = -width if side == self.NEAR_SIDE else width
        dist_signed *= np.sign(contour_points[1][1] - contour_points[0][1])
        for i in range(len(contour_points) - 1):
            p1, p2 = points_along_rectangles(contour_points[i, :], contour_points[i + 1, :], dist_signed)
            out.append(np.array([contour_points[i, :], contour_points[i + 1, :], p1, p2]))
        return out

    def create_boundary_polygons(self):
        """:306-373 -> (near quads, far quads, [low quad], [up quad])."""
        near, far = self.create_headland_countour_lines(self.field_range_poly)
        obstacle_near = self.cover_side_points(rdp(near, 0.15), self.NEAR_SIDE)
        obstacle_far = self.cover_side_points(rdp(far, 0.15), self.FAR_SIDE)
        ui = np.argmax(self.map_tree_rows[:, 0, 1])
        un, uf = np.copy(self.map_tree_rows[ui, 0, :]), np.copy(self.map_tree_rows[ui, 1, :])
        un[1] += self.row_width
        uf[1] += self.row_width
        un[0] -= 8
        uf[0] += 8
        uen, uef = np.copy(un), np.copy(uf)
        uen[1] += 1
        uef[1] += 1
        obstacle_up = np.vstack([un, uen, uef, uf])
        li = np.argmin(self.map_tree_rows[:, 0, 1])
        ln, lf = np.copy(self.map_tree_rows[li, 0, :]), np.copy(self.map_tree_rows[li, 1, :])
        ln[1] -= self.row_width
        lf[1] -= self.row_width
        ln[0] -= 8
        lf[0] += 8
        len_, lef = np.copy(ln), np.copy(lf)
        len_[1] -= 1
        lef[1] -= 1
        obstacle_low = np.vstack([ln, len_, lef, lf])
        return obstacle_near, obstacle_far, [obstacle_low], [obstacle_up]

    def _row_rect(self, row, rnd):
        n, f = np.copy(row[0]), np.copy(row[1])
        v1, v2, v3, v4 = np.copy(n), np.copy(n), np.copy(f), np.copy(f)
        v1[0] -= self.SAFETY_BOUND
        v1[1] -= self.tree_width / 2.0
        v2[0] -= self.SAFETY_BOUND
        v2[1] += self.tree_width / 2.0
        v3[0] += self.SAFETY_BOUND
        v3[1] += self.tree_width / 2.0
        v4[0] += self.SAFETY_BOUND
        v4[1] -= self.tree_width / 2.0
        r = np.vstack([v1, v2, v3, v4])
        return np.round(r, 7) if rnd else r

    def get_obstacle_tree_rows(self, start_pose, end_pose):
        """:477-591."""
        hi, lo = max(start_pose[1], end_pose[1]), min(start_pose[1], end_pose[1])
        idxs = np.sort(np.where((self.map_tree_rows[:, 0, 1] > lo) & (self.map_tree_rows[:, 0, 1] < hi))[0])
        low_idx, up_idx = idxs[0], idxs[-1]
        if low_idx == up_idx:
            a, b = max(up_idx - 2, 0), min(up_idx + 2, len(self.map_tree_rows) - 1)
            return [self._row_rect(self.map_tree_rows[i], True) for i in range(a, b)]
        a, b = max(low_idx - 2, 0), min(up_idx + 3, len(self.map_tree_rows) - 1)
        return [self._row_rect(row, False) for row in self.map_tree_rows[list(range(a, b))]]

    def get_obstacles_for_OBCA(self, boundary_polys, row_polys, start_pose, end_pose, side, width=2,
                               buffer_distance=1):
        """:593-677."""
        obstacles = []
        index = 0 if side == self.NEAR_SIDE else 1
        if len(boundary_polys[index]) <= 1:
            obstacles.append(*boundary_polys[index])
        else:
            rect = []
            ymax, ymin = max(start_pose[1], end_pose[1]), min(start_pose[1], end_pose[1])
            for poly in boundary_polys[index]:
                pmin, pmax = np.min(poly[:2, 1]), np.max(poly[:2, 1])
                if pmax > ymin - buffer_distance and pmin < ymax + buffer_distance:
                    rect += [poly]
            cp = np.array([o[0, :] for o in rect])
            cp = np.vstack([cp, rect[-1][1, :]])
            dist_signed = -width if side == self.NEAR_SIDE else width
            direction_signed = 1 if side == self.NEAR_SIDE else -1
            y_dir = np.sign(cp[1][1] - cp[0][1])
            dist_signed *= y_dir
            direction_signed *= y_dir
            s, e = 0, 1
            cur = np.array([cp[s], cp[e]])
            while e < len(cp) - 1:
                if point_side_of_line(cp[e - 1], cp[e], cp[e + 1]) == direction_signed:
                    cur = np.vstack([cur, cp[e + 1]])
                    e += 1
                else:
                    p1, p2 = points_along_rectangles(cur[0], cur[-1], dist_signed)
                    obstacles.append(np.vstack([cur, p1, p2]))
                    s, e = e, e + 1
                    cur = np.array([cp[s], cp[e]])
            p1, p2 = points_along_rectangles(cur[0], cur[-1], dist_signed)
            obstacles.append(np.vstack([cur, p1, p2]))
        if start_pose[1] > end_pose[1]:
            obstacles += [p for p in boundary_polys[2]]
        else:
            obstacles += [p for p in boundary_polys[3]]
        return obstacles + row_polys
