"""Host-side polygon utilities for the OBCA boundary.

* `polytope_halfspaces` replaces pypoman/cddlib's
  `compute_polytope_halfspaces` as used at R/obca_py/optimizer.py:184-186 and
  :198-200 (vertices rounded to 7 decimals, cdd row normalisation "smallest
  |entry| > 1e-7 becomes 1", result rounded to 7 decimals).  Facets are
  emitted in counter-clockwise hull order from the lexicographically smallest
  vertex (cddlib's own order is not reproducible without cddlib).
* `body_polygons` returns the vehicle body + implement rectangles exactly as
  R/path_planner/car_model.py builds them (body :102-120, implements :146-162).
"""
import numpy as np

_CDD_EPS = 1e-7


def _hull(pts):
    P = np.unique(np.asarray(pts, dtype=np.float64), axis=0)  # lexicographic sort
    if P.shape[0] < 3:
        raise ValueError("[OBCA] polygon needs >= 3 distinct vertices")
    out = []
    for seq in (P, P[::-1]):
        chain = []
        for p in seq:
            while len(chain) >= 2:
                o, a = chain[-2], chain[-1]
                if (a[0] - o[0]) * (p[1] - o[1]) - (a[1] - o[1]) * (p[0] - o[0]) > 0:
                    break
                chain.pop()
            chain.append(p)
        out.extend(chain[:-1])
    return np.array(out)


def polytope_halfspaces(vertices):
    """(A, b) with A x <= b for conv(vertices), cdd-normalised and rounded."""
    V = np.round(np.asarray(vertices, dtype=np.float64), 7)
    H = _hull(V)
    Q = np.roll(H, -1, axis=0)
    nrm = np.stack([Q[:, 1] - H[:, 1], H[:, 0] - Q[:, 0]], axis=1)  # outward (CCW)
    rows = np.concatenate([np.sum(nrm * H, axis=1)[:, None], -nrm], axis=1)  # [b | -A]
    mag = np.abs(rows)
    scale = np.where(mag > _CDD_EPS, mag, np.inf).min(axis=1)
    scale = np.where(np.isfinite(scale), scale, 1.0)
    rows = rows / scale[:, None]
    return np.round(-rows[:, 1:], 7), np.round(rows[:, 0], 7)


def body_rectangle(axle_to_front, axle_to_back, width):
    """car_model.py:106-123 (closing vertex dropped as optimizer.py:175)."""
    return np.array([[-axle_to_back, width / 2], [-axle_to_back, -width / 2],
                     [axle_to_front, -width / 2], [axle_to_front, width / 2]])


def implement_rectangle(feature):
    """car_model.py:146-162: feature = [[x, y] of left-top vertex, height, width]."""
    (x, y), hgt, wid = feature[0], feature[1], feature[2]
    return np.array([[x, y], [x + wid, y], [x + wid, y - hgt], [x, y - hgt]], dtype=np.float64)


def polygon_exterior_vertices(poly):
    """Vertices of a shapely-like polygon (`.exterior.xy`) or an (n,2) array,
    without the repeated closing vertex (optimizer.py:174-176)."""
    if hasattr(poly, "exterior"):
        xy = np.array(poly.exterior.xy, dtype=np.float64).T
        return xy[:-1]
    a = np.asarray(poly, dtype=np.float64)
    if a.shape[0] > 1 and np.all(a[0] == a[-1]):
        a = a[:-1]
    return a


def convex_hull_ring(points):
    """Vertices of conv(points) as shapely's `MultiPoint(points).convex_hull.exterior.coords[:-1]`
    (GEOS ConvexHull: Graham scan from the lowest point -- minimum y, then minimum x -- clockwise,
    collinear points dropped).  Used by optimizer_points.get_vehicle_vertices (:35-50)."""
    H = _hull(points)                 # counter-clockwise, collinear points removed
    start = min(range(len(H)), key=lambda k: (H[k][1], H[k][0]))
    ccw = np.roll(H, -start, axis=0)
    return np.vstack([ccw[:1], ccw[:0:-1]])  # same start, clockwise


def vehicle_hull_vertices(polys):
    """get_vehicle_vertices(car, convex_hull=True) (optimizer_points.py:35-50): the rear-axle
    origin plus every body / implement polygon vertex, convex hull."""
    pts = [np.zeros((1, 2))] + [polygon_exterior_vertices(p) for p in polys]
    return convex_hull_ring(np.vstack(pts))
