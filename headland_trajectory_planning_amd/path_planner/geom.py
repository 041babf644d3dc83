"""Shapely-free polygons for the warm-start planner (host side).

The reference builds its geometry with shapely/GEOS; these helpers produce the
same vertex rings so the lowered problem handed to the HIP search kernel
(libhtp.so htp_hastar_search_batch) is the reference's geometry:

* `buffer_segment_round`  LineString([p0, p1]).buffer(d, cap_style=1) as used for
  the heuristic's segment lanes (R/path_planner/reference_line_heuristic.py:65-67):
  GEOS OffsetCurveBuilder / OffsetSegmentGenerator with quadrant_segs = 16 --
  left offset at p1, 31 fillet points (p1 + d (cos a, sin a), a stepping
  clockwise from the segment angle + pi/2 by pi/32; the first one coincides
  with the offset point and is dropped by the 1e-6 d vertex snap), right offset
  at p1, then the same around p0.
* `buffer_segment_flat`   LineString(row).buffer(w/2, cap_style=2) for tree rows
  (R/path_planner/orchard_geometry_environment.py:277-286).
* `buffer_point_square`   Point(x, y).buffer(d, cap_style="square") for point
  obstacles (:345-353).
* `Polygon`               the duck type the reference reads (`.exterior.xy`,
  `.exterior.coords`), plus host predicates used by the host-side API methods
  (check_path_feasibility, get_search_length); the search itself runs on the GPU.
"""
import math

import numpy as np


class _Ring:
    def __init__(self, v):
        self._v = v

    @property
    def xy(self):
        c = np.vstack([self._v, self._v[:1]])
        return c[:, 0].copy(), c[:, 1].copy()

    @property
    def coords(self):
        return [tuple(p) for p in np.vstack([self._v, self._v[:1]])]


class Polygon:
    """Minimal polygon: vertex ring without the closing vertex."""

    def __init__(self, vertices):
        v = np.asarray(vertices, dtype=np.float64).reshape(-1, 2)
        if v.shape[0] > 1 and np.array_equal(v[0], v[-1]):
            v = v[:-1]
        self.vertices = v
        self.exterior = _Ring(v)

    @property
    def bounds(self):
        """(minx, miny, maxx, maxy), as shapely's."""
        lo, hi = self.vertices.min(axis=0), self.vertices.max(axis=0)
        return (float(lo[0]), float(lo[1]), float(hi[0]), float(hi[1]))

    def __repr__(self):
        return f"Polygon({self.vertices.shape[0]} vertices)"


def ring_of(poly):
    """Vertices (n, 2) of a shapely polygon, a Polygon or an array (closing vertex dropped)."""
    if hasattr(poly, "exterior"):
        xy = np.asarray(poly.exterior.xy, dtype=np.float64).T
    else:
        xy = np.asarray(poly, dtype=np.float64).reshape(-1, 2)
    if xy.shape[0] > 1 and np.array_equal(xy[0], xy[-1]):
        xy = xy[:-1]
    return xy


def _offset(p0, p1, side, d):
    """GEOS computeOffsetSegment: the offset of segment p0->p1 (side +1 left, -1 right)."""
    dx = p1[0] - p0[0]
    dy = p1[1] - p0[1]
    ln = math.sqrt(dx * dx + dy * dy)
    ux = side * d * dx / ln
    uy = side * d * dy / ln
    return (p0[0] - uy, p0[1] + ux), (p1[0] - uy, p1[1] + ux)


def _fillet(p, start, end, d, quad_segs):
    """GEOS addDirectedFillet, clockwise."""
    quantum = math.pi / 2.0 / quad_segs
    total = abs(start - end)
    n = int(total / quantum + 0.5)
    if n < 1:
        return []
    inc = total / n
    return [(p[0] + d * math.cos(start + (-i) * inc), p[1] + d * math.sin(start + (-i) * inc)) for i in range(n)]


def _add(ring, pt, snap):
    if ring and math.hypot(pt[0] - ring[-1][0], pt[1] - ring[-1][1]) < snap:
        return
    ring.append(pt)


def buffer_segment_round(p0, p1, d, quad_segs=16):
    p0 = (float(p0[0]), float(p0[1]))
    p1 = (float(p1[0]), float(p1[1]))
    snap = d * 1e-6
    ring = []
    for a, b in ((p0, p1), (p1, p0)):
        _add(ring, _offset(a, b, 1, d)[1], snap)                         # addLastSegment
        ang = math.atan2(b[1] - a[1], b[0] - a[0])
        _add(ring, _offset(a, b, 1, d)[1], snap)                         # cap: offsetL.p1
        for pt in _fillet(b, ang + math.pi / 2.0, ang - math.pi / 2.0, d, quad_segs):
            _add(ring, pt, snap)
        _add(ring, _offset(a, b, -1, d)[1], snap)                        # cap: offsetR.p1
    if math.hypot(ring[0][0] - ring[-1][0], ring[0][1] - ring[-1][1]) < snap:
        ring.pop()
    return Polygon(np.array(ring))


def buffer_segment_flat(p0, p1, d):
    p0 = (float(p0[0]), float(p0[1]))
    p1 = (float(p1[0]), float(p1[1]))
    L1 = _offset(p0, p1, 1, d)[1]
    R1 = _offset(p0, p1, -1, d)[1]
    R0 = _offset(p1, p0, 1, d)[1]
    L0 = _offset(p1, p0, -1, d)[1]
    return Polygon(np.array([L1, R1, R0, L0]))


def buffer_point_square(x, y, d):
    return Polygon(np.array([[x + d, y + d], [x + d, y - d], [x - d, y - d], [x - d, y + d]], dtype=np.float64))


def angle_wrap(a):
    """R/path_planner/utils/path_utils.py angle_wrap."""
    return (a + math.pi) % (2 * math.pi) - math.pi


# ------------------------------------------------------------ host predicates
def place(poly, poses):
    """car_model.get_path_poly :42-51: the ring at every pose -> (P, k, 2)."""
    poses = np.asarray(poses, dtype=np.float64).reshape(-1, 3)
    c = np.cos(poses[:, 2])[:, None]
    s = np.sin(poses[:, 2])[:, None]
    vx, vy = poly[None, :, 0], poly[None, :, 1]
    return np.stack([c * vx + (-s) * vy + poses[:, 0:1], s * vx + c * vy + poses[:, 1:2]], axis=2)


def convex_intersects(F, Q):
    """Closed convex rings F[p] (P,k,2) vs Q (m,2) touch or overlap (separating axes)."""
    sep = np.zeros(F.shape[0], dtype=bool)
    for E in (np.roll(F, -1, axis=1) - F, np.broadcast_to(np.roll(Q, -1, axis=0) - Q, (F.shape[0],) + Q.shape)):
        n = np.stack([E[..., 1], -E[..., 0]], axis=-1)
        pa = np.einsum("pkd,ped->pke", F, n)
        pb = np.einsum("md,ped->pme", Q, n)
        sep |= ((pa.max(1) < pb.min(1)) | (pb.max(1) < pa.min(1))).any(1)
    return ~sep


def ccw(v):
    a = np.sum(v[:, 0] * np.roll(v[:, 1], -1) - np.roll(v[:, 0], -1) * v[:, 1])
    return v if a > 0 else v[::-1].copy()


def convex_contains_point(C, x, y):
    """Point strictly inside the convex ring C (any orientation)."""
    C = ccw(C)
    a, b = C, np.roll(C, -1, axis=0)
    return bool(np.all((b[:, 0] - a[:, 0]) * (y - a[:, 1]) - (b[:, 1] - a[:, 1]) * (x - a[:, 0]) > 0))


def simple_contains(field, F):
    """Footprints F[p] inside the simple polygon `field`: corners inside, no proper edge crossing."""
    X, Y = F[..., 0], F[..., 1]
    V = field.shape[0]
    inside = np.zeros(X.shape, dtype=bool)
    ok = np.ones(F.shape[0], dtype=bool)
    A, B = F, np.roll(F, -1, axis=1)
    for i in range(V):
        (xi, yi), (xj, yj) = field[i], field[(i + 1) % V]
        with np.errstate(divide="ignore", invalid="ignore"):
            xc = (xj - xi) * (Y - yi) / (yj - yi) + xi
        inside ^= ((yi > Y) != (yj > Y)) & (X < xc)
        o1 = (B[..., 0] - A[..., 0]) * (yi - A[..., 1]) - (B[..., 1] - A[..., 1]) * (xi - A[..., 0])
        o2 = (B[..., 0] - A[..., 0]) * (yj - A[..., 1]) - (B[..., 1] - A[..., 1]) * (xj - A[..., 0])
        o3 = (xj - xi) * (A[..., 1] - yi) - (yj - yi) * (A[..., 0] - xi)
        o4 = (xj - xi) * (B[..., 1] - yi) - (yj - yi) * (B[..., 0] - xi)
        ok &= ~((o1 * o2 < 0) & (o3 * o4 < 0)).any(1)
    return ok & inside.all(1)


def union_contains(lanes, F):
    """Footprints F[p] inside the union of the convex rings `lanes` (edge coverage)."""
    A = F.reshape(-1, 2)
    B = np.roll(F, -1, axis=1).reshape(-1, 2)
    ivs = []
    for C in lanes:
        C = ccw(C)
        lo, hi = np.zeros(A.shape[0]), np.ones(A.shape[0])
        for i in range(C.shape[0]):
            v, w = C[i], C[(i + 1) % C.shape[0]]
            ex, ey = w[0] - v[0], w[1] - v[1]
            c0 = ex * (A[:, 1] - v[1]) - ey * (A[:, 0] - v[0])
            c1 = ex * (B[:, 1] - A[:, 1]) - ey * (B[:, 0] - A[:, 0])
            with np.errstate(divide="ignore", invalid="ignore"):
                t = -c0 / c1
            lo = np.where(c1 > 0, np.maximum(lo, t), lo)
            hi = np.where(c1 < 0, np.minimum(hi, t), hi)
            lo = np.where((c1 == 0) & (c0 < 0), 2.0, lo)
        ivs.append((lo, hi))
    ok = np.zeros(A.shape[0], dtype=bool)
    for e in range(A.shape[0]):
        reach = 0.0
        for lo, hi in sorted((lo[e], hi[e]) for lo, hi in ivs if lo[e] <= hi[e]):
            if lo > reach:
                break
            reach = max(reach, hi)
        ok[e] = reach >= 1.0
    return ok.reshape(F.shape[0], F.shape[1]).all(1)


def point_convex_distance(C, x, y):
    """Euclidean distance from (x, y) to the closed convex ring C (0 inside)."""
    if convex_contains_point(C, x, y):
        return 0.0
    a, b = C, np.roll(C, -1, axis=0)
    e = b - a
    ee = np.maximum(np.einsum("kd,kd->k", e, e), 1e-300)
    t = np.clip(((x - a[:, 0]) * e[:, 0] + (y - a[:, 1]) * e[:, 1]) / ee, 0.0, 1.0)
    px, py = a[:, 0] + t * e[:, 0] - x, a[:, 1] + t * e[:, 1] - y
    return float(np.sqrt(np.min(px * px + py * py)))


def polyline_buffer_intersects(xy, d, Q):
    """LineString(xy).buffer(d, cap_style=2 (flat), join_style=1 (round)) intersects the
    convex ring Q (R/path_planner/safety_forward_path_plan.py:815-818).

    With flat caps and round joins the buffer is the union of one rectangle per
    segment (the segment swept +-d along its normal) and a disc of radius d at
    every interior vertex, so it touches Q iff a rectangle does (separating
    axes) or an interior vertex lies within d of Q.  GEOS draws the join arcs
    as inscribed chords (quadrant_segs 16), so the two predicates can only
    disagree inside a band d (1 - cos(pi/64)) ~ 3.6e-4 d wide."""
    xy = np.asarray(xy, dtype=np.float64)[:, :2]
    keep = np.ones(len(xy), dtype=bool)
    keep[1:] = np.any(xy[1:] != xy[:-1], axis=1)  # GEOS drops repeated points
    xy = xy[keep]
    if len(xy) < 2:
        return point_convex_distance(Q, xy[0, 0], xy[0, 1]) <= d
    p0, p1 = xy[:-1], xy[1:]
    t = p1 - p0
    n = np.stack([-t[:, 1], t[:, 0]], axis=1) / np.linalg.norm(t, axis=1)[:, None] * d
    rects = np.stack([p0 + n, p1 + n, p1 - n, p0 - n], axis=1)
    if convex_intersects(rects, Q).any():
        return True
    return any(point_convex_distance(Q, x, y) <= d for x, y in xy[1:-1])
