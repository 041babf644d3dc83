"""Oracle: vertex list -> H-representation, as the reference obtains it.

Restates `pypoman.compute_polytope_halfspaces` (pypoman >= 0.5.4,
R/requirements.txt:3) on top of cddlib's double-description output, as
called at R/obca_py/optimizer.py:182-186 (bodies) and :197-200 (obstacles):

    V = round(vertices, 7)
    [b | -A] = cdd facets of conv(V); each row normalised by cddlib's
               dd_Normalize: divide by the smallest |entry| > 1e-7
    A, b     = round(A, 7), round(b, 7)

cddlib's facet *order* is an artefact of its insertion order and cannot be
reproduced without cddlib (absent here).  We emit facets in counter-clockwise
hull order starting at the lexicographically smallest vertex.  A permutation of
rows only permutes the matching dual variables inside one (obstacle, body)
block; the feasible (x, u) set is invariant.  Documented as an assumption in
DESIGN.md ("parity unpinned" for dual-variable order).
"""
import numpy as np

CDD_ALMOST_ZERO = 1e-7


def convex_hull_ccw(points):
    """Monotone-chain convex hull; CCW, starting at the lexicographic minimum,
    collinear points dropped (cdd reports only facets)."""
    pts = sorted(set(map(tuple, np.asarray(points, dtype=np.float64))))
    if len(pts) < 3:
        raise ValueError("[OBCA] polygon needs >= 3 distinct vertices")

    def cross(o, a, b):
        return (a[0] - o[0]) * (b[1] - o[1]) - (a[1] - o[1]) * (b[0] - o[0])

    lower, upper = [], []
    for p in pts:
        while len(lower) >= 2 and cross(lower[-2], lower[-1], p) <= 0:
            lower.pop()
        lower.append(p)
    for p in reversed(pts):
        while len(upper) >= 2 and cross(upper[-2], upper[-1], p) <= 0:
            upper.pop()
        upper.append(p)
    return np.array(lower[:-1] + upper[:-1], dtype=np.float64)


def _cdd_normalize(row):
    mags = np.abs(row)
    nz = mags[mags > CDD_ALMOST_ZERO]
    if nz.size == 0:
        return row
    return row / nz.min()


def compute_polytope_halfspaces(vertices):
    """Return (A, b) with A x <= b describing conv(vertices) (pypoman API)."""
    hull = convex_hull_ccw(vertices)
    n = len(hull)
    A = np.zeros((n, 2))
    b = np.zeros(n)
    for k in range(n):
        p, q = hull[k], hull[(k + 1) % n]
        # CCW polygon: interior on the left of p->q, outward normal = (dy, -dx)
        a = np.array([q[1] - p[1], -(q[0] - p[0])])
        bb = a @ p
        row = _cdd_normalize(np.array([bb, -a[0], -a[1]]))
        b[k] = row[0]
        A[k] = -row[1:]
    return A, b


def obca_halfspaces(vertices):
    """optimizer.py:184-186 / :198-200: round the vertices, extract, round."""
    v = np.round(np.asarray(vertices, dtype=np.float64), 7)
    A, b = compute_polytope_halfspaces(v)
    return np.round(A, 7), np.round(b, 7)
