"""H3 glue: calc_spline_course / get_init_ref_path restated in
headland_trajectory_planning_amd/obca_py/util.py against golden vectors
generated from R/path_planner/utils/cubic_spline.py (tests/golden/make_golden.py)."""
import os

import numpy as np

from headland_trajectory_planning_amd.obca_py import util
from headland_trajectory_planning_amd.obca_py.car_model_obca import CarModel

G = os.path.join(os.path.dirname(__file__), "golden")


def test_spline_course_matches_reference_golden():
    z = np.load(os.path.join(G, "spline_course.npz"))
    io, oo = z["in_offsets"], z["out_offsets"]
    for k in range(len(z["ds"])):
        xs, ys = z["x"][io[k]:io[k + 1]], z["y"][io[k]:io[k + 1]]
        ref = z["out"][oo[k]:oo[k + 1]]
        rx, ry, ryaw, rk, s = util.calc_spline_course(xs, ys, ds=float(z["ds"][k]))
        got = np.stack([rx, ry, ryaw, rk, s], axis=1)
        assert got.shape == ref.shape
        assert np.allclose(got, ref, rtol=0, atol=1e-12), k


def test_init_ref_path_shapes_and_gear_split():
    car = CarModel(with_aux=False)
    # forward arc then reverse straight (one gear change)
    t = np.linspace(0, 1.2, 13)
    xs = np.concatenate([3 * np.sin(t), 3 * np.sin(1.2) - np.linspace(0.2, 2, 10)])
    ys = np.concatenate([3 - 3 * np.cos(t), np.full(10, 3 - 3 * np.cos(1.2))])
    yaws = np.concatenate([t, np.full(10, 1.2)])
    ks = np.concatenate([np.full(13, 1 / 3), np.zeros(10)])
    dirs = np.concatenate([np.ones(13), -np.ones(10)])
    ref = util.get_init_ref_path(car, xs, ys, yaws, ks, dirs, desired_v=0.5, ds=0.2)
    assert ref.shape[1] == 5
    assert ref[0, 2] == 0 and ref[-1, 2] == 0
    assert np.all(np.abs(np.diff(ref[:, 3])) < np.pi)  # unwrapped heading
    assert np.any(ref[:, 2] < 0) and np.any(ref[:, 2] > 0)
