"""The notebook chain's heuristic lowering (csrc/ychain_core.h, the device code between the Y-park and the
hybrid A* searches of htp_ypark_hastar_chain_device) through its host build, against the restated reference
planner: get_topology_waypoints + ReferenceLineHeuristic + the search packer (path_planner/, _native.HastarPacked)
on randomised notebook scenes, at intermediate poses from the host build of the Y-park search.  Waypoints, lane
vertex counts, search lengths and guide row counts equal; coordinates within 1e-12 (the core's correctly rounded
libm against the platform's)."""
import numpy as np
import pytest

from headland_trajectory_planning_amd import _native, ychain
from headland_trajectory_planning_amd.path_planner import hybrid_a_star_search as has
from headland_trajectory_planning_amd.path_planner.reference_line_heuristic import ReferenceLineHeuristic
from headland_trajectory_planning_amd import synth

import _hostsim as H


@pytest.mark.parametrize("pid", range(10))
def test_lowering_core_equals_the_restated_planner(pid):
    scene = ychain.make_scene(pid)
    empty, _ = ychain.notebook_cars()
    yp, _ = ychain.lowered(scene)
    y = H.ypark_dicts(H.ypark_host([yp]))[0]
    if y["status"] != 0:
        pytest.skip(f"Y-park finds no manoeuvre for scene {pid}")
    inter = np.asarray(y["path"])[0][:3]
    with synth._legacy_random(scene["eps_seed"]):
        wps = scene["env"].get_topology_waypoints(scene["start"], inter, drive_row_offset=ychain.DRIVE_ROW_OFFSET)
    heur = ReferenceLineHeuristic(wps, inter, empty)
    prob = has.lower_problem(scene["start"], inter, scene["env"], empty, heur, motion_type="King",
                             plan_resolution=ychain.YP_ARGS["step_size"], max_nodes=ychain.MAX_NODES)
    got = ychain.cpu_lower(scene, inter)
    assert got["status"] == 0, got
    assert np.array_equal(got["waypoints"], np.asarray(wps)), (got["waypoints"], wps)
    ref_lanes = [_native._ccw(_native._clean_ring(q)) for q in prob["lanes"]]
    assert len(got["lanes"]) == len(ref_lanes)
    for a, b in zip(got["lanes"], ref_lanes):
        assert a.shape == b.shape and np.max(np.abs(a - b)) <= 1e-12
    assert np.array_equal(got["lengths"], np.asarray(prob["search_lengths"]))
    g = np.asarray(prob["guide"])[:, :4]
    assert got["guide"].shape == g.shape and np.max(np.abs(got["guide"] - g)) <= 1e-12
