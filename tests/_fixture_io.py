"""Problem instances stored inside parity fixtures (tests/golden/*/*.npz).

A fixture made by the oracle holds its own input, so the GPU parity tests do not depend on the
synthetic generator staying unchanged: `inst_*` arrays (init_traj, halfspaces with their edge
counts, the per-problem scalars) round-trip the oracle/nlp.py instance dict."""
import json

import numpy as np

SCALARS = ("dT", "wheelbase", "max_steer", "max_velocity", "max_accel", "max_steer_rate", "min_dist")


def instance_arrays(inst):
    """oracle/nlp.py instance dict -> flat arrays for np.savez (keys prefixed inst_)."""
    out = {
        "inst_traj": np.asarray(inst["init_traj"], dtype=np.float64),
        "inst_obs_edges": np.array([len(b) for b in inst["obs_b"]], dtype=np.int32),
        "inst_obs_A": np.concatenate([np.asarray(a, dtype=np.float64) for a in inst["obs_A"]]),
        "inst_obs_b": np.concatenate([np.asarray(b, dtype=np.float64) for b in inst["obs_b"]]),
        "inst_scalars": json.dumps({k: float(inst[k]) for k in SCALARS if k in inst}),
        "inst_QRW": np.stack([np.asarray(inst[k], dtype=np.float64) for k in ("Q", "R", "W")]) if "Q" in inst
        else np.zeros((0, 2, 2)),
        "inst_bounds": np.array([*inst.get("x_bound", [-np.inf, np.inf]), *inst.get("y_bound", [-np.inf, np.inf])],
                                dtype=np.float64),
    }
    if "body_G" in inst:
        out["inst_body_edges"] = np.array([len(g) for g in inst["body_g"]], dtype=np.int32)
        out["inst_body_G"] = np.concatenate([np.asarray(a, dtype=np.float64) for a in inst["body_G"]])
        out["inst_body_g"] = np.concatenate([np.asarray(g, dtype=np.float64) for g in inst["body_g"]])
    if "vertices" in inst:
        out["inst_vertices"] = np.asarray(inst["vertices"], dtype=np.float64)
    return out


def _split(flat, edges):
    off = np.concatenate([[0], np.cumsum(edges)])
    return [flat[off[k]:off[k + 1]].copy() for k in range(len(edges))]


def has_instance(z):
    return "inst_traj" in z.files


def load_instance(z):
    """npz (np.load result) with inst_* arrays -> oracle/nlp.py instance dict."""
    inst = dict(init_traj=z["inst_traj"].copy(), obs_A=_split(z["inst_obs_A"], z["inst_obs_edges"]),
                obs_b=_split(z["inst_obs_b"], z["inst_obs_edges"]))
    inst.update(json.loads(str(z["inst_scalars"])))
    if z["inst_QRW"].shape[0] == 3:
        inst["Q"], inst["R"], inst["W"] = (z["inst_QRW"][k].copy() for k in range(3))
    b = z["inst_bounds"]
    inst["x_bound"], inst["y_bound"] = [b[0], b[1]], [b[2], b[3]]
    if "inst_body_G" in z.files:
        inst["body_G"] = _split(z["inst_body_G"], z["inst_body_edges"])
        inst["body_g"] = _split(z["inst_body_g"], z["inst_body_edges"])
    if "inst_vertices" in z.files:
        inst["vertices"] = z["inst_vertices"].copy()
    return inst
