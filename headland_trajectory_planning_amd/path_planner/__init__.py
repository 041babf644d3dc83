"""Drop-in replacements for the reference's path_planner modules
(R/path_planner/*.py): hybrid A* warm start searched on the GPU, with the
environment / heuristic / car model restated without shapely."""
