"""R/path_planner/utils drop-in package (`import utils.reeds_shepp`, `from utils.cubic_spline import ...`)."""
