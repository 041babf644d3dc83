"""R/path_planner drop-in directory (flat-import aliases)."""
