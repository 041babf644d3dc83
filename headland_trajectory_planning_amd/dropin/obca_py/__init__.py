"""R/obca_py drop-in directory (flat-import aliases)."""
