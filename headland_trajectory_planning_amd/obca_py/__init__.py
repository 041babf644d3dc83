"""Drop-in replacements for R/obca_py (optimizer, car model, init-guess glue)."""
