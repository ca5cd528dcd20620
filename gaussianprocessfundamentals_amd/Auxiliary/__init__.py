"""gpbasics-compatible module group (see package docstring)."""
