"""Re-export (gpbasics/DataHandling/AbstractDataInput.py)."""
from .DataInput import AbstractDataInput  # noqa: F401
