"""Re-export (gpbasics/DataHandling/BatchDataInput.py)."""
from .DataInput import BatchDataInput  # noqa: F401
