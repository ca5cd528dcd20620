"""Re-export (gpbasics/DataHandling/BatchDataInput.py); its module-level is_equidistant is the batched form."""
from .DataInput import BatchDataInput  # noqa: F401
from .DataInput import is_equidistant_batch as is_equidistant  # noqa: F401
