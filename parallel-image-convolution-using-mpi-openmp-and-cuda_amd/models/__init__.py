"""Filter zoo ("model family") and multi-stage convolution pipelines."""
from .filters import Filter, get_filter, list_filters, register_filter  # noqa: F401
