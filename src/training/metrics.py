"""src.training.metrics (reference src/training/metrics.py) -> ncf_amd.metrics."""
from ncf_amd.metrics import metrics  # noqa: F401
