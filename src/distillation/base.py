"""src.distillation.base (reference) -> ncf_amd.distill."""
from ncf_amd.distill import BaseDistillation  # noqa: F401
